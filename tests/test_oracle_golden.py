"""Pin the oracle (oracle/) and the host-side restatements to the golden
fixtures generated from the reference's own functions (tests/golden/make_golden.py)."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import oracle
from oracle import embed_ref

GOLD = os.path.join(os.path.dirname(__file__), "golden")
sys.path.insert(0, GOLD)
import inputs as I  # noqa: E402


def load(name):
    return np.load(os.path.join(GOLD, name + ".npz"))


def near_tie_mask(sorted_scores, eps=2e-6):
    """True at rank r if the score there is within eps of rank r-1 or r+1."""
    s = sorted_scores
    d = np.abs(np.diff(s, axis=1)) < eps
    m = np.zeros_like(s, dtype=bool)
    m[:, 1:] |= d
    m[:, :-1] |= d
    return m


@pytest.mark.parametrize("tag", ["rank_a", "rank_b"])
def test_oracle_ranker_vs_reference(tag):
    fx = load(tag)
    q, g = I.rank_inputs(int(fx["seed"]), int(fx["nq"]), int(fx["n"]), int(fx["d"]))
    s, i = oracle.cosine_topk(q, g, 100)
    # cosine scores within 1e-5 of the reference's torch.mm (north_star bar)
    assert np.abs(s - fx["top_scores"]).max() < 1e-5
    # indices identical except at near-ties (|score gap| < 2e-6)
    ties = near_tie_mask(fx["top_scores"])
    mism = (i != fx["top_idx_stable"])
    assert not (mism & ~ties).any(), np.argwhere(mism & ~ties)[:5]
    # the planted exact duplicates make stable vs default-kind argsort matter
    assert (fx["top_idx_default"].shape == i.shape)


def test_oracle_gem_pooling_bitexact():
    fx = load("gem")
    x = torch.from_numpy(fx["x"])
    assert np.array_equal(embed_ref.gem(x).numpy(), fx["gem"])
    pt = torch.ones(1) * 3.0
    gp = F.avg_pool2d(x.clamp(min=1e-6).pow(pt), (7, 7)).pow(1.0 / pt)
    assert np.array_equal(gp.numpy(), fx["gempool"])
    # the two reference variants differ by at most a few ulp
    assert np.abs(fx["gem"] - fx["gempool"]).max() < 1e-6


def test_oracle_extractor_tails():
    fx = load("gem_tail")
    from research_image_retrieval_amd.weights import synthetic_linear
    x2 = torch.from_numpy(I.feature_map(int(fx["x2_seed"]), 2, 2048, 7, 7))
    ww, wb = synthetic_linear(2048, 2048, int(fx["whiten_seed"]))
    f = embed_ref.gem(x2)
    out = F.normalize(F.conv2d(f, ww.view(2048, 2048, 1, 1), wb).squeeze(-1).squeeze(-1), dim=-1)
    np.testing.assert_allclose(out.numpy(), fx["gem_net"], rtol=0, atol=1e-6)
    pw, pb = synthetic_linear(512, 2048, int(fx["proj_seed"]))
    pt = torch.ones(1) * 3.0
    f2 = F.avg_pool2d(x2.clamp(min=1e-6).pow(pt), (7, 7)).pow(1.0 / pt).view(2, -1)
    out2 = F.normalize(F.linear(f2, pw, pb), p=2, dim=1)
    np.testing.assert_allclose(out2.numpy(), fx["gem_model"], rtol=0, atol=1e-6)


def test_pca_whitening_learn_matches_reference():
    """The oracle's restatement of pcawhitenlearn_shrinkage + ConvDimReduction
    (networks/backbone.py:42-58, networks/spca.py:215-227) against the
    reference's own outputs, bit-exact."""
    fx = load("pcaw")
    m, PT = embed_ref.pcawhitenlearn_ref(fx["X"])
    np.testing.assert_array_equal(m, fx["mean"])
    np.testing.assert_array_equal(PT, fx["PT"])
    P = PT.T
    w = torch.tensor(P[:32, :], dtype=torch.float32)
    b = -torch.mm(torch.tensor(P, dtype=torch.float32), torch.tensor(m.T, dtype=torch.float32)).squeeze()[:32]
    np.testing.assert_array_equal(w.numpy(), fx["w"].reshape(32, 64))
    np.testing.assert_array_equal(b.numpy(), fx["b"])
    y = embed_ref.pcaw_apply(torch.from_numpy(fx["Y"]), w, b)
    np.testing.assert_allclose(y.numpy(), fx["y"], rtol=0, atol=1e-6)


def test_map_evaluator_bitexact():
    from research_image_retrieval_amd.evaluate import compute_map, compute_map_and_print
    fx = load("map")
    gnd, ranks = I.map_inputs(int(fx["seed"]))
    full = compute_map_and_print("roxford5k", "g", "global", ranks, gnd, kappas=[1, 5, 10])
    assert np.array_equal(np.array(full), fx["full"])
    lists = [ranks[:100, i] for i in range(ranks.shape[1])]
    trunc = compute_map_and_print("rparis6k", "g", "global", lists, gnd, kappas=[1, 5, 10], li=True)
    assert np.array_equal(np.array(trunc), fx["trunc"])
    g_m = [{"ok": np.concatenate([x["easy"], x["hard"]]), "junk": x["junk"]} for x in gnd]
    mAP, aps, pr, prs = compute_map(ranks, g_m, [1, 5, 10])
    assert mAP == fx["medium_map"]
    assert np.array_equal(aps, fx["medium_aps"]) and np.array_equal(pr, fx["medium_pr"])
    assert np.array_equal(prs, fx["medium_prs"])
    mAP2, aps2 = compute_map(ranks, g_m)
    assert mAP2 == fx["medium_map_nokeeps"] and np.array_equal(aps2, fx["medium_aps_nokeeps"])


def test_map_evaluator_handles_reference_crash_cases():
    from research_image_retrieval_amd.evaluate import compute_map, compute_map_and_print
    gnd = [{"ok": np.array([5, 6]), "junk": np.array([1])}, {"ok": np.array([0]), "junk": np.array([], dtype=int)}]
    lists = [np.array([0, 1, 2]), np.array([0, 3])]  # query 0 has no positive in its list
    mAP, aps, pr, prs = compute_map(lists, gnd, [1, 5], li=True)
    assert aps[0] == 0.0 and aps[1] == 1.0 and prs[0].tolist() == [0.0, 0.0]
    assert compute_map_and_print("oxford5k", "g", "global", np.array([[0, 0], [5, 3], [6, 1]]), gnd) >= 0


def test_oracle_extract_vectors_multiscale():
    fx = load("extract")
    tn = I.TinyNetRef(int(fx["net_seed"]))
    imgs = I.tiny_images(int(fx["img_seed"]))
    v1 = embed_ref.extract_vectors_ref(tn.forward_test, imgs, ms=(1,))
    v3 = embed_ref.extract_vectors_ref(tn.forward_test, imgs, ms=(1, 1 / np.sqrt(2), 1 / 2))
    np.testing.assert_array_equal(v1.numpy(), fx["v1"])
    np.testing.assert_array_equal(v3.numpy(), fx["v3"])


def test_oracle_merge_and_topk_rows_consistent():
    rs = np.random.RandomState(0)
    s = rs.standard_normal((5, 300)).astype(np.float32)
    s[:, 10] = s[:, 20]  # ties
    ts, ti = oracle.topk_rows(s, 50)
    np.testing.assert_array_equal(ti, oracle.argsort_stable_desc(s)[:, :50])
    parts_s = np.stack([s[:, :150], s[:, 150:]])
    p0s, p0i = oracle.topk_rows(parts_s[0], 50)
    p1s, p1i = oracle.topk_rows(parts_s[1], 50, idx_offset=150)
    ms, mi = oracle.topk_merge(np.stack([p0s, p1s]), np.stack([p0i, p1i]), 50)
    np.testing.assert_array_equal(mi, ti)
    np.testing.assert_array_equal(ms, ts)


@pytest.mark.parametrize("tag", ["tiny", "b16"])
def test_oracle_vit_vs_reference(tag):
    fx = load("vit")
    res, patch, width, layers, heads, out_dim, seed = (int(v) for v in fx[tag + "_cfg"])
    sd = I.vit_state_dict(seed, width, layers, heads, patch, res, out_dim)
    rsx = np.random.RandomState(seed + 100)
    x = torch.from_numpy(rsx.standard_normal((2, 3, res, res)).astype(np.float32))
    with torch.no_grad():
        out = embed_ref.vit_forward(x, sd, patch, width, layers, heads).numpy()
    ref = fx[tag]
    assert np.abs(out - ref).max() < 1e-4 * max(1.0, np.abs(ref).max())


@pytest.mark.parametrize("tag", ["b2_224", "b1_odd"])
def test_oracle_trunk_vs_reference_resnet_dolg(tag):
    """The oracle's ResNet-101 trunk with the stride on the 1x1 (stride_on="1x1")
    against the reference's own torchvision-free R101, ResNet_DOLG
    (networks/backbone.py:218-274, :305-346), run by make_golden.py with the
    same seeded weights remapped to its keys."""
    from research_image_retrieval_amd import weights as W
    fx = load("resnet_dolg")
    sd = W.synthetic_resnet_state_dict("resnet101", int(fx["weight_seed"]))
    seed, b, h, w = (int(v) for v in fx[tag + "_case"])
    with torch.no_grad():
        x3, x4 = embed_ref.resnet_trunk(I.trunk_input(seed, b, h, w), sd, W.RESNET_LAYERS["resnet101"],
                                        stride_on="1x1", return_x3=True)
    np.testing.assert_allclose(x4.numpy(), fx[tag + "_x4"], rtol=0, atol=1e-6)
    if tag + "_x3" in fx:
        np.testing.assert_allclose(x3.numpy(), fx[tag + "_x3"], rtol=0, atol=1e-6)


@pytest.mark.parametrize("tag", ["b2_224", "b1_odd"])
def test_oracle_trunk_v15_vs_reference_modules(tag):
    """The oracle's default torchvision-v1.5 trunk (stride on the 3x3) against
    the reference's ResNet_DOLG modules with each stage-entry stride moved to
    the 3x3 `b` conv (make_golden.py trunk_fixture_v15)."""
    from research_image_retrieval_amd import weights as W
    fx = load("resnet_dolg_v15")
    sd = W.synthetic_resnet_state_dict("resnet101", int(fx["weight_seed"]))
    seed, b, h, w = (int(v) for v in fx[tag + "_case"])
    with torch.no_grad():
        x3, x4 = embed_ref.resnet_trunk(I.trunk_input(seed, b, h, w), sd, W.RESNET_LAYERS["resnet101"],
                                        stride_on="3x3", return_x3=True)
    np.testing.assert_allclose(x4.numpy(), fx[tag + "_x4"], rtol=0, atol=1e-6)
    if tag + "_x3" in fx:
        np.testing.assert_allclose(x3.numpy(), fx[tag + "_x3"], rtol=0, atol=1e-6)


def test_dolg_key_layout_round_trip():
    """ResNet_DOLG keys (stem.*, s{K}.b{M}.{proj,bn,f.*}) <-> torchvision keys."""
    from research_image_retrieval_amd import weights as W
    sd = W.synthetic_resnet_state_dict("resnet101", 1)
    d = W.to_dolg_keys(sd)
    assert "stem.conv.weight" in d and "s3.b23.f.c_bn.running_var" in d and "s1.b1.proj.weight" in d
    t = W.to_torchvision_keys({"globalmodel.backbone." + k: v for k, v in d.items()})
    assert list(t) == list(sd) and all(torch.equal(t[k], sd[k]) for k in sd)
