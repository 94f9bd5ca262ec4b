"""End-to-end north_star parity at the bench's configuration (C3).

The GPU path embeds the bench's full 1280-image batch of 224x224 uint8 images
(ResNet-101-GeM -> whiten -> L2 -> PCA-w -> L2, networks.GeMPCAw on librr)
and ranks it with the default C3 ranker (bf16-bound prefilter + exact fp32
rescoring).  The reference CPU path — the oracle's torch-CPU restatement of the
extractor (trunk pinned to the reference's ResNet_DOLG, tails pinned to the
reference's own functions) followed by the reference's ranker op sequence
(F.normalize, torch.mm, argsort(-sim); iris_evaluate.py:378-386) — embeds 16
images sampled across the batch (first and last included, so the 4 M-row 1x1
convs' and the 1.03e9-element stem's far ends are covered) and ranks them
against the same 200k x 2048 gallery.

north_star bar: cosine scores within 1e-5 fp32, ranked indices identical except
where the reference's own sorted scores are closer than 2e-6 (near-ties, where
1-ulp accumulation-order differences may legally swap neighbours); the
near-tie count is printed.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import embed_ref
from research_image_retrieval_amd import ops
from research_image_retrieval_amd import weights as W
from research_image_retrieval_amd.networks import GeM, ConvDimReduction, GeMPCAw

pytestmark = pytest.mark.gpu

B = 1280          # bench.py's default images per GPU per step (C3)
N_GAL = 200_000   # one 8-way shard of the 1.6 M gallery
K = 100
TRUNK_TOL = 2e-6  # max-abs on the [7,7,2048] trunk output (values <= ~0.6)
DESC_TOL = 1e-6   # max-abs on unit-norm 2048-d descriptors
SCORE_TOL = 1e-5  # north_star: cosine scores within 1e-5 fp32
TIE_EPS = 2e-6


def _c3_weights(seed=0):
    sd = W.synthetic_resnet_state_dict("resnet101", seed)
    ww, wb = W.synthetic_linear(2048, 2048, seed + 1)
    pw, pb = W.synthetic_linear(2048, 2048, seed + 5, scale=1.0 / np.sqrt(2048))
    return sd, ww, wb, pw, pb


def test_c3_embed_and_rank_parity_at_bench_batch(cuda):
    sd, ww, wb, pw, pb = _c3_weights(0)
    net = GeM(2048, backbone="resnet101", state_dict=sd, whiten=(ww, wb), device=cuda)
    pca = ConvDimReduction(2048, 2048, device=cuda)
    pca.set_params(pw, pb)
    ext = GeMPCAw(net, pca)
    rs = np.random.RandomState(1234)
    imgs = torch.from_numpy(rs.randint(0, 256, size=(B, 224, 224, 3), dtype=np.uint8))
    imgs_d = imgs.to(cuda)
    desc = ext.forward_test_u8(imgs_d)
    # the trunk output too: random-weight trunks damp input-side errors strongly
    # (a wrong stem moved the descriptors by only ~1e-5), so it is checked on its own
    pick = np.unique(np.linspace(0, B - 1, 16).astype(np.int64))
    pick_d = torch.from_numpy(pick).to(cuda)
    feat = net.backbone(ops.preprocess_u8(imgs_d, out_c=4))[pick_d].permute(0, 3, 1, 2).cpu()
    torch.cuda.synchronize()
    assert desc.shape == (B, 2048) and torch.isfinite(desc).all()

    # oracle on 16 images spread over the batch (reference CPU path, batch 1 as extract_vectors runs it)
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    tr, ref = [], []
    with torch.no_grad():
        for i in pick:
            t = embed_ref.resnet_trunk(embed_ref.normalize_u8(imgs[i:i + 1]), sd, W.RESNET_LAYERS["resnet101"])
            f = F.conv2d(embed_ref.gem(t), ww.view(2048, 2048, 1, 1), wb).flatten(1)  # GeM.forward_test tail
            ref.append(embed_ref.pcaw_apply(F.normalize(f, dim=-1), pw, pb))
            tr.append(t)
    tr, ref = torch.cat(tr), torch.cat(ref)
    terr = (feat - tr).abs().max().item()
    got = desc[pick_d].cpu()
    err = (got - ref).abs().max().item()
    print(f"C3 trunk: max|err| {terr:.3e} (max|x| {tr.abs().max().item():.3f}); descriptors: max|err| {err:.3e} "
          f"over {len(pick)} sampled images of {B}")
    assert terr < TRUNK_TOL
    assert err < DESC_TOL

    # gallery: seeded Gaussian rows plus near-duplicates of 4 sampled queries (known top-1s)
    gen = torch.Generator().manual_seed(11)
    gal = torch.randn(N_GAL, 2048, generator=gen)
    for j, qi in enumerate(range(4)):
        gal[1000 + 37 * j] = ref[qi] + 0.002 * torch.randn(2048, generator=gen)  # cos ~ 0.996
    gal = F.normalize(gal, p=2, dim=1)  # iris_evaluate.py:380

    # reference ranker on oracle descriptors (iris_evaluate.py:379-386; stable argsort = index tie-break)
    sim = torch.mm(F.normalize(ref, p=2, dim=1), gal.t()).numpy()
    order = np.argsort(-sim, axis=1, kind="stable")[:, :K]
    ref_s = np.take_along_axis(sim, order, 1)

    # GPU: the bench's default C3 ranker on GPU descriptors
    g_dev = gal.to(cuda)
    g_bf, _ = ops.quantize_rows(g_dev, "bf16")
    bound = ops.prefilter_gallery_bound(g_dev, g_bf)
    s, i = ops.cosine_topk_prefilter(got.to(cuda), g_dev, g_bf, bound, K)
    s, i = s.cpu().numpy(), i.cpu().numpy()
    s_x, i_x = ops.cosine_topk(got.to(cuda), g_dev, K)
    assert np.array_equal(i, i_x.cpu().numpy()) and np.array_equal(s, s_x.cpu().numpy())

    serr = np.abs(s - ref_s).max()
    d = np.abs(np.diff(ref_s, axis=1)) < TIE_EPS
    tie = np.zeros_like(order, dtype=bool)
    tie[:, 1:] |= d
    tie[:, :-1] |= d
    mism = i != order
    print(f"C3 ranking: max|score err| {serr:.3e}; {int(tie.sum())} near-tie positions (gap < {TIE_EPS}) of "
          f"{tie.size}; {int(mism.sum())} index differences, all at near-ties: {not (mism & ~tie).any()}")
    assert serr < SCORE_TOL
    assert not (mism & ~tie).any(), np.argwhere(mism & ~tie)[:5]
    # the planted near-duplicates lead (as a set: this random-weight extractor maps
    # different images to highly correlated descriptors, so each query is close to all four)
    planted = set((1000 + 37 * np.arange(4)).tolist())
    assert all(set(i[q, :4].tolist()) == planted for q in range(4))
