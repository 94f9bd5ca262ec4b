"""End-to-end parity of the C4 and C5 bench configurations at the bench's
batch (1280 images of 224x224 uint8 per step), where the tile pickers select
the same kernels as bench.py does (the C3 counterpart is test_gpu_e2e.py).

C4 (bench.py --workload c4): networks.VisionTransformer ViT-B/16 in bf16 on
librr, 512-d CLS descriptors (reference networks/model.py:206-243, pinned by
tests/golden/vit.npz through the oracle's vit_forward), ranked with the bf16
ranker.  C5 (--workload c5): the C3 extractor at three scales
(utils/helpfunc.py:30-46 semantics), fp8 ranking, alpha-QE, fp8 re-search.

Oracles: 16 images sampled across the batch (first and last included) go
through the oracle's fp32 torch-CPU restatement of the reference extractor.
The rankings are checked against the same contraction on the dequantised
rows (the reduced-precision gallery is the build's C4 / C5 configuration):
float64 dot products of the bf16 / fp8 rows, stable order, identical except
where neighbouring float64 scores are closer than TIE_EPS (fp32 accumulation
may swap those).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import oracle
from oracle import embed_ref
from research_image_retrieval_amd import ops
from research_image_retrieval_amd import weights as W
from research_image_retrieval_amd.extract import _rescale
from research_image_retrieval_amd.networks import ConvDimReduction, GeM, GeMPCAw, VisionTransformer

pytestmark = pytest.mark.gpu

B = 1280
N_GAL = 200_000
K = 100
TIE_EPS = 2e-6
SCALES = (1.0, 1.0 / np.sqrt(2.0), 0.5)  # bench.py C5


def _images():
    rs = np.random.RandomState(1234)  # bench.py's images for rank 0
    return torch.from_numpy(rs.randint(0, 256, size=(B, 224, 224, 3), dtype=np.uint8))


def _pick():
    return np.unique(np.linspace(0, B - 1, 16).astype(np.int64))


def _gallery(d, planted, seed):
    gen = torch.Generator().manual_seed(seed)
    gal = torch.randn(N_GAL, d, generator=gen)
    for j, v in enumerate(planted):
        gal[1000 + 37 * j] = v + 0.002 * torch.randn(d, generator=gen)
    return F.normalize(gal, p=2, dim=1)


def _dequant(x, sc, dtype):
    if dtype == "bf16":
        return x.float().double()
    return x.view(torch.float8_e4m3fn).float().double() * sc.double()[:, None]


def _check_ranking(name, s, i, qd, gd):
    """GPU lists (s, i) [Q, K] vs the float64 stable ranking of the dequantised
    rows qd [Q, d] x gd [N, d]: scores within 1e-5, indices identical except at
    near-ties."""
    sim = (qd @ gd.t()).numpy()
    order = np.argsort(-sim, axis=1, kind="stable")[:, :K]
    ref_s = np.take_along_axis(sim, order, 1)
    serr = np.abs(s.astype(np.float64) - ref_s).max()
    d = np.abs(np.diff(ref_s, axis=1)) < TIE_EPS
    tie = np.zeros_like(order, dtype=bool)
    tie[:, 1:] |= d
    tie[:, :-1] |= d
    mism = i != order
    print(f"{name}: max|score - float64 dot of dequantised rows| {serr:.3e}; {int(tie.sum())} near-tie positions; "
          f"{int(mism.sum())} index differences, all at near-ties: {not (mism & ~tie).any()}")
    assert serr < 1e-5
    assert not (mism & ~tie).any(), np.argwhere(mism & ~tie)[:5]


def test_c4_vit_bf16_embed_and_rank_at_bench_batch(cuda):
    sd = W.synthetic_vit_state_dict(out_dim=512, seed=0)  # bench.py C4 weights
    net = VisionTransformer(224, 16, 768, 12, 12, 512, state_dict=sd, device=cuda, dtype="bf16")
    imgs = _images()
    desc = net.forward_test_u8(imgs.to(cuda))
    torch.cuda.synchronize()
    assert desc.shape == (B, 512) and bool(torch.isfinite(desc).all())
    pick = _pick()
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    with torch.no_grad():
        ref = torch.cat([F.normalize(embed_ref.vit_forward(embed_ref.normalize_u8(imgs[i:i + 1]), sd, 16, 768, 12, 12),
                                     dim=-1) for i in pick])
    got = desc[torch.from_numpy(pick).to(cuda)].cpu()
    cos = (got.double() * ref.double()).sum(1)
    print(f"C4 bf16 ViT vs the fp32 oracle over {len(pick)} of {B} images: min cosine {cos.min().item():.7f}, "
          f"max|err| {(got - ref).abs().max().item():.3e}")
    assert float(cos.min()) >= 0.9999

    # bf16 ranking of the bench batch (1280 queries, the bench's tile pick) vs the dequantised rows
    gal = _gallery(512, ref[:4], seed=21)
    g_lp, _ = ops.quantize_rows(gal.to(cuda), "bf16")
    q_lp, _ = ops.quantize_rows(desc, "bf16")
    s, i = ops.cosine_topk_lp(q_lp, None, g_lp, None, K, "bf16")
    sel = torch.from_numpy(np.r_[pick, np.arange(0, B, 97)]).unique()
    s, i = s.cpu()[sel].numpy(), i.cpu()[sel].numpy()
    _check_ranking("C4 bf16 ranking", s, i, _dequant(q_lp.cpu()[sel], None, "bf16"), _dequant(g_lp.cpu(), None, "bf16"))


def test_c5_multiscale_fp8_alpha_qe_at_bench_batch(cuda):
    sd = W.synthetic_resnet_state_dict("resnet101", 0)  # bench.py build_extractor(seed=0)
    ww, wb = W.synthetic_linear(2048, 2048, 1)
    pw, pb = W.synthetic_linear(2048, 2048, 5, scale=1.0 / np.sqrt(2048))
    net = GeM(2048, backbone="resnet101", state_dict=sd, whiten=(ww, wb), device=cuda)
    pca = ConvDimReduction(2048, 2048, device=cuda)
    pca.set_params(pw, pb)
    ext = GeMPCAw(net, pca)
    imgs = _images()
    # bench.py C5 embed(): rescale, embed, sum, / #scales, renormalise
    x = ops.preprocess_u8(imgs.to(cuda), out_c=4)
    acc = None
    for sc in SCALES:
        f = ext.forward_test_nhwc(x if sc == 1.0 else _rescale(x, sc))
        acc = f.clone() if acc is None else acc.add_(f)
    acc.div_(len(SCALES))
    desc = ops.l2_normalize(acc, 1e-12, out=acc)
    torch.cuda.synchronize()
    del x
    pick = _pick()
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))

    def fwd(t):  # GeMPCAw.forward_test in the reference op order (see test_gpu_e2e.py)
        f = F.conv2d(embed_ref.gem(embed_ref.resnet_trunk(t, sd, W.RESNET_LAYERS["resnet101"])),
                     ww.view(2048, 2048, 1, 1), wb).flatten(1)
        return embed_ref.pcaw_apply(F.normalize(f, dim=-1), pw, pb)

    with torch.no_grad():
        ref = embed_ref.extract_vectors_ref(fwd, [embed_ref.normalize_u8(imgs[i:i + 1]) for i in pick], ms=SCALES)
    got = desc[torch.from_numpy(pick).to(cuda)].cpu()
    err = (got - ref).abs().max().item()
    print(f"C5 3-scale descriptors vs extract_vectors_ref over {len(pick)} of {B} images: max|err| {err:.3e}")
    assert err < 1e-6

    gal = _gallery(2048, ref[:4], seed=22)
    g_d = gal.to(cuda)
    g_lp, g_sc = ops.quantize_rows(g_d, "fp8")
    q_lp, q_sc = ops.quantize_rows(desc, "fp8")
    s1, i1 = ops.cosine_topk_lp(q_lp, q_sc, g_lp, g_sc, K, "fp8")
    q2 = ops.alpha_qe(desc, g_d, i1, s1, n=2, alpha=3.0)
    q2_lp, q2_sc = ops.quantize_rows(q2, "fp8")
    s2, i2 = ops.cosine_topk_lp(q2_lp, q2_sc, g_lp, g_sc, K, "fp8")
    sel = torch.from_numpy(np.r_[pick, np.arange(0, B, 97)]).unique()
    gd = _dequant(g_lp.cpu(), g_sc.cpu(), "fp8")
    _check_ranking("C5 fp8 search", s1.cpu()[sel].numpy(), i1.cpu()[sel].numpy(),
                   _dequant(q_lp.cpu()[sel], q_sc.cpu()[sel], "fp8"), gd)
    # alpha-QE vs the oracle's float64 restatement on the same neighbour lists
    q2_ref = oracle.alpha_qe(desc.cpu()[sel].numpy(), gal.numpy(), i1.cpu()[sel].numpy(), s1.cpu()[sel].numpy(),
                             n=2, alpha=3.0)
    qerr = np.abs(q2.cpu()[sel].numpy() - q2_ref).max()
    print(f"C5 alpha-QE queries vs float64 oracle: max|err| {qerr:.3e}")
    assert qerr < 2e-6
    _check_ranking("C5 fp8 re-search", s2.cpu()[sel].numpy(), i2.cpu()[sel].numpy(),
                   _dequant(q2_lp.cpu()[sel], q2_sc.cpu()[sel], "fp8"), gd)
    # the planted near-duplicates lead the first search
    planted = set((1000 + 37 * np.arange(4)).tolist())
    i1c = i1.cpu().numpy()
    assert all(set(i1c[q, :4].tolist()) == planted for q in pick[:4])
