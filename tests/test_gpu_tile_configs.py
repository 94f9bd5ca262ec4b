"""Every GEMM tile config of the exact-fp32 and bf16 / fp8 cores, forced
through rr_set_tuning, on every operand mode it can serve — against float64
(the f16x2 split core's configs: tests/test_gpu_h2.py).

The library picks tiles by shape; a config the picker only reaches at large
batch is otherwise untested at small test sizes.  (Round 2 found exactly that:
the NHWC4 stem on the split-bf16 core's BK = 16 tiles, picked only at >= ~16
images of 224x224, read the wrong filter taps.)"""
import pytest
import torch
import torch.nn.functional as F

from research_image_retrieval_amd import ops

pytestmark = pytest.mark.gpu


def _ref_conv(x, wt, bias, s, p, res):
    xn, wn = x.permute(0, 3, 1, 2).double(), wt.permute(0, 3, 1, 2).double()
    ref = F.conv2d(xn, wn, None, s, p).permute(0, 2, 3, 1) + bias.double()
    if res is not None:
        ref = ref + res.double()
    scale = F.conv2d(xn.abs(), wn.abs(), None, s, p).permute(0, 2, 3, 1) + bias.double().abs()
    return torch.relu(ref), scale


def _check(y, ref, scale, tol):
    e = ((y.double() - ref).abs() / (scale + 1e-30)).max().item()
    assert e < tol, e
    return e


F32_CFGS = [(22, 16), (22, 32), (41, 16), (41, 32), (88, 32)]


@pytest.mark.parametrize("cfg,bk", F32_CFGS)
@pytest.mark.parametrize("mode", ["dense", "conv", "stem4", "generic"])
def test_f32_core_every_tile_config(cuda, cfg, bk, mode):
    g = torch.Generator().manual_seed(cfg + bk)
    if mode == "dense":
        b, h, w, cin, cout, k, s, p = 2, 9, 15, 64, 256, 1, 1, 0
    elif mode == "conv":
        b, h, w, cin, cout, k, s, p = 2, 11, 9, 32, 256, 3, 2, 1
    elif mode == "stem4":
        b, h, w, cin, cout, k, s, p = 1, 45, 37, 4, 64, 7, 2, 3
    else:
        b, h, w, cin, cout, k, s, p = 2, 13, 12, 3, 64, 3, 1, 1
    x = torch.randn(b, h, w, cin, generator=g)
    if mode == "stem4":
        x[..., 3] = 0
    wt = torch.randn(cout, k, k, cin, generator=g) * (2.0 / (k * k * cin)) ** 0.5
    bias = torch.randn(cout, generator=g) * 0.1
    ref, scale = _ref_conv(x, wt, bias, s, p, None)
    with ops.tuning(cuda.index, gemm_cfg=cfg, gemm_bk=bk):
        y = ops.conv2d(x.to(cuda), wt.contiguous().to(cuda), bias.to(cuda), s, p, None, True).cpu()
    _check(y, ref, scale, 2e-6)


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
def test_lowp_every_tile_config(cuda, cfg, dtype):
    """bf16 / fp8 linears (stored C) and filter sweeps (top-k) on every config:
    the dot products of the quantised operands, exact products with fp32
    accumulation, against float64 on the same quantised values."""
    g = torch.Generator().manual_seed(cfg + (7 if dtype == "fp8" else 0))
    m, n, k = 700, 320, 2048
    a = F.normalize(torch.randn(m, k, generator=g), dim=1).to(cuda)
    b = F.normalize(torch.randn(n, k, generator=g), dim=1).to(cuda)
    qa, sa = ops.quantize_rows(a, dtype)
    qb, sb = ops.quantize_rows(b, dtype)
    if dtype == "bf16":
        fa, fb = qa.double().cpu(), qb.double().cpu()
    else:
        fa = qa.cpu().view(torch.float8_e4m3fn).double() * sa.cpu().double()[:, None]
        fb = qb.cpu().view(torch.float8_e4m3fn).double() * sb.cpu().double()[:, None]
    ref = fb @ fa.t()  # [n queries, m rows]
    with ops.tuning(cuda.index, lp_cfg=cfg):
        s, i = ops.cosine_topk_lp(qb, sb, qa, sa, 50, dtype)
        if dtype == "bf16":
            y = ops.linear_bf16(qa, qb).cpu().double()
            assert (y - fa @ fb.t()).abs().max().item() < 1e-5
    s, i = s.cpu().double(), i.cpu()
    assert (s - torch.gather(ref, 1, i)).abs().max().item() < 1e-5
    kth = ref.topk(50, dim=1).values[:, -1:]
    assert bool((s[:, -1:] >= kth - 1e-5).all())


def test_h2_round_stagger_changes_nothing_but_timing(cuda):
    """The first-round stagger of the split core (RR_TUNE_S3_STAGGER; default
    on for residual layers) only delays blocks: the f16x2 conv's outputs are
    bit-identical for every value, on a grid of several rounds."""
    g = torch.Generator().manual_seed(5)
    x = torch.relu(torch.randn(8, 28, 28, 256, generator=g)).to(cuda)
    wt = (torch.randn(1024, 1, 1, 256, generator=g) * (2.0 / 256) ** 0.5).to(cuda)
    bias = (torch.randn(1024, generator=g) * 0.1).to(cuda)
    r = torch.randn(8, 28, 28, 1024, generator=g).to(cuda)
    wc = ops.H2Conv(wt)
    rec = ops.amax_records(1, cuda)
    ops.amax_f32(x, rec[0])
    outs = []
    for st in (0, 3, 20, -1):
        with ops.tuning(cuda.index, s3_stagger=st):
            outs.append(ops.conv2d_h2(x, rec[0], wc, bias, 1, 0, r, True).cpu())
    assert all(torch.equal(outs[0], o) for o in outs[1:])
