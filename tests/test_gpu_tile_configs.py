"""Every GEMM tile config of every core, forced through rr_set_tuning, on every
operand mode it can serve — against float64.

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


# (b, h, w, cin, cout, k, stride, pad, residual): a dense 1x1, a strided 3x3
# with ragged N, a 1x1/2 projection, and a residual 1x1
S3_CONVS = [(3, 13, 11, 64, 96, 1, 1, 0, True), (2, 15, 13, 32, 160, 3, 2, 1, False),
            (2, 14, 14, 64, 256, 1, 2, 0, False), (2, 9, 11, 128, 512, 3, 1, 1, True),
            (2, 7, 9, 32, 128, 1, 1, 0, False)]  # K = 32: a single BK = 32 k-tile


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("shape", S3_CONVS)
def test_s3_conv_every_tile_config(cuda, cfg, shape):
    b, h, w, cin, cout, k, s, p, res = shape
    g = torch.Generator().manual_seed(cfg * 100 + cin + cout)
    x = torch.relu(torch.randn(b, h, w, cin, generator=g))
    wt = torch.randn(cout, k, k, cin, generator=g) * (2.0 / (k * k * cin)) ** 0.5
    bias = torch.randn(cout, generator=g) * 0.1
    oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    r = torch.randn(b, oh, ow, cout, generator=g) if res else None
    ref, scale = _ref_conv(x, wt, bias, s, p, r)
    w3 = ops.split3_bf16(wt.to(cuda))
    with ops.tuning(cuda.index, s3_cfg=cfg):
        y = ops.conv2d_s3(x.to(cuda), w3, bias.to(cuda), s, p, None if r is None else r.to(cuda), True).cpu()
    _check(y, ref, scale, 4e-7)


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5, 6, 7])
@pytest.mark.parametrize("b,h,w", [(2, 224, 224), (1, 37, 53)])
def test_s3_stem_every_tile_config(cuda, cfg, b, h, w):
    """The NHWC4 stem (7x7/2, K = 196 padded to 224): BK = 16 tiles (configs 1
    and 6) cover 4 filter taps per k-tile, BK = 32 tiles 8."""
    g = torch.Generator().manual_seed(cfg + b * h)
    x = torch.randn(b, h, w, 3, generator=g) * 1.5
    wt = torch.randn(64, 7, 7, 3, generator=g) * (2.0 / 147) ** 0.5
    bias = torch.randn(64, generator=g) * 0.1
    ref, scale = _ref_conv(x, wt, bias, 2, 3, None)
    w3p, shp = ops.split3_stem(F.pad(wt, (0, 1)).contiguous().to(cuda))
    with ops.tuning(cuda.index, s3_cfg=cfg):
        y = ops.conv2d_s3_stem(F.pad(x, (0, 1)).contiguous().to(cuda), w3p, shp, bias.to(cuda), 2, 3, True).cpu()
    _check(y, ref, scale, 4e-7)


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5, 6, 7, 8])
def test_s3_linear_every_tile_config(cuda, cfg):
    g = torch.Generator().manual_seed(cfg)
    m, k, n = 517, 320, 320
    a = torch.relu(torch.randn(m, k, generator=g))
    wt = torch.randn(n, k, generator=g) / k ** 0.5
    ref = a.double() @ wt.double().t()
    scale = a.double().abs() @ wt.double().abs().t()
    with ops.tuning(cuda.index, s3_cfg=cfg):
        y = ops.linear_s3(a.to(cuda), ops.split3_bf16(wt.to(cuda))).cpu()
    _check(y, ref, scale, 4e-7)


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


def test_s3_round_stagger_changes_nothing_but_timing(cuda):
    """The first-round stagger (RR_TUNE_S3_STAGGER; default on for residual
    layers) only delays blocks: outputs are bit-identical for every value, on a
    grid of several rounds."""
    g = torch.Generator().manual_seed(5)
    x = torch.relu(torch.randn(8, 28, 28, 256, generator=g)).to(cuda)
    wt = (torch.randn(1024, 1, 1, 256, generator=g) * (2.0 / 256) ** 0.5).to(cuda)
    bias = (torch.randn(1024, generator=g) * 0.1).to(cuda)
    r = torch.randn(8, 28, 28, 1024, generator=g).to(cuda)
    w3 = ops.split3_bf16(wt)
    outs = []
    for st in (0, 3, 20, -1):
        with ops.tuning(cuda.index, s3_stagger=st):
            outs.append(ops.conv2d_s3(x, w3, bias, 1, 0, r, True).cpu())
    assert all(torch.equal(outs[0], o) for o in outs[1:])


@pytest.mark.parametrize("b,h,cin,cout,res,relu", [(4, 56, 256, 1024, True, True), (3, 37, 64, 256, True, True),
                                                   (2, 29, 512, 256, False, True), (1, 14, 1024, 512, False, False),
                                                   (9, 14, 128, 512, True, True)])
def test_s3_persistent_tile_bit_identical(cuda, b, h, cin, cout, res, relu):
    """Config 8 (one block per CU walking its tiles as one k-stream, the
    epilogue in the freed stage) computes exactly what config 4 computes: the
    same k order and epilogue arithmetic.  Shapes with several tiles per block
    (b = 4: 392 tiles), ragged M, K = 64 (one pair of k-tiles per tile), no
    residual and no ReLU (the projection conv)."""
    g = torch.Generator().manual_seed(b * 1000 + cin + cout)
    x = torch.relu(torch.randn(b, h, h, cin, generator=g)).to(cuda)
    wt = (torch.randn(cout, 1, 1, cin, generator=g) * (2.0 / cin) ** 0.5).to(cuda)
    bias = (torch.randn(cout, generator=g) * 0.1).to(cuda)
    r = torch.randn(b, h, h, cout, generator=g).to(cuda) if res else None
    w3 = ops.split3_bf16(wt)
    outs = {}
    for cfg in (4, 8):
        with ops.tuning(cuda.index, s3_cfg=cfg):
            outs[cfg] = ops.conv2d_s3(x, w3, bias, 1, 0, r, relu).cpu()
    assert torch.equal(outs[4], outs[8])
    ref = torch.einsum("bhwc,oc->bhwo", x.double().cpu(), wt[:, 0, 0].double().cpu()) + bias.double().cpu()
    if res:
        ref = ref + r.double().cpu()
    if relu:
        ref = torch.relu(ref)
    assert (outs[8].double() - ref).abs().max().item() < 1e-4
