"""The split-bf16 GEMM core (gemm_s3.hip): exactness of the 3-way split, and
fp32-grade accuracy of the convolutions / linears it runs, measured against
float64 next to the exact-fp32 MFMA core on the same inputs.

The bar: the split core's error vs float64 is at most the exact-fp32 core's
(max and mean over the outputs, errors relative to sum |a||b| per output), so
switching the ResNet trunk onto it loses no precision against the reference's
fp32 CPU path (networks/backbone.py:60-109)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import embed_ref
from research_image_retrieval_amd import ops
from research_image_retrieval_amd import weights as W
from research_image_retrieval_amd.networks import GeM

pytestmark = pytest.mark.gpu

DESC_TOL = 1e-6  # as tests/test_gpu_embed.py (measured 1.4e-7)


def _planes_to_f32(p):
    return (p.to(torch.int32) << 16).view(torch.float32)


def test_split3_exact(cuda):
    rs = np.random.RandomState(0)
    x = (rs.standard_normal(1 << 16) * np.exp2(rs.randint(-40, 40, 1 << 16))).astype(np.float32)
    x[:7] = [0.0, -0.0, 1.0, -1.0, 3.4e38, 1.17549435e-38, 2.0 ** -126 * 1.5]
    p = ops.split3_bf16(torch.from_numpy(x).to(cuda)).cpu()
    f = _planes_to_f32(p).double()
    assert torch.equal(f.sum(0), torch.from_numpy(x).double()), "x != x0 + x1 + x2"
    # the pieces shrink by >= 2^7 each: x1 < 2^-7 |x|, x2 < 2^-15 |x|
    ax = torch.from_numpy(np.abs(x)).double()
    assert bool((f[1].abs() <= ax * 2.0 ** -7).all()) and bool((f[2].abs() <= ax * 2.0 ** -15).all())


def _rel_err(got, ref64, scale64):
    e = (got.double() - ref64).abs() / scale64.clamp_min(1e-300)
    return e.max().item(), e.mean().item()


@pytest.mark.parametrize("m,k,n", [(300, 256, 200), (517, 2048, 256), (130, 4608, 96), (64, 1024, 198)])
def test_linear_s3_accuracy_vs_float64(cuda, m, k, n):
    g = torch.Generator().manual_seed(m + k + n)
    a = torch.relu(torch.randn(m, k, generator=g))  # post-ReLU activations
    w = torch.randn(n, k, generator=g) / k ** 0.5
    ref = a.double() @ w.double().t()
    scale = a.double().abs() @ w.double().abs().t()
    ad, wd = a.to(cuda), w.to(cuda)
    y_s3 = ops.linear_s3(ad, ops.split3_bf16(wd)).cpu()
    y_f32 = ops.linear(ad, wd).cpu()
    es3, ef32 = _rel_err(y_s3, ref, scale), _rel_err(y_f32, ref, scale)
    print(f"linear {m}x{k}x{n}: s3 max {es3[0]:.3g} mean {es3[1]:.3g} | f32 max {ef32[0]:.3g} mean {ef32[1]:.3g}")
    assert es3[0] <= ef32[0] and es3[1] <= ef32[1]


@pytest.mark.parametrize("m,k,n", [(77, 32, 130), (300, 64, 64), (129, 96, 257), (513, 160, 64), (33, 32, 64),
                                   (77, 32, 256), (129, 96, 512), (33, 160, 256), (300, 64, 768)])
def test_linear_s3_kloop_edges(cuda, m, k, n):
    """Edges of the async-A k-loop (1, 2, 3, 5 k-tiles; ragged M and N on both
    tile configs, N = 64 -> 256x64 tiles, N % 256 == 0 -> the 128x256 tile on
    16x16x32 MFMAs): fp32-grade against float64 (error
    relative to sum |a||b| below 4e-7; at these short K the final hi + lo
    rounding dominates, so no ordering against the fp32 core is asserted)."""
    g = torch.Generator().manual_seed(7 * m + k + n)
    a = torch.relu(torch.randn(m, k, generator=g))
    w = torch.randn(n, k, generator=g) / k ** 0.5
    ref = a.double() @ w.double().t()
    scale = a.double().abs() @ w.double().abs().t()
    y = ops.linear_s3(a.to(cuda), ops.split3_bf16(w.to(cuda))).cpu()
    e = _rel_err(y, ref, scale)
    assert e[0] < 4e-7, e


@pytest.mark.parametrize("n", [320, 256])
def test_linear_s3_epilogue(cuda, n):
    """bias / residual / ReLU / QuickGELU through the stored-C epilogue, on the
    32x32x16 accumulator map (n = 320) and the 16x16x32 one (n = 256)."""
    g = torch.Generator().manual_seed(5)
    m, k = 200, 512
    a, w = torch.randn(m, k, generator=g), torch.randn(n, k, generator=g) / k ** 0.5
    b, r = torch.randn(n, generator=g), torch.randn(m, n, generator=g)
    w3 = ops.split3_bf16(w.to(cuda))
    for act in (0, 1, 2):
        y = ops.linear_s3(a.to(cuda), w3, b.to(cuda), r.to(cuda), act).cpu().double()
        z = a.double() @ w.double().t() + b.double() + r.double()
        z = torch.relu(z) if act == 1 else (z * torch.sigmoid(1.702 * z) if act == 2 else z)
        assert (y - z).abs().max().item() < 2e-5, act


CONV_SHAPES = [  # b, h, w, cin, cout, k, stride, pad, residual
    (2, 14, 14, 64, 128, 3, 1, 1, False),
    (3, 15, 13, 32, 96, 3, 2, 1, False),
    (2, 28, 28, 64, 256, 1, 2, 0, False),
    (2, 9, 11, 256, 64, 1, 1, 0, True),
    (4, 7, 7, 512, 2048, 1, 1, 0, True),
    (2, 14, 14, 256, 256, 3, 1, 1, True),
]


@pytest.mark.parametrize("b,h,w,cin,cout,k,s,p,res", CONV_SHAPES)
def test_conv2d_s3_vs_float64(cuda, b, h, w, cin, cout, k, s, p, res):
    g = torch.Generator().manual_seed(b * h + cin + cout)
    x = torch.relu(torch.randn(b, h, w, cin, generator=g))
    wt = torch.randn(cout, k, k, cin, generator=g) * (2.0 / (k * k * cin)) ** 0.5
    bias = torch.randn(cout, generator=g) * 0.1
    oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    r = torch.randn(b, oh, ow, cout, generator=g) if res else None
    xn, wn = x.permute(0, 3, 1, 2).double(), wt.permute(0, 3, 1, 2).double()
    conv = F.conv2d(xn, wn, None, s, p).permute(0, 2, 3, 1)
    scale = F.conv2d(xn.abs(), wn.abs(), None, s, p).permute(0, 2, 3, 1)
    ref = conv + bias.double() + (r.double() if res else 0.0)
    ref = torch.relu(ref)
    xd, wd = x.to(cuda), wt.to(cuda)
    rd = r.to(cuda) if res else None
    y_s3 = ops.conv2d_s3(xd, ops.split3_bf16(wd), bias.to(cuda), s, p, rd, True).cpu()
    y_f32 = ops.conv2d(xd, wd, bias.to(cuda), s, p, rd, True).cpu()
    # compare where ReLU passes (elsewhere both are 0)
    live = ref > 0
    es3 = _rel_err(y_s3[live], ref[live], scale[live])
    ef32 = _rel_err(y_f32[live], ref[live], scale[live])
    print(f"conv {b}x{h}x{w}x{cin}->{cout} k{k}s{s}: s3 max {es3[0]:.3g} mean {es3[1]:.3g} | "
          f"f32 max {ef32[0]:.3g} mean {ef32[1]:.3g}")
    assert torch.equal(y_s3 == 0, y_f32 == 0) or (y_s3 - y_f32).abs().max().item() < 1e-5
    assert es3[0] <= max(ef32[0], 1e-7) and es3[1] <= ef32[1] * 1.05 + 1e-9


@pytest.mark.parametrize("b,h,w", [(2, 224, 224), (3, 37, 53)])
def test_stem_s3_vs_float64(cuda, b, h, w):
    """The NHWC4 stem (7x7/2, pad 3, 3 channels + a zero channel, K padded to
    224) on the split-bf16 core vs float64, next to the exact-fp32 core."""
    g = torch.Generator().manual_seed(b * h + w)
    x = torch.randn(b, h, w, 3, generator=g) * 1.5
    x4 = F.pad(x, (0, 1)).contiguous()
    wt = torch.randn(64, 7, 7, 3, generator=g) * (2.0 / 147) ** 0.5
    w4 = F.pad(wt, (0, 1)).contiguous()
    bias = torch.randn(64, generator=g) * 0.1
    xn, wn = x.permute(0, 3, 1, 2).double(), wt.permute(0, 3, 1, 2).double()
    ref = torch.relu(F.conv2d(xn, wn, None, 2, 3).permute(0, 2, 3, 1) + bias.double())
    scale = F.conv2d(xn.abs(), wn.abs(), None, 2, 3).permute(0, 2, 3, 1)
    w3p, shp = ops.split3_stem(w4.to(cuda))
    y_s3 = ops.conv2d_s3_stem(x4.to(cuda), w3p, shp, bias.to(cuda), 2, 3, True).cpu()
    y_f32 = ops.conv2d(x4.to(cuda), w4.to(cuda), bias.to(cuda), 2, 3, None, True).cpu()
    assert y_s3.shape == ref.shape
    live = ref > 0
    es3 = _rel_err(y_s3[live], ref[live], scale[live])
    ef32 = _rel_err(y_f32[live], ref[live], scale[live])
    print(f"stem {b}x{h}x{w}: s3 max {es3[0]:.3g} mean {es3[1]:.3g} | f32 max {ef32[0]:.3g} mean {ef32[1]:.3g}")
    assert (y_s3 - torch.relu(ref).float()).abs().max().item() < 1e-4
    assert es3[0] <= max(ef32[0], 1e-7) and es3[1] <= ef32[1] * 1.05 + 1e-9


def test_resnet_s3_descriptors_vs_float64(cuda):
    """The whole R50-GeM extractor: split-bf16 trunk vs exact-fp32 trunk, both
    against the oracle evaluated in float64."""
    rs = np.random.RandomState(3)
    img = torch.from_numpy(rs.randint(0, 256, size=(3, 64, 72, 3), dtype=np.uint8))
    x = embed_ref.normalize_u8(img)
    got = {}
    for math in ("s3", "f32"):
        net = GeM(2048, backbone="resnet50", seed=4, device=cuda, conv_math=math)
        got[math] = net.forward_test(x.to(cuda)).cpu().double()
    sd = {k: v.double() for k, v in W.synthetic_resnet_state_dict("resnet50", 4).items()}
    ww, wb = W.synthetic_linear(2048, 2048, 5)
    ref = embed_ref.gem_net_forward_test(x.double(), sd, W.RESNET_LAYERS["resnet50"], ww.double(), wb.double())
    e_s3 = (got["s3"] - ref).abs().max().item()
    e_f32 = (got["f32"] - ref).abs().max().item()
    print(f"R50-GeM descriptors vs float64: s3 {e_s3:.3g}  f32 {e_f32:.3g}")
    assert e_s3 < DESC_TOL and e_s3 <= 2.0 * e_f32
