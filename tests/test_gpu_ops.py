"""GPU parity of the embed-path kernels against torch-CPU fp32 references of
the same ops (conv+BN-folded bias+residual+ReLU, max-pool, GeM, Linear,
F.normalize, ToTensor+Normalize)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from research_image_retrieval_amd import ops

pytestmark = pytest.mark.gpu


def _conv_ref(x_nhwc, w_okkc, b, stride, pad, res=None, relu=False):
    x = x_nhwc.permute(0, 3, 1, 2)
    w = w_okkc.permute(0, 3, 1, 2)
    y = F.conv2d(x.double(), w.double(), b.double() if b is not None else None, stride=stride, padding=pad)
    y = y.permute(0, 2, 3, 1)
    if res is not None:
        y = y + res.double()
    if relu:
        y = y.clamp_min(0)
    return y.float()


@pytest.mark.parametrize("b,h,w,cin,cout,k,s,p,res,relu", [
    (2, 14, 14, 64, 64, 3, 1, 1, False, True),
    (2, 15, 13, 128, 256, 3, 2, 1, False, True),
    (3, 7, 7, 512, 2048, 1, 1, 0, True, True),
    (2, 16, 16, 256, 512, 1, 2, 0, False, False),
    (2, 33, 35, 3, 64, 7, 2, 3, False, True),     # stem (generic gather)
    (2, 33, 35, 4, 64, 7, 2, 3, False, True),     # stem on NHWC4 (one tap per float4)
    (3, 224, 224, 4, 64, 7, 2, 3, False, True),   # full-size stem
    (1, 9, 9, 64, 96, 1, 1, 0, False, False),
])
def test_conv2d(cuda, b, h, w, cin, cout, k, s, p, res, relu):
    g = torch.Generator().manual_seed(b * 1000 + cin)
    x = torch.randn(b, h, w, cin, generator=g)
    wt = torch.randn(cout, k, k, cin, generator=g) * (2.0 / (k * k * cin)) ** 0.5
    bias = torch.randn(cout, generator=g)
    oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    r = torch.randn(b, oh, ow, cout, generator=g) if res else None
    ref = _conv_ref(x, wt, bias, s, p, r, relu)
    out = ops.conv2d(x.to(cuda), wt.to(cuda), bias.to(cuda), s, p, r.to(cuda) if r is not None else None, relu).cpu()
    err = (out - ref).abs().max().item()
    assert err < 1e-4 * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize("shape,k,s,p", [((2, 17, 19, 64), 3, 2, 1), ((3, 112, 112, 64), 3, 2, 1),
                                         ((1, 1, 1, 4), 3, 2, 1), ((2, 2, 3, 8), 3, 2, 1), ((1, 6, 5, 12), 3, 2, 1),
                                         ((2, 9, 7, 8), 2, 2, 0), ((1, 5, 6, 4), 3, 1, 1)])
def test_maxpool(cuda, shape, k, s, p):
    """The 2x2-blocked 3x3/2 kernel (odd and even output sizes, 1x1 input)
    and the row-blocked kernel == torch max_pool2d."""
    x = torch.randn(*shape)
    ref = F.max_pool2d(x.permute(0, 3, 1, 2), k, s, p).permute(0, 2, 3, 1)
    out = ops.maxpool2d(x.to(cuda), k, s, p).cpu()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("p", [3.0, 2.5])
def test_gem(cuda, p):
    x = torch.randn(3, 7, 7, 2048)
    ref = F.avg_pool2d(x.permute(0, 3, 1, 2).clamp(min=1e-6).pow(p), (7, 7)).pow(1.0 / p).flatten(1)
    out = ops.gem_pool(x.to(cuda), p, 1e-6).cpu()
    torch.testing.assert_close(out, ref, rtol=2e-6, atol=1e-7)


def test_linear_and_l2(cuda):
    x = torch.randn(19, 2048)
    w = torch.randn(512, 2048) * 0.02
    b = torch.randn(512)
    ref = F.normalize(F.linear(x.double(), w.double(), b.double()).float(), dim=-1)
    y = ops.linear(x.to(cuda), w.to(cuda), b.to(cuda))
    out = ops.l2_normalize(y).cpu()
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-6)


def test_preprocess_bitexact(cuda):
    rng = np.random.RandomState(1234)
    img = rng.randint(0, 256, size=(2, 31, 29, 3), dtype=np.uint8)
    t = torch.from_numpy(img)
    mean = torch.tensor([0.485, 0.456, 0.406])
    std = torch.tensor([0.229, 0.224, 0.225])
    ref = (t.float().div(255) - mean) / std          # ToTensor + Normalize (HWC view)
    out = ops.preprocess_u8(t.to(cuda)).cpu()
    assert torch.equal(out, ref)


def test_nchw_to_nhwc(cuda):
    x = torch.randn(2, 3, 11, 13)
    assert torch.equal(ops.nchw_to_nhwc(x.to(cuda)).cpu(), x.permute(0, 2, 3, 1))
    y4 = ops.nchw_to_nhwc(x.to(cuda), out_c=4).cpu()
    assert torch.equal(y4[..., :3], x.permute(0, 2, 3, 1)) and (y4[..., 3] == 0).all()


def test_preprocess_pad4(cuda):
    rng = np.random.RandomState(7)
    t = torch.from_numpy(rng.randint(0, 256, size=(2, 9, 7, 3), dtype=np.uint8)).to(cuda)
    a = ops.preprocess_u8(t).cpu()
    b = ops.preprocess_u8(t, out_c=4).cpu()
    assert torch.equal(b[..., :3], a) and (b[..., 3] == 0).all()


def test_maxpool_scalar_path(cuda):
    x = torch.randn(2, 9, 8, 6)  # C % 4 != 0 -> scalar kernel
    ref = F.max_pool2d(x.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    assert torch.equal(ops.maxpool2d(x.to(cuda), 3, 2, 1).cpu(), ref)


def test_handle_device_and_tuning_validation(cuda):
    """rr_get_device reports the handle's device; rr_set_tuning rejects unknown
    keys and out-of-range values (RR_EINVAL, message set) and accepts 0."""
    import ctypes
    from research_image_retrieval_amd import _lib
    L, h = _lib.lib(), _lib.handle(cuda.index)
    d = ctypes.c_int(-1)
    assert L.rr_get_device(h, ctypes.byref(d)) == 0 and d.value == cuda.index
    assert L.rr_set_tuning(h, 99, 1) == _lib.RR_EINVAL and b"unknown key" in L.rr_last_error(h)
    assert L.rr_set_tuning(h, _lib.TUNE_GEMM_CFG, 23) == _lib.RR_EINVAL
    assert L.rr_set_tuning(h, _lib.TUNE_S3_CFG, 16) == _lib.RR_EINVAL
    for retired in (6, 7, 12):  # sweep_order, sweep_pf, lp_il (ABI 5)
        assert L.rr_set_tuning(h, retired, 0) == _lib.RR_EINVAL and b"unknown key" in L.rr_last_error(h)
    assert L.rr_set_tuning(h, _lib.TUNE_LP_CFG, 7) == _lib.RR_EINVAL
    assert L.rr_set_tuning(h, _lib.TUNE_SWEEP_MF16, 2) == _lib.RR_EINVAL
    assert L.rr_set_tuning(h, _lib.TUNE_SWEEP_IL, 2) == _lib.RR_EINVAL
    assert L.rr_set_tuning(h, _lib.TUNE_CONV_IL, 2) == _lib.RR_EINVAL
    assert L.rr_set_tuning(h, _lib.TUNE_HALO_MF, 5) == _lib.RR_EINVAL  # (2-4: the N = 64 / 128 forms, round 6)
    assert L.rr_set_tuning(h, _lib.TUNE_SWEEP_FORM, 3) == _lib.RR_EINVAL
    assert L.rr_set_tuning(h, _lib.TUNE_HALO_2D, 2) == _lib.RR_EINVAL
    assert L.rr_set_tuning(h, _lib.TUNE_S3_CFG_RES, 16) == _lib.RR_EINVAL
    for key in (_lib.TUNE_GEMM_CFG, _lib.TUNE_GEMM_BK, _lib.TUNE_LP_CFG, _lib.TUNE_S3_CFG, _lib.TUNE_SWEEP_MF16,
                _lib.TUNE_SWEEP_IL, _lib.TUNE_CONV_IL, _lib.TUNE_HALO_MF, _lib.TUNE_S3_CFG_RES, _lib.TUNE_HALO_2D):
        assert L.rr_set_tuning(h, key, 0) == 0
    for key in (_lib.TUNE_S3_STAGGER, _lib.TUNE_SWEEP_MF16, _lib.TUNE_SWEEP_IL, _lib.TUNE_CONV_IL,
                _lib.TUNE_HALO_MF, _lib.TUNE_HALO_2D):
        assert L.rr_set_tuning(h, key, -1) == 0
    # a call made while another device is current still runs on the handle's device
    # (one-GPU box: the guard is exercised with the current device equal to the handle's)
    torch.cuda.set_device(cuda)
    x = torch.randn(64, 128, device=cuda)
    y = ops.l2_normalize(x)
    assert torch.allclose(y.norm(dim=1), torch.ones(64, device=cuda), atol=1e-6)
