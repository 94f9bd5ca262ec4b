"""rr_bottleneck_seam_h2: block i's conv3 (+ residual, ReLU) and block i+1's
conv1 (+ ReLU) as one f16x2 launch (gemm_seam.hip), against float64 and
against the same two convs as separate rr_conv2d_h2 launches.

The reference chains the blocks of a stage as torchvision Bottlenecks
(networks/backbone.py:60-109) / its own ResBlocks (:305-346):
out = ReLU(conv3(y2) + b3 + x), then the next block's conv1 = ReLU(conv1(out) + b1)."""
import pytest
import torch

from research_image_retrieval_amd import ops

pytestmark = pytest.mark.gpu


def _case(cuda, b, h, w, planes, seed, res_scale=None):
    g = torch.Generator().manual_seed(seed)
    y2 = torch.relu(torch.randn(b, h, w, planes, generator=g))  # a conv2 output (post-ReLU)
    res = torch.relu(torch.randn(b, h, w, 4 * planes, generator=g)) * 2.0
    if res_scale is not None:
        res = res * res_scale
    w3 = torch.randn(4 * planes, 1, 1, planes, generator=g) * (2.0 / planes) ** 0.5
    b3 = torch.randn(4 * planes, generator=g) * 0.1
    w1 = torch.randn(planes, 1, 1, 4 * planes, generator=g) * (2.0 / (4 * planes)) ** 0.5
    b1 = torch.randn(planes, generator=g) * 0.1
    return y2, res, w3, b3, w1, b1


def _run(cuda, y2, res, w3, b3, w1, b1):
    y2d, resd = y2.to(cuda).contiguous(), res.to(cuda).contiguous()
    rec = ops.amax_records(5, cuda)
    ops.amax_f32(y2d, rec[0])
    c3, c1 = ops.H2Conv(w3.to(cuda)), ops.H2Conv(w1.to(cuda))
    out, h1 = ops.bottleneck_seam_h2(y2d, rec[0], resd, c3, b3.to(cuda), c1, b1.to(cuda), rec[1], rec[2])
    return out, h1, rec, (y2d, resd, c3, c1)


def _rel_err(y, ref, scale):
    e = (y.double() - ref).abs() / scale.clamp_min(1e-30)
    return float(e.max()), float(e.mean())


def _f64_conv1x1(x, w, b):
    """x [B,H,W,K], w [N,1,1,K] -> (x w^T + b, |x| |w|^T) in float64."""
    xd, wd = x.double(), w.double().reshape(w.shape[0], -1)
    return xd @ wd.t() + b.double(), xd.abs() @ wd.abs().t()


@pytest.mark.parametrize("b,h,w,planes", [
    (2, 14, 14, 256),   # 392 rows: three full 128-row groups + 8 rows
    (1, 28, 28, 128),   # 784 rows: ragged last group of 16
    (1, 56, 56, 64),    # 3136 rows: half a group at the end
    (1, 3, 5, 256),     # 15 rows: one partial group
])
def test_seam_vs_float64_and_two_launches(cuda, b, h, w, planes):
    y2, res, w3, b3, w1, b1 = _case(cuda, b, h, w, planes, seed=b * h * w + planes)
    out, h1, rec, (y2d, resd, c3, c1) = _run(cuda, y2, res, w3, b3, w1, b1)
    # float64: the block output from the inputs; h1 from the GPU's own output,
    # so each conv's error is measured alone
    ref3, sc3 = _f64_conv1x1(y2, w3, b3)
    ref3 = torch.relu(ref3 + res.double())
    sc3 = sc3 + res.double()
    out_c = out.cpu()
    ref1, sc1 = _f64_conv1x1(out_c, w1, b1)
    ref1 = torch.relu(ref1)
    h1_c = h1.cpu()
    # the exact-fp32 core on the same inputs, for the bar
    e3_f32 = ops.conv2d(y2d, w3.to(cuda), b3.to(cuda), 1, 0, resd, True).cpu()
    e1_f32 = ops.conv2d(out, w1.to(cuda), b1.to(cuda), 1, 0, None, True).cpu()
    live3, live1 = ref3 > 0, ref1 > 0
    es, ef = _rel_err(out_c[live3], ref3[live3], sc3[live3]), _rel_err(e3_f32[live3], ref3[live3], sc3[live3])
    hs, hf = _rel_err(h1_c[live1], ref1[live1], sc1[live1]), _rel_err(e1_f32[live1], ref1[live1], sc1[live1])
    print(f"seam {b}x{h}x{w} P={planes}: out max {es[0]:.3g} mean {es[1]:.3g} (f32 {ef[0]:.3g} / {ef[1]:.3g}); "
          f"h1 max {hs[0]:.3g} mean {hs[1]:.3g} (f32 {hf[0]:.3g} / {hf[1]:.3g})")
    # the f16x2 bar (tests/test_gpu_h2.py): mean <= 1.05x the exact-fp32 core's, max <= 1.25x
    assert es[0] <= 1.25 * max(ef[0], 1e-7) and es[1] <= 1.05 * ef[1] + 1e-9
    assert hs[0] <= 1.25 * max(hf[0], 1e-7) and hs[1] <= 1.05 * hf[1] + 1e-9
    # the records hold exactly max |out| and max |h1|
    assert ops.amax_value(rec[1]) == float(out_c.abs().max())
    assert ops.amax_value(rec[2]) == float(h1_c.abs().max())
    # against the two launches (the library's picks): both outputs to within
    # accumulation-order rounding (the seam's conv3 runs 16x16x32 MFMAs, the
    # two-launch path 32x32x16 or 16x16x32 tiles; the same products)
    ru = ops.amax_records(2, cuda)
    out_u = ops.conv2d_h2(y2d, rec[0], c3, b3.to(cuda), 1, 0, resd, True, ru[0])
    h1_u = ops.conv2d_h2(out_u, ru[0], c1, b1.to(cuda), 1, 0, None, True, ru[1])
    d3 = (out - out_u).abs()
    print(f"  out vs two launches: {int((d3 > 0).sum())} of {d3.numel()} elements differ, max {float(d3.max()):.3g}")
    assert float(d3.max()) <= 2.0 ** -20 * float(out_u.abs().max())
    d = (h1 - h1_u).abs()
    n_diff = int((d > 0).sum())
    print(f"  h1 vs two launches: {n_diff} of {d.numel()} elements differ, max {float(d.max()):.3g}")
    assert float(d.max()) <= 2.0 ** -20 * float(h1_u.abs().max())


def test_seam_running_max_rescale(cuda):
    """The last chunk's block outputs 2^13 larger than the others: conv1's A
    scale drops at that chunk and the accumulator is rescaled exactly; h1
    stays within the f16x2 bar against float64."""
    b, h, w, planes = 2, 14, 14, 256
    y2, res, w3, b3, w1, b1 = _case(cuda, b, h, w, planes, seed=41)
    res[..., 7 * 128:] *= 2.0 ** 13
    out, h1, rec, (y2d, resd, c3, c1) = _run(cuda, y2, res, w3, b3, w1, b1)
    out_c, h1_c = out.cpu(), h1.cpu()
    ref1, sc1 = _f64_conv1x1(out_c, w1, b1)
    ref1 = torch.relu(ref1)
    e1_f32 = ops.conv2d(out, w1.to(cuda), b1.to(cuda), 1, 0, None, True).cpu()
    live = ref1 > 0
    hs, hf = _rel_err(h1_c[live], ref1[live], sc1[live]), _rel_err(e1_f32[live], ref1[live], sc1[live])
    print(f"rescaled: h1 max {hs[0]:.3g} mean {hs[1]:.3g} (f32 {hf[0]:.3g} / {hf[1]:.3g})")
    assert hs[0] <= 1.25 * max(hf[0], 1e-7) and hs[1] <= 1.05 * hf[1] + 1e-9


def test_seam_nonfinite_and_empty(cuda):
    """A NaN conv2 output reaches every block output of its row (NaN, or 0
    where the ReLU's fmaxf(NaN, 0) = 0 took it, as rr_conv2d_h2's epilogue
    does) and so that row's h1, and leaves the other rows as without it (NaN
    stays out of the split scales); m = 0 is a no-op; bad shapes raise."""
    b, h, w, planes = 1, 7, 9, 128
    y2, res, w3, b3, w1, b1 = _case(cuda, b, h, w, planes, seed=5)
    out0, h10, _, _ = _run(cuda, y2, res, w3, b3, w1, b1)
    y2[0, 3, 4, 17] = float("nan")
    out1, h11, _, _ = _run(cuda, y2, res, w3, b3, w1, b1)
    bad = torch.zeros(b, h, w, dtype=torch.bool)
    bad[0, 3, 4] = True
    ob = out1[bad.to(cuda)]
    assert bool((torch.isnan(ob) | (ob == 0)).all()) and not torch.equal(ob, out0[bad.to(cuda)])
    assert not torch.equal(h11[bad.to(cuda)], h10[bad.to(cuda)])
    assert torch.equal(out1[~bad.to(cuda)], out0[~bad.to(cuda)]) and torch.equal(h11[~bad.to(cuda)], h10[~bad.to(cuda)])
    y2e, rese, w3e, b3e, w1e, b1e = _case(cuda, 0, 7, 9, planes, seed=6)
    oute, h1e = ops.bottleneck_seam_h2(y2e.to(cuda), ops.amax_records(1, cuda)[0], rese.to(cuda),
                                       ops.H2Conv(w3e.to(cuda)), None, ops.H2Conv(w1e.to(cuda)), None)
    assert oute.shape == (0, 7, 9, 4 * planes) and h1e.shape == (0, 7, 9, planes)
    with pytest.raises(ValueError):
        ops.bottleneck_seam_h2(y2.to(cuda), ops.amax_records(1, cuda)[0], res[..., :-4].contiguous().to(cuda),
                               ops.H2Conv(w3.to(cuda)), None, ops.H2Conv(w1.to(cuda)), None)
