"""GPU parity of the ViT extractor (networks.VisionTransformer on librr)
against the reference's own VisionTransformer outputs (golden fixture) and the
oracle's functional restatement."""
import os
import sys

import numpy as np
import pytest
import torch

from oracle import embed_ref
from research_image_retrieval_amd import ops
from research_image_retrieval_amd.networks import VisionTransformer

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
sys.path.insert(0, GOLD)
import inputs as I  # noqa: E402


@pytest.mark.parametrize("tag", ["tiny", "b16"])
def test_vit_vs_reference_fixture(cuda, tag):
    fx = np.load(os.path.join(GOLD, "vit.npz"))
    res, patch, width, layers, heads, out_dim, seed = (int(v) for v in fx[tag + "_cfg"])
    sd = I.vit_state_dict(seed, width, layers, heads, patch, res, out_dim)
    net = VisionTransformer(res, patch, width, layers, heads, out_dim, state_dict=sd, device=cuda)
    rsx = np.random.RandomState(seed + 100)
    x = torch.from_numpy(rsx.standard_normal((2, 3, res, res)).astype(np.float32))
    got = net(x.to(cuda)).cpu().numpy()
    ref = fx[tag]
    err = np.abs(got - ref).max() / max(1.0, np.abs(ref).max())
    print(tag, "rel max err", err)
    assert err < 1e-5  # measured 1.2e-6 (B/16, fp32 MFMA core vs the reference's torch CPU fp32)
    d = net.forward_test(x.to(cuda)).cpu().numpy()
    np.testing.assert_allclose(np.linalg.norm(d, axis=1), 1.0, rtol=1e-5)


@pytest.mark.parametrize("seq", [17, 197, 256, 40])
def test_attention_kernel_vs_torch(cuda, seq):
    b, heads = 3, 2
    g = torch.Generator().manual_seed(seq)
    qkv = torch.randn(b * seq, 3 * heads * 64, generator=g)
    out = ops.attention(qkv.to(cuda), b, seq, heads).cpu()
    q, k, v = qkv.view(b, seq, 3, heads, 64).permute(2, 0, 3, 1, 4).double()
    ref = torch.softmax(q @ k.transpose(-2, -1) / 8.0, dim=-1) @ v
    ref = ref.permute(0, 2, 1, 3).reshape(b * seq, heads * 64).float()
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)


def test_layernorm_and_quickgelu(cuda):
    x = torch.randn(37, 768)
    w, bb = torch.randn(768), torch.randn(768)
    ref = torch.nn.functional.layer_norm(x.double(), (768,), w.double(), bb.double(), 1e-5).float()
    torch.testing.assert_close(ops.layernorm(x.to(cuda), w.to(cuda), bb.to(cuda)).cpu(), ref, rtol=1e-5, atol=1e-5)
    cls = ops.layernorm(x.to(cuda), w.to(cuda), bb.to(cuda), rows=3, row_stride=12 * 768).cpu()
    torch.testing.assert_close(cls, ref[::12][:3], rtol=1e-5, atol=1e-5)
    a = torch.randn(19, 64)
    wt = torch.randn(96, 64) * 0.1
    b2 = torch.randn(96)
    z = torch.nn.functional.linear(a.double(), wt.double(), b2.double())
    refg = (z * torch.sigmoid(1.702 * z)).float()
    torch.testing.assert_close(ops.linear_ex(a.to(cuda), wt.to(cuda), b2.to(cuda), act=2).cpu(), refg,
                               rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("b,h,w,c,p", [(3, 224, 224, 3, 16), (2, 32, 48, 3, 16), (2, 30, 20, 5, 10),
                                       (1, 16, 16, 4, 4)])
def test_patchify_fp32_and_bf16(cuda, b, h, w, c, p):
    """patchify (vectorised when p*c and w*c are multiples of 4, else scalar)
    against torch's unfold order (kh, kw, c); the bf16 form is bit-identical
    to patchify fp32 + quantize_rows bf16."""
    x = torch.randn(b, h, w, c, generator=torch.Generator().manual_seed(h * w + c))
    ref = x.view(b, h // p, p, w // p, p, c).permute(0, 1, 3, 2, 4, 5).reshape(-1, p * p * c)
    got = ops.patchify(x.to(cuda), p)
    assert torch.equal(got.cpu(), ref)
    got16 = ops.patchify(x.to(cuda), p, out_bf16=True)
    q, _ = ops.quantize_rows(got, "bf16")
    assert got16.dtype == torch.bfloat16 and torch.equal(got16.cpu(), q.cpu())
    assert torch.equal(got16.cpu(), ref.to(torch.bfloat16))


@pytest.mark.parametrize("b,npatch,width", [(3, 196, 768), (2, 49, 512), (2, 16, 384), (1, 5, 200)])
def test_vit_tokens_ln_pre_fused(cuda, b, npatch, width):
    """tokens + ln_pre in one kernel (vectorised for widths 512 / 768, a
    per-lane row loop for other widths): bit-identical to vit_tokens followed
    by layernorm, and within 1e-5 of torch float64."""
    g = torch.Generator().manual_seed(width + npatch)
    pt = torch.randn(b * npatch, width, generator=g)
    cls, pos = torch.randn(width, generator=g), torch.randn(npatch + 1, width, generator=g)
    gm, bt = torch.randn(width, generator=g), torch.randn(width, generator=g)
    d = [t.to(cuda) for t in (pt, cls, pos, gm, bt)]
    plain = ops.vit_tokens(d[0], b, d[1], d[2])
    fused = ops.vit_tokens(d[0], b, d[1], d[2], ln=(d[3], d[4]))
    two = ops.layernorm(plain, d[3], d[4])
    assert torch.equal(fused.cpu(), two.cpu())
    tok = torch.cat([cls.expand(b, 1, width), pt.view(b, npatch, width)], 1) + pos
    assert torch.equal(plain.cpu(), tok.reshape(-1, width))
    ref = torch.nn.functional.layer_norm(tok.double(), (width,), gm.double(), bt.double(), 1e-5).float()
    torch.testing.assert_close(fused.cpu(), ref.reshape(-1, width), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("seq", [197, 50, 256, 31])
def test_attention_bf16_kernel_vs_float64(cuda, seq):
    """bf16-MFMA attention (C4): q/k/v and P rounded to bf16, fp32 softmax.
    Against the float64 attention of the bf16-rounded q/k/v: per-row cosine
    >= 0.9999 and max-abs error <= 1e-2 (P's bf16 rounding is the error)."""
    b, heads, hd = 3, 4, 64
    g = torch.Generator().manual_seed(seq)
    qkv = torch.randn(b * seq, 3 * heads * hd, generator=g)
    out = ops.attention_bf16(qkv.to(cuda), b, seq, heads).float().cpu().double()
    out32 = ops.attention_bf16(qkv.to(cuda), b, seq, heads, bf16_math=False).float().cpu().double()
    x = qkv.bfloat16().double().view(b, seq, 3, heads, hd)
    q, k, v = x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2), x[:, :, 2].transpose(1, 2)
    ref = torch.softmax(q @ k.transpose(-1, -2) / 8.0, -1) @ v
    ref = ref.transpose(1, 2).reshape(b * seq, heads * hd)
    cos = torch.nn.functional.cosine_similarity(out.view(-1, hd), ref.view(-1, hd), dim=1)
    err = (out - ref).abs().max().item()
    print(f"seq {seq}: bf16-math max|err| {err:.3g} min cos {cos.min().item():.6f}; "
          f"fp32-math max|err| {(out32 - ref).abs().max().item():.3g}")
    assert cos.min().item() >= 0.9999 and err <= 1e-2
    # bf16 QKV rows (the QKV linear's bf16 output): bit-identical to the fp32-input kernel
    out16 = ops.attention_bf16(qkv.bfloat16().to(cuda), b, seq, heads).float().cpu().double()
    assert torch.equal(out16, out)


def test_vit_bf16_linear_bf16_qkv_matches_fp32_qkv(cuda):
    """rr_linear_bf16 with bf16 output rounds (acc + bias) RNE, exactly as the
    attention rounds fp32 QKV rows: the fused bf16 path equals the fp32 one."""
    g = torch.Generator().manual_seed(5)
    m, k, n = 2 * 197, 768, 3 * 768
    x = torch.randn(m, k, generator=g).bfloat16().to(cuda)
    w = (torch.randn(n, k, generator=g) / k ** 0.5).bfloat16().to(cuda)
    bias = torch.randn(n, generator=g).to(cuda)
    q32 = ops.linear_bf16(x, w, bias)
    q16 = ops.linear_bf16(x, w, bias, out_bf16=True)
    assert torch.equal(q32.bfloat16(), q16)
    a32 = ops.attention_bf16(q32, 2, 197, 12)
    a16 = ops.attention_bf16(q16, 2, 197, 12)
    assert torch.equal(a32, a16)


def test_ln_partials_and_produce_epilogue(cuda):
    """The LayerNorm fold's producer side: rr_ln_partials_bf16 and the residual
    GEMM's EP_STATS epilogue give per-tile (mean_t, M2) whose Chan combination
    matches float64 LayerNorm statistics and the tile-centred copy
    bf16(y - mean_t) exactly; the GEMM's fp32 output is bit-identical to
    rr_linear_bf16's."""
    g = torch.Generator().manual_seed(3)
    m, k, n = 3 * 197 + 11, 768, 768
    a = (torch.randn(m, k, generator=g)).bfloat16().to(cuda)
    w = (torch.randn(n, k, generator=g) / k ** 0.5).bfloat16().to(cuda)
    bias = torch.randn(n, generator=g).to(cuda)
    r = (torch.randn(m, n, generator=g) * 3 + 0.5).to(cuda)  # a residual stream with a mean offset
    y, yb, st = ops.linear_bf16_ln_produce(a, w, bias, r)
    with ops.tuning(cuda.index, lp_cfg=3):
        y_ref = ops.linear_bf16(a, w, bias, residual=r)
    assert torch.equal(y.view(torch.int32), y_ref.view(torch.int32))
    centred = (y.view(m, n // 256, 256) - st[..., 0:1]).view(m, n)  # the same fp32 subtraction
    assert torch.equal(yb.view(torch.int16), centred.bfloat16().view(torch.int16))
    xb, st2 = ops.ln_partials_bf16(y)
    assert torch.equal(xb.view(torch.int16), yb.view(torch.int16))
    yd = y.double().cpu().view(m, n // 256, 256)
    mt = yd.mean(-1)
    m2 = ((yd - mt[..., None]) ** 2).sum(-1)
    for s in (st, st2):
        s = s.double().cpu()
        assert (s[..., 0] - mt).abs().max() <= 1e-6 * (1 + mt.abs().max())
        assert ((s[..., 1] - m2).abs() / m2).max() <= 1e-5
    torch.testing.assert_close(st, st2, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("act", [0, 2])
def test_linear_bf16_ln_fold_vs_float64(cuda, act):
    """The consumer side: act(LayerNorm(x) W^T + b) with the LayerNorm folded
    into the GEMM epilogue (bf16(x) rows, W o gamma, the row statistics from
    the partials) against float64, next to the unfused LayerNorm -> bf16 ->
    GEMM path: the same error scale (bf16 operand rounding), on rows with a
    mean offset and heavy channels (|x| up to 60x the rest)."""
    g = torch.Generator().manual_seed(4 + act)
    m, k, n = 2 * 197 + 3, 768, 3072 if act else 2304
    x = torch.randn(m, k, generator=g) + 0.7
    x[:, :4] *= 60.0  # a few massive-activation channels, as CLIP residual streams have
    w = torch.randn(n, k, generator=g) / k ** 0.5
    b = torch.randn(n, generator=g) * 0.1
    gam = 1.0 + 0.2 * torch.randn(k, generator=g)
    bet = 0.1 * torch.randn(k, generator=g)
    xd = x.to(cuda)
    xb, st = ops.ln_partials_bf16(xd)
    wf, cs, bf = ops.ln_fold_weights(w.to(cuda), b.to(cuda), gam.to(cuda), bet.to(cuda))
    y_fold = ops.linear_bf16_ln_fold(xb, st, wf, cs, bf, act=act).float().cpu().double()
    y_ln = ops.linear_bf16(ops.layernorm_bf16(xd, gam.to(cuda), bet.to(cuda)), w.bfloat16().to(cuda), b.to(cuda),
                           act=act, out_bf16=True).float().cpu().double()
    ref = torch.nn.functional.layer_norm(x.double(), (k,), gam.double(), bet.double(), 1e-5) @ w.double().t() + b.double()
    if act == 2:
        ref = ref * torch.sigmoid(1.702 * ref)
    e_fold = (y_fold - ref).abs()
    e_ln = (y_ln - ref).abs()
    scale = ref.abs().mean()
    print(f"act {act}: fold max {e_fold.max().item() / scale:.3e} mean {e_fold.mean().item() / scale:.3e} | "
          f"LayerNorm path max {e_ln.max().item() / scale:.3e} mean {e_ln.mean().item() / scale:.3e} (x mean |ref|)")
    # bf16 output rounding alone is 2^-9 relative; the operand roundings add a few times that
    assert e_fold.mean() <= 2.0 * e_ln.mean() + 1e-6
    assert e_fold.max() <= 2.0 * e_ln.max() + 1e-6


@pytest.mark.parametrize("offset", [20.0, -300.0])
def test_linear_bf16_ln_fold_large_mean(cuda, offset):
    """Rows whose mean is far from 0 against their spread (mean 20 and -300
    standard deviations): the tile-centred bf16 rows keep the fold's error at
    the LayerNorm -> bf16 path's scale (uncentred, bf16(x) would round
    2^-9 |x| ~ 2^-9 |mean|, 20-300x that)."""
    g = torch.Generator().manual_seed(11)
    m, k, n = 2 * 197 + 1, 768, 2304
    x = torch.randn(m, k, generator=g) + offset
    x[:, 7] += 5.0  # one heavier channel
    w = torch.randn(n, k, generator=g) / k ** 0.5
    b = torch.randn(n, generator=g) * 0.1
    gam = 1.0 + 0.2 * torch.randn(k, generator=g)
    bet = 0.1 * torch.randn(k, generator=g)
    xd = x.to(cuda)
    xb, st = ops.ln_partials_bf16(xd)
    wf, cs, bf = ops.ln_fold_weights(w.to(cuda), b.to(cuda), gam.to(cuda), bet.to(cuda))
    y_fold = ops.linear_bf16_ln_fold(xb, st, wf, cs, bf).float().cpu().double()
    y_ln = ops.linear_bf16(ops.layernorm_bf16(xd, gam.to(cuda), bet.to(cuda)), w.bfloat16().to(cuda), b.to(cuda),
                           out_bf16=True).float().cpu().double()
    ref = torch.nn.functional.layer_norm(x.double(), (k,), gam.double(), bet.double(), 1e-5) @ w.double().t() + b.double()
    e_fold, e_ln = (y_fold - ref).abs(), (y_ln - ref).abs()
    scale = ref.abs().mean()
    print(f"offset {offset}: fold max {e_fold.max().item() / scale:.3e} mean {e_fold.mean().item() / scale:.3e} | "
          f"LayerNorm path max {e_ln.max().item() / scale:.3e} mean {e_ln.mean().item() / scale:.3e}")
    assert e_fold.mean() <= 2.0 * e_ln.mean() + 1e-6
    assert e_fold.max() <= 2.0 * e_ln.max() + 1e-6


def test_vit_bf16_ln_fold_matches_unfused(cuda):
    """The whole ViT-B/16 bf16 forward with the ln_1 / ln_2 fold against the
    same network with LayerNorm passes: descriptors within the C4 bar of each
    other (cosine >= 0.99999) and of the fp32 oracle (>= 0.9999)."""
    from research_image_retrieval_amd import weights as W
    sd = W.synthetic_vit_state_dict(out_dim=512, seed=0)
    net = VisionTransformer(224, 16, 768, 12, 12, 512, state_dict=sd, device=cuda, dtype="bf16")
    assert net.ln_fold
    rs = np.random.RandomState(7)
    imgs = torch.from_numpy(rs.randint(0, 256, size=(6, 224, 224, 3), dtype=np.uint8))
    d_fold = net.forward_test_u8(imgs.to(cuda)).cpu().double()
    net.ln_fold = False
    d_ln = net.forward_test_u8(imgs.to(cuda)).cpu().double()
    cos = (d_fold * d_ln).sum(1)
    with torch.no_grad():
        ref = torch.cat([torch.nn.functional.normalize(
            embed_ref.vit_forward(embed_ref.normalize_u8(imgs[i:i + 1]), sd, 16, 768, 12, 12), dim=-1)
            for i in range(2)]).double()
    cos_ref = (d_fold[:2] * ref).sum(1)
    print(f"fold vs LayerNorm passes: min cosine {cos.min().item():.8f}; fold vs fp32 oracle {cos_ref.min().item():.8f}")
    assert float(cos.min()) >= 0.99999
    assert float(cos_ref.min()) >= 0.9999


def test_vit_bf16_width1024_takes_layernorm_passes(cuda):
    """a width-1024 bf16 ViT (ViT-L/14's width, 16 heads of 64;
    one block at 112 px to stay small) is past the fold's K <= 768: it runs
    the LayerNorm passes, and its descriptors match the fp32 network's."""
    from research_image_retrieval_amd import weights as W
    sd = W.synthetic_vit_state_dict(width=1024, layers=1, heads=16, res=112, out_dim=256, seed=2)
    net = VisionTransformer(112, 16, 1024, 1, 16, 256, state_dict=sd, device=cuda, dtype="bf16")
    assert not net.ln_fold
    ref = VisionTransformer(112, 16, 1024, 1, 16, 256, state_dict=sd, device=cuda, dtype="fp32")
    imgs = torch.from_numpy(np.random.RandomState(3).randint(0, 256, size=(4, 112, 112, 3), dtype=np.uint8)).to(cuda)
    d16 = net.forward_test_u8(imgs).double()
    d32 = ref.forward_test_u8(imgs).double()
    assert torch.isfinite(d16).all()
    assert float((d16 * d32).sum(1).min()) >= 0.9999


def test_linear_bf16_ln_argument_checks_and_edges(cuda):
    """rr_linear_bf16_ln: exactly one of stats_in / stats_out, the producer's
    n % 256 and residual requirements, the consumer's k % 64 and bf16 output
    (RR_EINVAL otherwise); m = 0 is a no-op; a single row works."""
    import ctypes
    from research_image_retrieval_amd import _lib
    L, h = _lib.lib(), _lib.handle(cuda.index)
    m, k, n = 1, 768, 768
    x = torch.randn(m, k, device=cuda).bfloat16()
    w = (torch.randn(n, k, device=cuda) / k ** 0.5).bfloat16()
    bias = torch.randn(n, device=cuda)
    r = torch.randn(m, n, device=cuda)
    y = torch.empty(m, n, device=cuda)
    yb = torch.empty(m, n, device=cuda, dtype=torch.bfloat16)
    st = torch.empty(m, n // 256, 2, device=cuda)
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    s = torch.cuda.current_stream(cuda).cuda_stream
    # neither / both stats pointers
    assert L.rr_linear_bf16_ln(h, p(x), m, k, p(w), p(bias), n, p(r), 0, 0, p(y), None, None, 0.0, None, None,
                               s) == _lib.RR_EINVAL
    assert L.rr_linear_bf16_ln(h, p(x), m, k, p(w), p(bias), n, p(r), 0, 0, p(y), p(st), p(bias), 1e-5, p(st), p(yb),
                               s) == _lib.RR_EINVAL
    # producer without a residual / with n % 256 != 0
    assert L.rr_linear_bf16_ln(h, p(x), m, k, p(w), p(bias), n, None, 0, 0, p(y), None, None, 0.0, p(st), p(yb),
                               s) == _lib.RR_EINVAL
    assert L.rr_linear_bf16_ln(h, p(x), m, k, p(w), p(bias), 640, p(r), 0, 0, p(y), None, None, 0.0, p(st), p(yb),
                               s) == _lib.RR_EINVAL
    # consumer with fp32 output; with k > 768 (more than three LayerNorm tiles)
    cs = w.float().view(n, 3, 256).sum(-1).t().contiguous()
    x4 = torch.randn(m, 1024, device=cuda).bfloat16()
    w4 = torch.randn(n, 1024, device=cuda).bfloat16()
    st4 = torch.zeros(m, 4, 2, device=cuda)
    cs4 = torch.zeros(4, n, device=cuda)
    assert L.rr_linear_bf16_ln(h, p(x4), m, 1024, p(w4), p(bias), n, None, 0, 1, p(yb), p(st4), p(cs4), 1e-5, None,
                               None, s) == _lib.RR_EINVAL
    # producer with k % 64 != 0
    assert L.rr_linear_bf16_ln(h, p(x[:, :736].contiguous()), m, 736, p(w[:, :736].contiguous()), p(bias), n, p(r), 0,
                               0, p(y), None, None, 0.0, p(st), p(yb), s) == _lib.RR_EINVAL
    assert L.rr_linear_bf16_ln(h, p(x), m, k, p(w), p(bias), n, None, 0, 0, p(y), p(st), p(cs), 1e-5, None, None,
                               s) == _lib.RR_EINVAL
    # m = 0: nothing to do
    assert L.rr_linear_bf16_ln(h, p(x), 0, k, p(w), p(bias), n, p(r), 0, 0, p(y), None, None, 0.0, p(st), p(yb),
                               s) == 0
    # one row, producer then consumer
    y1, yb1, st1 = ops.linear_bf16_ln_produce(x, w, bias, r)
    assert torch.equal(yb1.view(torch.int16), (y1.view(m, 3, 256) - st1[..., 0:1]).view(m, n).bfloat16().view(torch.int16))
    gam, bet = torch.ones(n, device=cuda), torch.zeros(n, device=cuda)
    wf, csum, bf = ops.ln_fold_weights(w.float(), bias, gam, bet)
    out = ops.linear_bf16_ln_fold(yb1, st1, wf, csum, bf).float()
    ref = ops.linear_bf16(ops.layernorm_bf16(y1, gam, bet), w, bias).float()
    assert (out - ref).abs().max().item() <= 0.05 * ref.abs().mean().item()


@pytest.mark.parametrize("kind", ["bf16_out", "residual", "gelu", "produce", "produce_k3072", "fold", "fold_gelu"])
def test_linear_bf16_persistent_tile_bit_identical(cuda, kind):
    """The default for the ViT linears with K <= 1024 (gemm_lpp.hip: the
    256x256 bf16 tile as a persistent k-stream, slab epilogue, residual two
    bands ahead) keeps the one-tile kernel's (lp_cfg 3) fragments,
    per-accumulator MFMA order and epilogue arithmetic: identical bits for
    every ViT linear epilogue, with several tiles per block and a ragged last
    row tile."""
    g = torch.Generator().manual_seed(23)
    n = 2304 if kind in ("bf16_out", "gelu", "fold", "fold_gelu") else 768
    m = 8000 + 37 if n == 2304 else 30001  # > 256 tiles either way
    k = 3072 if kind == "produce_k3072" else 768  # (c_proj's K: the one-tile kernel by default, lp_cfg 6 streams it)
    x = (torch.randn(m, k, generator=g) + 0.3).to(cuda)
    w = (torch.randn(n, k, generator=g) * k ** -0.5).to(cuda)
    bias = (torch.randn(n, generator=g) * 0.1).to(cuda)
    r = torch.randn(m, n, generator=g).to(cuda)
    gam, bet = (1 + 0.1 * torch.randn(k, generator=g)).to(cuda), (0.1 * torch.randn(k, generator=g)).to(cuda)
    xb16, wb16 = x.bfloat16().contiguous(), w.bfloat16().contiguous()

    def run():
        if kind == "bf16_out":
            return (ops.linear_bf16(xb16, wb16, bias, out_bf16=True),)
        if kind == "residual":
            return (ops.linear_bf16(xb16, wb16, bias, residual=r),)
        if kind == "gelu":
            return (ops.linear_bf16(xb16, wb16, bias, act=2, out_bf16=True),)
        if kind in ("produce", "produce_k3072"):
            return ops.linear_bf16_ln_produce(xb16, wb16, bias, r)
        xb, st = ops.ln_partials_bf16(x)
        wf, cs, bf = ops.ln_fold_weights(w, bias, gam, bet)
        return (ops.linear_bf16_ln_fold(xb, st, wf, cs, bf, act=2 if kind == "fold_gelu" else 0),)

    with ops.tuning(0, lp_cfg=3):
        ref = run()
    outs = [run()]
    with ops.tuning(0, lp_cfg=6):  # the three-A-stage form (no-fold flag sets)
        outs.append(run())
    as_int = lambda t: t.view(torch.int16) if t.dtype == torch.bfloat16 else t.view(torch.int32)  # noqa: E731
    for out in outs:
        for a, b in zip(ref, out):
            assert a.shape == b.shape and a.dtype == b.dtype
            assert torch.equal(as_int(a), as_int(b)), kind
