"""Host-side algebra of the ViT LayerNorm fold (rr_linear_bf16_ln; DESIGN.md
ViT section): the per-256-column-tile partials combined as Chan et al. give
the row's LayerNorm mean and biased variance, and with xc = x centred per
256-column tile t on its mean mean_t,
    LayerNorm(x) W^T + b == rstd (xc (W o gamma)^T + sum_t (mean_t - mean) colsum_t(W o gamma)) + (b + W beta)
holds in float64 (networks/model.py:157-163, 188-190).  ops.ln_fold_weights
is the weight preparation the GPU path uses (its bf16 rounding aside)."""
import numpy as np
import torch

from research_image_retrieval_amd import ops


def _partials(x, tile=256):
    m, d = x.shape
    t = x.reshape(m, d // tile, tile)
    mt = t.mean(-1)
    return mt, ((t - mt[..., None]) ** 2).sum(-1)


def _combine(mt, m2, d, tile=256):
    n = np.minimum(tile, d - tile * np.arange(mt.shape[1]))
    mean = (n * mt).sum(1) / d
    m2_tot = m2.sum(1) + (n * (mt - mean[:, None]) ** 2).sum(1)
    return mean, m2_tot / d


def test_chan_combination_matches_layernorm_statistics():
    rs = np.random.RandomState(0)
    x = rs.standard_normal((37, 768)) * 3 + 5.0
    x[:, :3] *= 80.0
    mean, var = _combine(*_partials(x), 768)
    np.testing.assert_allclose(mean, x.mean(1), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(var, x.var(1), rtol=1e-12)


def test_fold_identity_float64():
    rs = np.random.RandomState(1)
    m, k, n = 19, 768, 96
    x = rs.standard_normal((m, k)) + 0.4
    w = rs.standard_normal((n, k)) / np.sqrt(k)
    b = rs.standard_normal(n)
    gam = 1 + 0.3 * rs.standard_normal(k)
    bet = 0.2 * rs.standard_normal(k)
    eps = 1e-5
    ref = torch.nn.functional.layer_norm(torch.from_numpy(x), (k,), torch.from_numpy(gam), torch.from_numpy(bet),
                                         eps).numpy() @ w.T + b
    mt, m2 = _partials(x)
    mean, var = _combine(mt, m2, k)
    rstd = 1 / np.sqrt(var + eps)
    wf = w * gam[None, :]
    xc = (x.reshape(m, k // 256, 256) - mt[..., None]).reshape(m, k)
    cst = wf.reshape(n, k // 256, 256).sum(-1)  # [n, T]
    got = rstd[:, None] * (xc @ wf.T + (mt - mean[:, None]) @ cst.T) + (b + w @ bet)
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-10)


def test_ln_fold_weights_prep():
    g = torch.Generator().manual_seed(2)
    w = torch.randn(64, 256, generator=g)
    b = torch.randn(64, generator=g)
    gam = 1 + 0.1 * torch.randn(256, generator=g)
    bet = 0.1 * torch.randn(256, generator=g)
    wf, cs, bf = ops.ln_fold_weights(w, b, gam, bet)
    assert wf.dtype == torch.bfloat16 and cs.dtype == torch.float32 and bf.dtype == torch.float32
    assert torch.equal(wf, (w * gam[None, :]).to(torch.bfloat16))
    # colsum per 256-deep k tile [T, N] of the bf16-rounded matrix the GEMM
    # multiplies, not of the fp32 one
    assert cs.shape == (1, 64)
    torch.testing.assert_close(cs[0].double(), wf.double().sum(1), rtol=1e-6, atol=1e-6)
    w2 = torch.randn(8, 640, generator=g)
    _, cs2, _ = ops.ln_fold_weights(w2, torch.zeros(8), torch.ones(640), torch.zeros(640))
    ref2 = torch.stack([w2.bfloat16().double()[:, 256 * t:256 * t + 256].sum(1) for t in range(3)])
    assert cs2.shape == (3, 8)
    torch.testing.assert_close(cs2.double(), ref2, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(bf.double(), b.double() + w.double() @ bet.double(), rtol=1e-6, atol=1e-6)


def test_fold_gate_matches_the_kernel_limit():
    """the network's fold gate and rr_linear_bf16_ln's consumer
    limit agree (LN_TMAX = 3 column-sum tiles of 256 in
    csrc/gemm_epilogue.hpp, rr.h: stats_in needs k <= 768), so a wider bf16
    ViT (ViT-L/14, width 1024, networks/model.py:405) takes the LayerNorm
    passes instead of failing at its first folded GEMM."""
    import os
    import re
    hpp = os.path.join(os.path.dirname(ops.__file__), "csrc", "gemm_epilogue.hpp")
    tmax = int(re.search(r"constexpr int LN_TMAX = (\d+)", open(hpp).read()).group(1))
    assert ops.LN_FOLD_MAX_K == 256 * tmax
    assert ops.ln_fold_supported(768, "bf16") and ops.ln_fold_supported(512, "bf16")
    assert not ops.ln_fold_supported(1024, "bf16")  # ViT-L/14
    assert not ops.ln_fold_supported(640, "bf16")   # not 256-column tiles
    assert not ops.ln_fold_supported(768, "fp32")
