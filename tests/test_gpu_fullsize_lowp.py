"""C4 / C5 rankers at the bench's full size: 1280 queries against a 1.6 M-row
gallery, bf16 d = 512 (C4) and fp8 d = 2048 (C5, block-scaled MFMA).

Reference: iris_evaluate.py:383-386 (cosine GEMM + ranking); the reduced-
precision gallery is this build's C4/C5 configuration (BASELINE.json configs),
so the oracle is the same contraction on the dequantised rows:
  * returned scores == fp32 dot products of the dequantised rows (rtol 1e-4,
    atol 1e-5, as test_gpu_lowp.py);
  * lists descending and unique; no unreturned row beats the k-th returned
    score by more than 1e-5 (torch scan of 64 sampled queries);
  * an 8-way contiguous sharding merged by rr_topk_merge matches the
    single-gallery lists (scores within 1e-5, index sets >= 99.9 % equal:
    only exact-tie ordering may differ if the shard picks another tile).
"""
import pytest
import torch

from research_image_retrieval_amd import ops

pytestmark = pytest.mark.gpu

N, NQ, K = 1_600_000, 1280, 100


def _rows(sc, lo, hi):
    return None if sc is None else sc[lo:hi]


def _dequant(x, sc, dtype):
    if dtype == "bf16":
        return x.float()
    return x.view(torch.float8_e4m3fn).float() * sc[:, None]


@pytest.mark.parametrize("dtype,d", [("bf16", 512), ("fp8", 2048)])
def test_fullsize_lowp_ranker(cuda, dtype, d):
    gen = torch.Generator(device=cuda).manual_seed(7 + d)
    gl = torch.empty((N, d), dtype=torch.bfloat16 if dtype == "bf16" else torch.uint8, device=cuda)
    gs = torch.empty(N, dtype=torch.float32, device=cuda) if dtype == "fp8" else None
    for lo in range(0, N, 200_000):  # quantise in slices: the fp32 gallery never exists whole
        part = torch.nn.functional.normalize(torch.randn(200_000, d, device=cuda, generator=gen), dim=1)
        ql_, qs_ = ops.quantize_rows(part, dtype)
        gl[lo:lo + 200_000] = ql_
        if gs is not None:
            gs[lo:lo + 200_000] = qs_
    q = torch.nn.functional.normalize(torch.randn(NQ, d, device=cuda, generator=gen), dim=1)
    ql, qs = ops.quantize_rows(q, dtype)
    s, i = ops.cosine_topk_lp(ql, qs, gl, gs, K, dtype)

    assert bool(((i >= 0) & (i < N)).all())
    assert bool((s[:, :-1] >= s[:, 1:]).all())
    srt = torch.sort(i, dim=1).values
    assert bool((srt[:, 1:] != srt[:, :-1]).all())

    qd = _dequant(ql, qs, dtype)
    sel = torch.arange(0, NQ, NQ // 64, device=cuda)[:64]
    ref = torch.empty((64, N), dtype=torch.float32, device=cuda)
    for lo in range(0, N, 200_000):
        ref[:, lo:lo + 200_000] = qd[sel] @ _dequant(gl[lo:lo + 200_000], _rows(gs, lo, lo + 200_000), dtype).t()
    got = torch.gather(ref, 1, i[sel])
    torch.testing.assert_close(s[sel], got, rtol=1e-4, atol=1e-5)
    ref.scatter_(1, i[sel], float("-inf"))
    assert int((ref > s[sel, -1:] + 1e-5).sum().item()) == 0
    del ref

    ps, pi = [], []
    for r in range(8):
        lo, hi = r * N // 8, (r + 1) * N // 8
        a, b = ops.cosine_topk_lp(ql, qs, gl[lo:hi], _rows(gs, lo, hi), K, dtype, idx_offset=lo)
        ps.append(a)
        pi.append(b)
    sm, im = ops.topk_merge(torch.stack(ps).contiguous(), torch.stack(pi).contiguous(), K)
    torch.testing.assert_close(sm, s, rtol=0, atol=1e-5)
    same = sum(len(set(a.tolist()) & set(b.tolist())) for a, b in zip(im.cpu(), i.cpu()))
    assert same >= 0.999 * NQ * K
