"""The C3 ranker at BASELINE.json's full size (1.6 M x 2048 gallery, top-100):
size-independent properties plus an oracle check on sampled queries.

Reference: iris_evaluate.py:383 (torch.mm of query and gallery descriptors)
and :386 (np.argsort, here with the stable tie-break).
The smaller parity cases live in test_gpu_rank.py; here the sizes are the
bench's, so the checks are the ones that do not need a full CPU ranking:
  * the bf16 prefilter ranker equals the exhaustive fp32 ranker bit for bit;
  * lists are sorted (score desc, index asc), unique and in range;
  * planted exact ties across the seed boundary come out in index order;
  * returned scores equal an independent fp32 recomputation within 1e-5
    (north_star's score tolerance) and no unreturned row beats the k-th
    score by more than 1e-5 (completeness against a torch fp32 scan);
  * an 8-way contiguous row sharding (the 8-GPU layout) merged by
    rr_topk_merge equals the single-gallery result bit for bit;
  * two queries equal the C oracle (oracle/cosine_topk.c) bit for bit.
"""
import numpy as np
import pytest
import torch

import oracle
from research_image_retrieval_amd import ops

pytestmark = pytest.mark.gpu

N, D, K, NQ = 1_600_000, 2048, 100, 64
TIE_SRC, TIE_ROWS = 1_234_567, (5, 1_234_567, 1_599_999)  # row 5 lies inside the 32 768-row seed sample


@pytest.fixture(scope="module")
def full(cuda):
    gen = torch.Generator(device=cuda).manual_seed(2024)
    g = torch.randn(N, D, device=cuda, generator=gen)
    g = torch.nn.functional.normalize(g, dim=1)
    q = torch.nn.functional.normalize(torch.randn(NQ, D, device=cuda, generator=gen), dim=1)
    for r in TIE_ROWS:
        g[r] = g[TIE_SRC]
    q[0] = g[TIE_SRC]
    q[1] = torch.nn.functional.normalize(g[777_777] + 0.05 * torch.randn(D, device=cuda, generator=gen), dim=0)
    g = g.contiguous()
    q = q.contiguous()
    gb, _ = ops.quantize_rows(g, "bf16")
    bound = ops.prefilter_gallery_bound(g, gb)
    s_p, i_p = ops.cosine_topk_prefilter(q, g, gb, bound, K)
    torch.cuda.synchronize()
    yield dict(q=q, g=g, gb=gb, s=s_p, i=i_p)
    del g, gb
    torch.cuda.empty_cache()


def test_fullsize_prefilter_equals_exhaustive(full):
    s0, i0 = ops.cosine_topk(full["q"], full["g"], K)
    assert torch.equal(full["i"], i0)
    assert torch.equal(full["s"].view(torch.int32), s0.view(torch.int32))


def test_fullsize_sorted_unique_ties(full):
    s, i = full["s"].cpu().numpy(), full["i"].cpu().numpy()
    assert ((i >= 0) & (i < N)).all()
    assert all(len(set(r)) == K for r in i)
    ds = np.diff(s, axis=1)
    assert (ds <= 0).all()
    tie = ds == 0
    assert (np.diff(i, axis=1)[tie] > 0).all()  # equal scores: ascending index
    assert list(i[0, :3]) == list(TIE_ROWS) and s[0, 0] == s[0, 1] == s[0, 2]
    assert i[1, 0] == 777_777


def test_fullsize_scores_and_completeness(full):
    q, g, s, i = full["q"], full["g"], full["s"], full["i"]
    rec = (q[:, None, :] * g[i]).sum(-1)  # independent fp32 recomputation
    assert (rec - s).abs().max().item() <= 1e-5
    for lo in range(0, NQ, 16):  # torch fp32 scan, 16 queries at a time
        sc = q[lo:lo + 16] @ g.t()
        sc.scatter_(1, i[lo:lo + 16], float("-inf"))
        kth = s[lo:lo + 16, -1:]
        assert int((sc > kth + 1e-5).sum().item()) == 0


def test_fullsize_eight_shards_merge(full):
    q, g, gb = full["q"], full["g"], full["gb"]
    bounds = np.linspace(0, N, 9).astype(np.int64)
    ps, pi = [], []
    for r in range(8):
        lo, hi = int(bounds[r]), int(bounds[r + 1])
        shard, shard_b = g[lo:hi], gb[lo:hi]
        s, i = ops.cosine_topk_prefilter(q, shard, shard_b, ops.prefilter_gallery_bound(shard, shard_b), K,
                                         idx_offset=lo)
        ps.append(s)
        pi.append(i)
    sm, im = ops.topk_merge(torch.stack(ps).contiguous(), torch.stack(pi).contiguous(), K)
    assert torch.equal(im, full["i"])
    assert torch.equal(sm.view(torch.int32), full["s"].view(torch.int32))


def test_fullsize_two_queries_vs_oracle(full):
    g_host = full["g"].cpu().numpy()
    q_host = full["q"][:2].cpu().numpy()
    s_o, i_o = oracle.cosine_topk(q_host, g_host, K)
    assert np.array_equal(full["i"][:2].cpu().numpy(), i_o)
    assert np.array_equal(full["s"][:2].cpu().numpy(), s_o)
