"""The hand-scheduled bf16 filter sweep (csrc/sweep16.hip; rr_set_tuning
sweep_form 1 = 8 waves, 2 = 4 waves) inside the exact prefilter ranker
(iris_evaluate.py:383-386): a different bf16 accumulation order inside the
filter, the same final ranking bit for bit as the exhaustive fp32 ranker
(itself pinned to the oracle in test_gpu_rank.py) -- the prefilter's bound
covers any order and the survivors are rescored exactly.  Shapes cover ragged
gallery tiles (rows past M read as zeros through the buffer descriptor's
range check), ragged query panels (queries past N), one to three k-steps (the
prologue's re-fetches and the odd-step tail), and the C3 shape's d = 2048."""
import numpy as np
import pytest
import torch

import oracle
from research_image_retrieval_amd import ops

pytestmark = pytest.mark.gpu


def _data(nq, n, d, seed, plant=True):
    rs = np.random.RandomState(seed)
    g = rs.standard_normal((n, d)).astype(np.float32)
    q = rs.standard_normal((nq, d)).astype(np.float32)
    if plant:
        g[n // 3], g[n - 1] = q[0], q[nq - 1]  # planted exact matches, one in the last (ragged) tile
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    return q, g


def _prefilter(cuda, q, g, k, form):
    qd, gd = torch.from_numpy(q).to(cuda), torch.from_numpy(g).to(cuda)
    gb, _ = ops.quantize_rows(gd, "bf16")
    bound = ops.prefilter_gallery_bound(gd, gb)
    with ops.tuning(cuda.index, sweep_form=form):
        s, i = ops.cosine_topk_prefilter(qd, gd, gb, bound, k)
    s0, i0 = ops.cosine_topk(qd, gd, k)
    return s, i, s0, i0


@pytest.mark.parametrize("form", [1, 2])
@pytest.mark.parametrize("nq,n,d,k", [(1280, 70_003, 2048, 100), (333, 50_001, 512, 100), (7, 40_000, 96, 50),
                                      (321, 33_000, 64, 100), (5, 41_000, 32, 10)])
def test_sweep16_prefilter_bitexact(cuda, form, nq, n, d, k):
    q, g = _data(nq, n, d, seed=nq + d)
    s, i, s0, i0 = _prefilter(cuda, q, g, k, form)
    assert torch.equal(i, i0) and torch.equal(s.view(torch.int32), s0.view(torch.int32))
    assert int(i[0, 0]) == n // 3 and int(i[nq - 1, 0]) == n - 1


@pytest.mark.parametrize("form", [1, 2])
def test_sweep16_prefilter_vs_oracle_ties(cuda, form):
    """Exact ties across tiles and a dense cluster that sends thousands of
    rows per query through the filter: equal to the oracle bit for bit."""
    rs = np.random.RandomState(5)
    d = 256
    g = rs.standard_normal((60_000, d)).astype(np.float32)
    base = rs.standard_normal(d).astype(np.float32)
    g[40_000:45_000] = base + 0.01 * rs.standard_normal((5000, d)).astype(np.float32)
    g[1000] = g[50_000] = g[59_999] = g[7]
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    q = np.stack([g[7], base / np.linalg.norm(base), rs.standard_normal(d).astype(np.float32)])
    q = (q / np.linalg.norm(q, axis=1, keepdims=True)).astype(np.float32)
    s, i, s0, i0 = _prefilter(cuda, q, g, 300, form)
    assert torch.equal(i, i0) and torch.equal(s.view(torch.int32), s0.view(torch.int32))
    s_o, i_o = oracle.cosine_topk(q, g, 300)
    assert np.array_equal(i.cpu().numpy(), i_o) and np.array_equal(s.cpu().numpy(), s_o)
    assert list(i_o[0, :4]) == [7, 1000, 50_000, 59_999]


@pytest.mark.parametrize("form", [1, 2])
def test_sweep16_lp_bf16_scores(cuda, form):
    """The bf16 ranker (rr_cosine_topk_lp, config C4's) on the new sweep: its
    scores are the bf16 dot products in fp32 (within 1e-5 of a float64 sum of
    the same bf16 operands), its lists sorted and complete against a torch scan
    of those scores."""
    nq, n, d, k = 640, 30_011, 512, 100
    q, g = _data(nq, n, d, seed=3)
    qb, _ = ops.quantize_rows(torch.from_numpy(q).to(cuda), "bf16")
    gb, _ = ops.quantize_rows(torch.from_numpy(g).to(cuda), "bf16")
    with ops.tuning(cuda.index, sweep_form=form):
        s, i = ops.cosine_topk_lp(qb, None, gb, None, k, "bf16")
    qf = qb.view(torch.bfloat16).double()
    gf = gb.view(torch.bfloat16).double()
    ref = qf @ gf.T
    got = torch.gather(ref, 1, i)
    assert (s.double() - got).abs().max().item() < 1e-5
    assert (s[:, :-1] >= s[:, 1:]).all()
    kth = torch.topk(ref, k, dim=1).values[:, -1]
    assert (got[:, -1] >= kth - 2e-5).all()
    assert int(i[0, 0]) == n // 3 and int(i[nq - 1, 0]) == n - 1
