"""GPU parity of the ranker (rr_cosine_topk / rr_cosine_scores / rr_topk_merge)
against the C oracle (oracle/cosine_topk.c): bit-exact scores and indices.

Reference: iris_evaluate.py:383 torch.mm + :386 np.argsort (stable tie-break)."""
import numpy as np
import pytest
import torch

import oracle
from research_image_retrieval_amd import ops

pytestmark = pytest.mark.gpu


def _normed(rng, n, d):
    x = rng.randn(n, d).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    return x


def test_mfma_chain_order_bitexact(cuda):
    rng = np.random.RandomState(1)
    q = _normed(rng, 37, 96)
    g = _normed(rng, 1000, 96)
    gpu = ops.cosine_scores(torch.from_numpy(q).to(cuda), torch.from_numpy(g).to(cuda)).cpu().numpy().T
    res = {o: int((oracle.cosine_scores(q, g, order=o) != gpu).sum()) for o in (0, 1, 2)}
    print("mismatches by oracle order:", res)
    assert res[0] == 0, res


@pytest.mark.parametrize("nq,n,d,k", [(16, 20000, 512, 100), (8, 50000, 2048, 100), (3, 40000, 512, 7),
                                      (70, 4993, 512, 4993), (5, 60, 64, 100), (130, 33000, 128, 1)])
def test_cosine_topk_matches_oracle(cuda, nq, n, d, k):
    rng = np.random.RandomState(nq * 7 + n)
    q = _normed(rng, nq, d)
    g = _normed(rng, n, d)
    # plant near-duplicates and exact ties (same row repeated)
    for i in range(min(nq, 4)):
        j = rng.randint(n)
        g[j] = q[i]
        if n > 10:
            g[(j + 3) % n] = q[i]
    s_gpu, i_gpu = ops.cosine_topk(torch.from_numpy(q).to(cuda), torch.from_numpy(g).to(cuda), k)
    s_ref, i_ref = oracle.cosine_topk(q, g, k)
    np.testing.assert_array_equal(i_gpu.cpu().numpy(), i_ref)
    np.testing.assert_array_equal(s_gpu.cpu().numpy(), s_ref)


def test_cosine_topk_idx_offset_and_empty(cuda):
    rng = np.random.RandomState(3)
    q = torch.from_numpy(_normed(rng, 4, 64)).to(cuda)
    g = torch.from_numpy(_normed(rng, 300, 64)).to(cuda)
    s, i = ops.cosine_topk(q, g, 10, idx_offset=1_000_000)
    s2, i2 = ops.cosine_topk(q, g, 10)
    assert torch.equal(i, i2 + 1_000_000) and torch.equal(s, s2)
    s3, i3 = ops.cosine_topk(q, g[:0], 5)
    assert (i3 == -1).all() and torch.isinf(s3).all()


def test_topk_merge_matches_oracle(cuda):
    rng = np.random.RandomState(5)
    P, nq, kin, kout = 8, 33, 100, 100
    ps = rng.randn(P, nq, kin).astype(np.float32)
    pi = rng.permutation(P * nq * kin).reshape(P, nq, kin).astype(np.int64)
    ps[1, :, :5] = ps[0, :, :5]  # cross-part exact ties
    pi[2, :, -10:] = -1          # padding
    so, io = ops.topk_merge(torch.from_numpy(ps).to(cuda), torch.from_numpy(pi).to(cuda), kout)
    sr, ir = oracle.topk_merge(ps, pi, kout)
    np.testing.assert_array_equal(io.cpu().numpy(), ir)
    np.testing.assert_array_equal(so.cpu().numpy(), sr)


def test_alpha_qe_vs_oracle(cuda):
    from research_image_retrieval_amd.search import GallerySearcher, alpha_qe_search
    rng = np.random.RandomState(9)
    q = _normed(rng, 12, 256)
    g = _normed(rng, 20000, 256)
    srch = GallerySearcher(g, device=cuda, normalize=False)
    s, i = srch.topk(q, 10, normalize=False)
    q2 = ops.alpha_qe(torch.from_numpy(q).to(cuda), srch.gallery, i, s, n=3, alpha=3.0).cpu().numpy()
    q2_ref = oracle.alpha_qe(q, g, i.cpu().numpy(), s.cpu().numpy(), n=3, alpha=3.0)
    np.testing.assert_allclose(q2, q2_ref, rtol=0, atol=2e-6)
    s2, i2, _ = alpha_qe_search(srch, q, k=10, n=3, alpha=3.0, normalize=False)
    s2r, i2r = oracle.cosine_topk(q2, g, 10)
    assert (i2.cpu().numpy() == i2r).mean() > 0.99  # q2 differs from the oracle's by <= 2e-6


def test_descriptor_store_to_hbm_and_search(cuda, tmp_path):
    """Gallery streamed from the on-disk store (pinned double buffer, side
    stream) equals the source rows bit for bit and ranks like the oracle."""
    from research_image_retrieval_amd import store as S
    rs = np.random.RandomState(77)
    g = rs.standard_normal((70_001, 128)).astype(np.float32)
    q = rs.standard_normal((9, 128)).astype(np.float32)
    st = S.write_store(str(tmp_path / "g"), g, shard_rows=20_000)
    dev_g = st.to_device(0, st.n, cuda, chunk_rows=8192)
    assert torch.equal(dev_g.cpu(), torch.from_numpy(g))
    part, lo = S.load_gallery_shard(st, 1, 3, cuda)
    assert torch.equal(part.cpu(), torch.from_numpy(g[lo:lo + part.shape[0]]))
    s, i = ops.cosine_topk(torch.from_numpy(q).to(cuda), dev_g, 50)
    s_o, i_o = oracle.cosine_topk(q, g, 50)
    assert np.array_equal(i.cpu().numpy(), i_o) and np.array_equal(s.cpu().numpy(), s_o)


def _prefilter_vs_exhaustive(cuda, q, g, k, idx_offset=0):
    qd = torch.from_numpy(q).to(cuda)
    gd = torch.from_numpy(g).to(cuda)
    gb, _ = ops.quantize_rows(gd, "bf16")
    bound = ops.prefilter_gallery_bound(gd, gb)
    s1, i1 = ops.cosine_topk_prefilter(qd, gd, gb, bound, k, idx_offset=idx_offset)
    s0, i0 = ops.cosine_topk(qd, gd, k, idx_offset=idx_offset)
    assert torch.equal(i1, i0)
    assert torch.equal(s1.view(torch.int32), s0.view(torch.int32))  # bit-identical scores
    return s1.cpu().numpy(), i1.cpu().numpy()


@pytest.mark.parametrize("nq,n,d,k", [(64, 100_000, 512, 100), (7, 50_000, 2048, 100), (33, 40_000, 128, 1000),
                                      (5, 60, 64, 100), (3, 70_001, 24, 1)])
def test_prefilter_bitexact_random(cuda, nq, n, d, k):
    """bf16-bound prefilter + exact rescoring == exhaustive fp32 ranker, bit
    for bit (scores and indices), incl. n < k and d not a multiple of 16."""
    rs = np.random.RandomState(n + d)
    q = rs.standard_normal((nq, d)).astype(np.float32)
    g = rs.standard_normal((n, d)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    s, i = _prefilter_vs_exhaustive(cuda, q, g, k, idx_offset=123)
    s_o, i_o = oracle.cosine_topk(q, g, k, idx_offset=123)
    assert np.array_equal(i, i_o) and np.array_equal(s, s_o)


@pytest.mark.parametrize("nq", [256, 768])
def test_prefilter_query_panels_of_256(cuda, nq):
    """Query counts that tile into 256-wide panels send the bf16 sweep to the
    8-phase 256x256 pipeline (gemm_8p.hip) by default: still bit-identical to
    the exhaustive fp32 ranker (itself oracle-pinned above)."""
    rs = np.random.RandomState(nq)
    d = 2048
    g = rs.standard_normal((120_000, d)).astype(np.float32)
    q = rs.standard_normal((nq, d)).astype(np.float32)
    g[77_777] = q[3]  # a planted exact match
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    s, i = _prefilter_vs_exhaustive(cuda, q, g, 100)
    assert i[3, 0] == 77_777


def test_prefilter_bitexact_ties_and_clusters(cuda):
    """Exact ties (duplicate rows on both sides of the seed boundary), planted
    near-duplicates, and a dense cluster where thousands of rows score within
    the bf16 bound of the k-th best (every one must be rescored)."""
    rs = np.random.RandomState(5)
    d = 256
    g = rs.standard_normal((80_000, d)).astype(np.float32)
    base = rs.standard_normal(d).astype(np.float32)
    g[40_000:45_000] = base + 0.01 * rs.standard_normal((5000, d)).astype(np.float32)  # cluster
    g[1000] = g[50_000] = g[79_999] = g[7]  # exact ties across the seed boundary
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    q = np.stack([g[7], base / np.linalg.norm(base), g[60_000] + 1e-4 * rs.standard_normal(d).astype(np.float32),
                  rs.standard_normal(d).astype(np.float32)])
    q = (q / np.linalg.norm(q, axis=1, keepdims=True)).astype(np.float32)
    s, i = _prefilter_vs_exhaustive(cuda, q, g, 300)
    assert list(i[0, :4]) == [7, 1000, 50_000, 79_999]
    s_o, i_o = oracle.cosine_topk(q, g, 300)
    assert np.array_equal(i, i_o) and np.array_equal(s, s_o)


def test_prefilter_unnormalised_rows(cuda):
    """The bound uses the gallery's row-norm maxima: rows of very different
    norms (not unit) still rank exactly."""
    rs = np.random.RandomState(9)
    g = (rs.standard_normal((30_000, 64)) * rs.uniform(0.01, 3.0, size=(30_000, 1))).astype(np.float32)
    q = (rs.standard_normal((11, 64)) * 2.5).astype(np.float32)
    _prefilter_vs_exhaustive(cuda, q, g, 50)


@pytest.mark.parametrize("ranker", ["exhaustive", "prefilter"])
def test_nan_rows_and_queries_rank_last(cuda, ranker):
    """NaN descriptors (extract_vectors yields them when every scale is dropped,
    utils/helpfunc.py:39-44) rank after every number, by index, as
    np.argsort(-similarity, kind="stable") places them (iris_evaluate.py:386):
    NaN gallery rows inside and outside the threshold-seeding sample, a NaN
    query (all scores NaN: indices 0..k-1), and k > #finite rows."""
    rs = np.random.RandomState(17)
    n, d = 20000, 128
    g = rs.standard_normal((n, d)).astype(np.float32)
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    q = rs.standard_normal((6, d)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    g[5] = np.nan           # inside the seed sample (first 4096 rows)
    g[15000, 7] = np.nan    # outside it
    g[16000] = g[5]
    q[4] = np.nan           # a NaN query
    for gal, k in ((g, 100), (g[:40].copy(), 60)):
        sim = oracle.cosine_scores(q, gal)
        order = oracle.argsort_stable_desc(sim)[:, :k]
        qd, gd = torch.from_numpy(q).to(cuda), torch.from_numpy(gal).to(cuda)
        if ranker == "exhaustive":
            s, i = ops.cosine_topk(qd, gd, k)
        else:
            gb, _ = ops.quantize_rows(gd, "bf16")
            s, i = ops.cosine_topk_prefilter(qd, gd, gb, ops.prefilter_gallery_bound(gd, gb), k)
        s, i = s.cpu().numpy(), i.cpu().numpy()
        kk = min(k, gal.shape[0])
        assert np.array_equal(i[:, :kk], order[:, :kk]), np.argwhere(i[:, :kk] != order[:, :kk])[:5]
        ref_s = np.take_along_axis(sim, order[:, :kk], 1)
        assert np.array_equal(np.isnan(s[:, :kk]), np.isnan(ref_s))
        fin = ~np.isnan(ref_s)
        assert np.array_equal(s[:, :kk][fin], ref_s[fin])
        assert (i[:, kk:] == -1).all() and np.isneginf(s[:, kk:]).all()
        assert list(i[4, :kk]) == list(range(kk))  # the NaN query: every score NaN -> index order


def test_alpha_qe_skips_padding_and_foreign_indices(cuda):
    """rr_alpha_qe reads only local rows [idx_offset, idx_offset + n_rows):
    padding (-1) and indices of another shard contribute nothing."""
    rs = np.random.RandomState(5)
    q = rs.standard_normal((3, 64)).astype(np.float32)
    g = rs.standard_normal((50, 64)).astype(np.float32)
    idx = np.array([[100, 101], [100, -1], [100, 150 + 7]], dtype=np.int64)  # local rows 100..149
    sc = np.array([[0.9, 0.5], [0.7, -np.inf], [0.8, 0.6]], dtype=np.float32)
    out = ops.alpha_qe(torch.from_numpy(q).to(cuda), torch.from_numpy(g).to(cuda), torch.from_numpy(idx).to(cuda),
                       torch.from_numpy(sc).to(cuda), n=2, alpha=3.0, idx_offset=100).cpu().numpy()
    keep = np.where((idx >= 100) & (idx < 150), idx, -1)
    ref = oracle.alpha_qe(q, g, keep, sc, n=2, alpha=3.0, idx_offset=100)
    np.testing.assert_allclose(out, ref, rtol=0, atol=2e-6)


def test_bounded_workspace_overflow_recovery(cuda):
    """Bounded candidate buffers (rr.h): with room for 2000 candidates per
    query, a query facing a 30k-row cluster overflows (counted in the
    workspace's overflow int, its raw row wrong); the ops wrappers re-run it
    and every ranker's output equals the worst-case-workspace run bit for bit."""
    from research_image_retrieval_amd import _lib
    rs = np.random.RandomState(3)
    n, d, k = 60_000, 256, 100
    g = rs.standard_normal((n, d)).astype(np.float32)
    base = rs.standard_normal(d).astype(np.float32)
    g[20_000:50_000] = base + 0.05 * rs.standard_normal((30_000, d)).astype(np.float32)  # past the seed rows
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    rq = rs.standard_normal((5, d)).astype(np.float32)
    bh = base / np.linalg.norm(base)
    rq -= (rq @ bh)[:, None] * bh[None]  # orthogonal to the cluster: these queries never overflow
    q = np.concatenate([base[None], rq])
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    qd, gd = torch.from_numpy(q).to(cuda), torch.from_numpy(g).to(cuda)
    nq = q.shape[0]
    L = _lib.lib()
    budget = L.rr_cosine_topk_workspace_size_cap(nq, n, d, k, 2000)
    assert budget < L.rr_cosine_topk_workspace_size(nq, n, d, k) // 10
    # raw C call on the bounded workspace: the overflow is reported, not hidden
    ws = torch.empty(budget, dtype=torch.uint8, device=cuda)
    s_raw = torch.empty((nq, k), dtype=torch.float32, device=cuda)
    i_raw = torch.empty((nq, k), dtype=torch.int64, device=cuda)
    hd = _lib.handle(cuda.index)
    _lib.check(L.rr_cosine_topk(hd, qd.data_ptr(), nq, gd.data_ptr(), n, d, k, 0, s_raw.data_ptr(), i_raw.data_ptr(),
                                ws.data_ptr(), budget, torch.cuda.current_stream(cuda).cuda_stream), hd, "topk")
    off = L.rr_cosine_topk_overflow_offset(nq, n, d, k)
    assert ws[off:off + 4].view(torch.int32).item() == 1
    cnt = ws[L.rr_cosine_topk_counts_offset(nq, n, d, k):][:4 * nq].view(torch.int32).cpu()
    assert cnt[0] > 2000 and (cnt[1:] <= 2000).all()

    s0, i0 = ops.cosine_topk(qd, gd, k)
    assert not torch.equal(i_raw[0], i0[0]) and torch.equal(i_raw[1:], i0[1:])
    s1, i1 = ops.cosine_topk(qd, gd, k, max_workspace_bytes=budget)
    assert torch.equal(i1, i0) and torch.equal(s1.view(torch.int32), s0.view(torch.int32))
    s_o, i_o = oracle.cosine_topk(q, g, k)
    assert np.array_equal(i0.cpu().numpy(), i_o) and np.array_equal(s0.cpu().numpy(), s_o)

    gb, _ = ops.quantize_rows(gd, "bf16")
    bound = ops.prefilter_gallery_bound(gd, gb)
    pbudget = L.rr_cosine_topk_prefilter_workspace_size_cap(nq, n, d, k, 2000)
    s2, i2 = ops.cosine_topk_prefilter(qd, gd, gb, bound, k, max_workspace_bytes=pbudget)
    assert torch.equal(i2, i0) and torch.equal(s2.view(torch.int32), s0.view(torch.int32))

    qb, _ = ops.quantize_rows(qd, "bf16")
    s3, i3 = ops.cosine_topk_lp(qb, None, gb, None, k, "bf16")
    s4, i4 = ops.cosine_topk_lp(qb, None, gb, None, k, "bf16", max_workspace_bytes=budget)
    assert torch.equal(i3, i4) and torch.equal(s3, s4)


@pytest.mark.parametrize("il", [0, 1])
def test_prefilter_sweep_mf16_bit_identical(cuda, il):
    """The 256x320 bf16 filter sweep on v_mfma_f32_16x16x32_bf16 (rr_set_tuning
    sweep_mf16): a different bf16 accumulation order inside the filter, the
    same final ranking bit for bit (the rigorous bound covers any order; the
    survivors are rescored exactly).  il = 1: both forms with the next
    k-tile's DMA spread among the MFMAs (sweep_il)."""
    rs = np.random.RandomState(78)
    d, nq, n = 2048, 1280, 70_003
    g = rs.standard_normal((n, d)).astype(np.float32)
    q = rs.standard_normal((nq, d)).astype(np.float32)
    g[5], g[n - 1] = q[0], q[nq - 1]
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    qd, gd = torch.from_numpy(q).to(cuda), torch.from_numpy(g).to(cuda)
    gbf, _ = ops.quantize_rows(gd, "bf16")
    bound = ops.prefilter_gallery_bound(gd, gbf)
    out = {}
    for v in (0, 1):
        with ops.tuning(cuda.index, sweep_mf16=v, sweep_il=il):
            out[v] = ops.cosine_topk_prefilter(qd, gd, gbf, bound, 100)
    with ops.tuning(cuda.index, sweep_mf16=0, sweep_il=0):
        ref = ops.cosine_topk_prefilter(qd, gd, gbf, bound, 100)
    for v in (0, 1):
        assert torch.equal(out[v][1], ref[1]) and torch.equal(out[v][0].view(torch.int32), ref[0].view(torch.int32)), v
    assert int(out[1][1][0, 0]) == 5 and int(out[1][1][nq - 1, 0]) == n - 1


@pytest.mark.parametrize("dt,d", [("fp8", 2048), ("bf16", 512)])
def test_lp_sweep_issue_spread_bit_identical(cuda, dt, d):
    """sweep_il = 1 on the 256x256 filter sweeps (the C5 fp8 and C4 bf16
    rankers): the next k-tile's DMA spread among the MFMAs, the same scores
    and indices bit for bit as one burst."""
    rs = np.random.RandomState(91)
    nq, n = 1280, 60_007
    g = rs.standard_normal((n, d)).astype(np.float32)
    q = rs.standard_normal((nq, d)).astype(np.float32)
    g[7], g[n - 1] = q[0], q[nq - 1]
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    ql, qs = ops.quantize_rows(torch.from_numpy(q).to(cuda), dt)
    gl, gs = ops.quantize_rows(torch.from_numpy(g).to(cuda), dt)
    out = {}
    for il in (0, 1):
        with ops.tuning(cuda.index, sweep_il=il):
            out[il] = ops.cosine_topk_lp(ql, qs, gl, gs, 100, dt)
    assert torch.equal(out[0][1], out[1][1]) and torch.equal(out[0][0].view(torch.int32), out[1][0].view(torch.int32))
    assert int(out[1][1][0, 0]) == 7 and int(out[1][1][nq - 1, 0]) == n - 1
