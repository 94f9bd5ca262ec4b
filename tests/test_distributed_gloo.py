"""World-size-2 gloo test of the sharded search choreography (query
all-gather -> per-shard top-k -> all-to-all of partial lists -> merge), with
the oracle standing in for the local kernels.  Must equal the single-process
stable top-k over the whole gallery, bit for bit."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _local_topk(q, shard, k, offset):
    import oracle
    s, i = oracle.cosine_topk(q.numpy(), shard.numpy(), k, idx_offset=offset)
    return torch.from_numpy(s), torch.from_numpy(i)


def _merge(ps, pi, k):
    import oracle
    s, i = oracle.topk_merge(ps.numpy(), pi.numpy(), k)
    return torch.from_numpy(s), torch.from_numpy(i)


def _worker(rank, world, port, q_all, g_all, k, sizes, out):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from research_image_retrieval_amd.distributed import ShardedGallery, shard_bounds
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_bounds(g_all.shape[0], world, rank)
    sg = ShardedGallery(g_all[lo:hi].contiguous(), lo, local_topk=_local_topk, merge=_merge)
    qlo = sum(sizes[:rank])
    s, i = sg.search(q_all[qlo:qlo + sizes[rank]].contiguous(), k)
    # every rank's query count known up front: no size exchange, same result
    s_c, i_c = sg.search(q_all[qlo:qlo + sizes[rank]].contiguous(), k, counts=sizes)
    assert torch.equal(s, s_c) and torch.equal(i, i_c)
    try:
        sg.search(q_all[qlo:qlo + sizes[rank]].contiguous(), k, counts=sizes[::-1])
        raise AssertionError("mismatched counts accepted")
    except ValueError:
        pass
    out[rank] = (s.numpy(), i.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_search_world2_matches_single():
    import oracle
    rs = np.random.RandomState(0)
    q = rs.standard_normal((7, 64)).astype(np.float32)
    g = rs.standard_normal((1001, 64)).astype(np.float32)
    g[500] = g[10]  # exact tie across the shard boundary
    k = 20
    sizes = [3, 4]  # ragged query counts per rank
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(2, _free_port(), torch.from_numpy(q), torch.from_numpy(g), k, sizes, out),
                       nprocs=2, join=True, start_method="spawn")
    s_ref, i_ref = oracle.cosine_topk(q, g, k)
    s = np.concatenate([out[0][0], out[1][0]])
    i = np.concatenate([out[0][1], out[1][1]])
    np.testing.assert_array_equal(i, i_ref)
    np.testing.assert_array_equal(s, s_ref)


def _expand(q, rows, top_s, n, alpha):
    """alpha-QE on fetched rows with the oracle's float64 restatement."""
    import oracle
    b = q.shape[0]
    idx = np.arange(b * n).reshape(b, n)
    return torch.from_numpy(oracle.alpha_qe(q.numpy(), rows.reshape(b * n, rows.shape[-1]).numpy(), idx, top_s.numpy(), n, alpha))


def _qe_worker(rank, world, port, q_all, g_all, k, sizes, out):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from research_image_retrieval_amd.distributed import ShardedGallery, shard_bounds
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_bounds(g_all.shape[0], world, rank)
    sg = ShardedGallery(g_all[lo:hi].contiguous(), lo, local_topk=_local_topk, merge=_merge)
    qlo = sum(sizes[:rank])
    mine = q_all[qlo:qlo + sizes[rank]].contiguous()
    # first row, a padding slot (idx -1: fewer gallery rows than neighbours), last row
    rows = sg.gather_rows(torch.tensor([[0, -1, g_all.shape[0] - 1]] * sizes[rank], dtype=torch.int64).view(-1, 3))
    s, i, q2 = sg.alpha_qe_search(mine, k, n=3, alpha=3.0, expand=_expand)
    s_c, i_c, q2_c = sg.alpha_qe_search(mine, k, n=3, alpha=3.0, expand=_expand, counts=sizes)
    assert torch.equal(s, s_c) and torch.equal(i, i_c) and torch.equal(q2, q2_c)
    out[rank] = (s.numpy(), i.numpy(), q2.numpy(), rows.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_alpha_qe_world3_matches_single():
    """C5 over a sharded gallery: neighbour rows fetched from their owning
    shards; expanded queries and the second search equal the single-process
    pipeline bit for bit (3 ranks, ragged queries, one rank with none)."""
    import oracle
    rs = np.random.RandomState(1)
    q = rs.standard_normal((6, 48)).astype(np.float32)
    g = rs.standard_normal((700, 48)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    g[650] = q[0] * 0.9 + g[650] * 0.1  # a neighbour on the last shard
    k, n = 15, 3
    sizes = [4, 0, 2]
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_qe_worker, args=(3, _free_port(), torch.from_numpy(q), torch.from_numpy(g), k, sizes, out),
                       nprocs=3, join=True, start_method="spawn")
    s1, i1 = oracle.cosine_topk(q, g, k)
    q2 = oracle.alpha_qe(q, g, i1, s1, n, 3.0)
    s2, i2 = oracle.cosine_topk(q2, g, k)
    got = [out[r] for r in range(3)]
    np.testing.assert_array_equal(np.concatenate([o[2] for o in got]), q2)
    np.testing.assert_array_equal(np.concatenate([o[1] for o in got]), i2)
    np.testing.assert_array_equal(np.concatenate([o[0] for o in got]), s2)
    for o in got:  # gather_rows of the first gallery row, a padding slot, the last row
        assert np.array_equal(o[3][:, 0], np.broadcast_to(g[0], o[3][:, 0].shape))
        assert not o[3][:, 1].any()
        assert np.array_equal(o[3][:, 2], np.broadcast_to(g[-1], o[3][:, 2].shape))


def _step_worker(rank, world, port, q_all, g_all, k, batch, out):
    """bench.py's sharded rank step (distributed.sharded_step) for C3 and C5
    with every rank's query count known, as bench runs it (fixed batch; a
    list gives each rank its own count, zero included)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from research_image_retrieval_amd import distributed as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = D.shard_bounds(g_all.shape[0], world, rank)
    sg = D.ShardedGallery(g_all[lo:hi].contiguous(), lo, local_topk=_local_topk, merge=_merge)
    counts = list(batch) if isinstance(batch, (list, tuple)) else [batch] * world
    sg._bounds()  # the shard bounds are all-gathered once per gallery, before the timed steps
    qlo = sum(counts[:rank])
    desc = q_all[qlo:qlo + counts[rank]].contiguous()
    reads0 = D.HOST_READS[0]
    res = {w: D.sharded_step(sg, desc, w, k, counts, n=2, alpha=3.0, expand=_expand) for w in ("c3", "c5")}
    # exact copies through the fixed-size exchange, -0.0 included
    rows = sg.gather_rows(torch.tensor([[3, g_all.shape[0] - 1]] * counts[rank], dtype=torch.int64).view(-1, 2),
                          counts)
    assert D.HOST_READS[0] == reads0, "the counted sharded step read the device from the host"
    out[rank] = {w: (s.numpy(), i.numpy()) for w, (s, i) in res.items()}, rows.numpy()
    dist.barrier()
    dist.destroy_process_group()


def test_bench_sharded_step_world2_world4_matches_single():
    """bench.py's C3 and C5 sharded choreography at world 2 and 4 (gloo, the
    oracle as the local kernels): equal to the single-process pipeline bit
    for bit, and no host read anywhere in the counted step."""
    import oracle
    rs = np.random.RandomState(5)
    batch, k, dim = 3, 12, 32
    g = rs.standard_normal((997, dim)).astype(np.float32)
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    g[3, :4] = -0.0
    for world in (2, 4):
        q = rs.standard_normal((batch * world, dim)).astype(np.float32)
        q /= np.linalg.norm(q, axis=1, keepdims=True)
        g[900] = q[0] * 0.95 + g[900] * 0.05  # a close neighbour on the last shard
        mgr = mp.Manager()
        out = mgr.dict()
        mp.start_processes(_step_worker, args=(world, _free_port(), torch.from_numpy(q), torch.from_numpy(g), k,
                                               batch, out), nprocs=world, join=True, start_method="spawn")
        s1, i1 = oracle.cosine_topk(q, g, k)
        q2 = oracle.alpha_qe(q, g, i1, s1, 2, 3.0)
        s2, i2 = oracle.cosine_topk(q2, g, k)
        got = [out[r] for r in range(world)]
        for w, (s_ref, i_ref) in (("c3", (s1, i1)), ("c5", (s2, i2))):
            np.testing.assert_array_equal(np.concatenate([o[0][w][1] for o in got]), i_ref)
            np.testing.assert_array_equal(np.concatenate([o[0][w][0] for o in got]), s_ref)
        for o in got:
            assert np.array_equal(o[1][:, 0].view(np.int32), np.broadcast_to(g[3], o[1][:, 0].shape).view(np.int32))
            assert np.array_equal(o[1][:, 1], np.broadcast_to(g[-1], o[1][:, 1].shape))


def test_bench_sharded_step_world8_matches_single():
    """The target node's world size: 8 contiguous shards, bench.py's C3 and
    C5 choreography (gloo, the oracle as the local kernels), ragged query
    counts with one rank holding none; equal to the single-process pipeline
    bit for bit, no host read in the counted step."""
    import oracle
    rs = np.random.RandomState(8)
    k, dim = 10, 24
    counts = [3, 2, 0, 3, 1, 3, 2, 3]
    g = rs.standard_normal((1203, dim)).astype(np.float32)
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    g[3, :4] = -0.0
    q = rs.standard_normal((sum(counts), dim)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    g[1190] = q[0] * 0.95 + g[1190] * 0.05  # a close neighbour on the last shard
    g[151] = g[150]  # an exact tie across the first shard boundary (1203 / 8: shard 0 is [0, 151))
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_step_worker, args=(8, _free_port(), torch.from_numpy(q), torch.from_numpy(g), k, counts, out),
                       nprocs=8, join=True, start_method="spawn")
    s1, i1 = oracle.cosine_topk(q, g, k)
    q2 = oracle.alpha_qe(q, g, i1, s1, 2, 3.0)
    s2, i2 = oracle.cosine_topk(q2, g, k)
    got = [out[r] for r in range(8)]
    assert got[2][0]["c3"][1].shape == (0, k) and got[2][0]["c5"][1].shape == (0, k)
    for w, (s_ref, i_ref) in (("c3", (s1, i1)), ("c5", (s2, i2))):
        np.testing.assert_array_equal(np.concatenate([o[0][w][1] for o in got]), i_ref)
        np.testing.assert_array_equal(np.concatenate([o[0][w][0] for o in got]), s_ref)
    for o in got:
        assert np.array_equal(o[1][:, 0].view(np.int32), np.broadcast_to(g[3], o[1][:, 0].shape).view(np.int32))
        assert np.array_equal(o[1][:, 1], np.broadcast_to(g[-1], o[1][:, 1].shape))


def test_prefilter_workspace_fits_budget_at_world8():
    """bench.py at N = 8 (weak scaling: 1280 queries per rank, all 10,240
    ranked against each 200,000-row shard, d = 2048, k = 100, --ws-budget-gb
    4): the seed sample shrinks to 4,166 rows per shard; the minimum ranker
    workspace fits the budget, and the candidate cap that 4 GB affords
    (49,831 per query) is over 4x the k * n / s survivors the seed threshold
    leaves per query (the bf16 bound's band adds to that; a query past the
    cap is counted and re-run with a worst-case workspace, results
    unchanged: test_gpu_rank.py::test_bounded_workspace_overflow_recovery)."""
    import importlib.util
    from research_image_retrieval_amd import ops
    from research_image_retrieval_amd import _lib
    from research_image_retrieval_amd.distributed import shard_bounds
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    world, batch, n_total, d, k, budget = 8, 1280, 1_600_000, 2048, 100, 4 << 30
    L = _lib.lib()
    for rank in range(world):
        lo, hi = shard_bounds(n_total, world, rank)
        n = hi - lo
        s = bench.seed_rows(n, k)
        assert s == 4166
        q_total = batch * world
        ws_lo, ws_full = ops.ranker_workspace_bounds("prefilter", q_total, n, d, k)
        ws = max(ws_lo, min(ws_full, budget))  # bench.py's allocation
        assert ws_lo <= budget and ws <= budget
        cap = L.rr_cosine_topk_prefilter_cap_for(q_total, n, d, k, ws)
        expected = k * n / s
        assert cap >= 4 * expected, (cap, expected)
