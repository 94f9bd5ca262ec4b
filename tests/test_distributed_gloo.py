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
