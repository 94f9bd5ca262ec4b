"""The sharded search with the real librr kernels (fused top-k or the exact
prefilter on each shard, rr_topk_merge), two ranks sharing the box's one GPU
over gloo (host-staged collectives; on an 8-GPU node the same code runs over
RCCL).  Must equal the single-process oracle ranking bit for bit."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, q_all, g_all, k, sizes, prefilter, out, dtype="fp32"):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from research_image_retrieval_amd.distributed import ShardedGallery, shard_bounds
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    lo, hi = shard_bounds(g_all.shape[0], world, rank)
    sg = ShardedGallery(g_all[lo:hi].contiguous().to(dev), lo, prefilter=prefilter, dtype=dtype)
    qlo = sum(sizes[:rank])
    s, i = sg.search(q_all[qlo:qlo + sizes[rank]].contiguous().to(dev), k)
    out[rank] = (s.cpu().numpy(), i.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("prefilter", [False, True])
def test_sharded_search_real_kernels_world2(prefilter):
    import oracle
    from test_distributed_gloo import _free_port
    rs = np.random.RandomState(3)
    d = 256
    q = rs.standard_normal((9, d)).astype(np.float32)
    g = rs.standard_normal((90_001, d)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    g[60_000] = g[10]  # exact tie across the shard boundary
    q[0] = g[10]
    k = 64
    sizes = [4, 5]
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(2, _free_port(), torch.from_numpy(q), torch.from_numpy(g), k, sizes, prefilter,
                                      out), nprocs=2, join=True, start_method="spawn")
    s = np.concatenate([out[0][0], out[1][0]])
    i = np.concatenate([out[0][1], out[1][1]])
    s_o, i_o = oracle.cosine_topk(q, g, k)
    assert np.array_equal(i, i_o) and np.array_equal(s, s_o)
    assert list(i[0, :2]) == [10, 60_000]


@pytest.mark.parametrize("n,d", [(90_001, 512), (33_333, 256)])
def test_sharded_search_bf16_real_kernels_world2(cuda, n, d):
    """C4's N > 1 ranker: ShardedGallery(dtype="bf16") -- the all-gathered
    queries quantised and swept against each rank's bf16 shard
    (quantize_rows + cosine_topk_lp), the partial lists all-to-all'd and
    merged -- equals GallerySearcher(dtype="bf16") on the whole gallery bit
    for bit, with a tie planted across the shard boundary."""
    from test_distributed_gloo import _free_port
    from research_image_retrieval_amd.search import GallerySearcher
    rs = np.random.RandomState(n + d)
    q = rs.standard_normal((11, d)).astype(np.float32)
    g = rs.standard_normal((n, d)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    g[n - 7] = g[12]  # exact tie across the shard boundary
    q[2] = g[12]
    k = 100
    sizes = [5, 6]
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(2, _free_port(), torch.from_numpy(q), torch.from_numpy(g), k, sizes, False,
                                      out, "bf16"), nprocs=2, join=True, start_method="spawn")
    s = np.concatenate([out[0][0], out[1][0]])
    i = np.concatenate([out[0][1], out[1][1]])
    srch = GallerySearcher(torch.from_numpy(g), device=cuda, normalize=False, dtype="bf16")
    s_ref, i_ref = srch.topk(torch.from_numpy(q), k, normalize=False)
    assert np.array_equal(i, i_ref.cpu().numpy()) and np.array_equal(s, s_ref.cpu().numpy())
    assert list(i[2, :2]) == [12, n - 7]


def _qe_worker(rank, world, port, q_all, g_all, k, sizes, dtype, out):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from research_image_retrieval_amd.distributed import ShardedGallery, shard_bounds
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    lo, hi = shard_bounds(g_all.shape[0], world, rank)
    sg = ShardedGallery(g_all[lo:hi].contiguous().to(dev), lo, dtype=dtype)
    qlo = sum(sizes[:rank])
    s, i, q2 = sg.alpha_qe_search(q_all[qlo:qlo + sizes[rank]].contiguous().to(dev), k, n=2, alpha=3.0)
    out[rank] = (s.cpu().numpy(), i.cpu().numpy(), q2.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("dtype", ["fp8", "fp32"])
def test_sharded_alpha_qe_real_kernels_world2(cuda, dtype):
    """C5's alpha-QE re-search over a 2-way sharded gallery (rows fetched from
    their owning shard) == the single-GPU alpha_qe_search, bit for bit."""
    from test_distributed_gloo import _free_port
    from research_image_retrieval_amd.search import GallerySearcher, alpha_qe_search
    rs = np.random.RandomState(5)
    d = 256
    q = rs.standard_normal((7, d)).astype(np.float32)
    g = rs.standard_normal((50_001, d)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    g[40_000] = q[1] * 0.8 + g[40_000] * 0.2  # a strong neighbour on shard 1 for a rank-0 query
    g[40_000] /= np.linalg.norm(g[40_000])
    k = 50
    sizes = [3, 4]
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_qe_worker, args=(2, _free_port(), torch.from_numpy(q), torch.from_numpy(g), k, sizes, dtype,
                                         out), nprocs=2, join=True, start_method="spawn")
    srch = GallerySearcher(torch.from_numpy(g), device=cuda, normalize=False, dtype=dtype)
    s_ref, i_ref, q2_ref = alpha_qe_search(srch, torch.from_numpy(q), k=k, n=2, alpha=3.0, normalize=False)
    got = [out[0], out[1]]
    assert np.array_equal(np.concatenate([o[2] for o in got]), q2_ref.cpu().numpy())
    assert np.array_equal(np.concatenate([o[1] for o in got]), i_ref.cpu().numpy())
    assert np.array_equal(np.concatenate([o[0] for o in got]), s_ref.cpu().numpy())
