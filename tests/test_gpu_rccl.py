"""The multi-GPU code path over RCCL itself, on the box's one GPU: a process
group of one rank with the "nccl" backend (RCCL on ROCm), device tensors in
every collective (query all-gather, partial-list all-to-all, the alpha-QE row
exchange with uneven splits).  The 2-rank tests (test_gpu_distributed.py) share
one GPU and therefore run over gloo; this one executes the RCCL calls the
8-GPU node runs, and must equal the single-GPU path bit for bit."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _rccl_worker(rank, port, q, g, k, out):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from research_image_retrieval_amd import ops
    from research_image_retrieval_amd.distributed import ShardedGallery
    from research_image_retrieval_amd.search import GallerySearcher, alpha_qe_search
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    res = {"backend": dist.get_backend()}
    qd, gd = q.to(dev), g.to(dev)
    nq = q.shape[0]
    s0, i0 = ops.cosine_topk(qd, gd, k)
    for pre in (False, True):
        sg = ShardedGallery(gd, 0, prefilter=pre, max_workspace_bytes=64 << 20)
        s1, i1 = sg.search(qd, k)
        s2, i2 = sg.search(qd, k, counts=[nq])
        res[f"search_pre{int(pre)}"] = bool(torch.equal(i1, i0) and torch.equal(s1, s0) and torch.equal(i2, i0)
                                            and torch.equal(s2, s0))
    # C4's ranker: the bf16 shard (quantize_rows + cosine_topk_lp inside search)
    sg = ShardedGallery(gd, 0, dtype="bf16")
    s5, i5 = sg.search(qd, k, counts=[nq])
    s6, i6 = GallerySearcher(g, device=dev, normalize=False, dtype="bf16").topk(q, k, normalize=False)
    res["search_bf16"] = bool(torch.equal(i5, i6) and torch.equal(s5, s6))
    # rows of the global gallery by index, padding slots (-1) zero
    sg = ShardedGallery(gd, 0)
    idx = torch.tensor([[0, -1, g.shape[0] - 1]] * nq, dtype=torch.int64, device=dev)
    rows = sg.gather_rows(idx, counts=[nq])
    res["gather_rows"] = bool(torch.equal(rows[:, 0], gd[0].expand(nq, -1)) and not rows[:, 1].any()
                              and torch.equal(rows[:, 2], gd[-1].expand(nq, -1)))
    for dtype in ("fp8", "fp32"):
        sg = ShardedGallery(gd, 0, dtype=dtype)
        s3, i3, q3 = sg.alpha_qe_search(qd, k, n=2, alpha=3.0, counts=[nq])
        srch = GallerySearcher(g, device=dev, normalize=False, dtype=dtype)
        s4, i4, q4 = alpha_qe_search(srch, q, k=k, n=2, alpha=3.0, normalize=False)
        res[f"alpha_qe_{dtype}"] = bool(torch.equal(q3, q4) and torch.equal(i3, i4) and torch.equal(s3, s4))
    dist.barrier()
    dist.destroy_process_group()
    out.update(res)


def test_sharded_path_over_rccl_world1():
    """fp32 / prefilter / bf16 sharded search, gather_rows and the fp8 / fp32
    alpha-QE re-search over RCCL on a world of one: each equals the
    single-GPU path bit for bit."""
    from test_distributed_gloo import _free_port
    rs = np.random.RandomState(17)
    d = 256
    q = rs.standard_normal((11, d)).astype(np.float32)
    g = rs.standard_normal((60_001, d)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    g[30_000] = q[2]
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_rccl_worker, args=(_free_port(), torch.from_numpy(q), torch.from_numpy(g), 50, out),
                       nprocs=1, join=True, start_method="spawn")
    res = dict(out)
    print(res)
    assert res.pop("backend") == "nccl"
    assert all(res.values()), res
