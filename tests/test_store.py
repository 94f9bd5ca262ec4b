"""Descriptor store (store.py): on-disk format round trips, shard-spanning
reads, labels, integrity checks, and per-rank shard loading that feeds the
sharded search (world-size-2 gloo, oracle local kernels)."""
import json
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from research_image_retrieval_amd import store as S
from research_image_retrieval_amd.distributed import shard_bounds


def _vecs(n, d, seed=0):
    return np.random.RandomState(seed).standard_normal((n, d)).astype(np.float32)


def test_round_trip_and_spanning_reads(tmp_path):
    v = _vecs(1003, 24)
    lab = np.arange(1003, dtype=np.int64) * 7
    st = S.write_store(str(tmp_path / "g"), v, shard_rows=250, labels=lab)
    assert st.n == 1003 and st.d == 24 and len(st.shards) == 5
    assert st.verify()
    for lo, hi in [(0, 1003), (249, 251), (0, 0), (500, 1003), (999, 1003), (100, 760)]:
        assert np.array_equal(st.rows(lo, hi), v[lo:hi])
        assert np.array_equal(st.to_device(lo, hi, "cpu", chunk_rows=77).numpy(), v[lo:hi])
    assert np.array_equal(st.labels(10, 20), lab[10:20])
    with pytest.raises(IndexError):
        st.rows(0, 1004)


def test_streaming_append_and_checks(tmp_path):
    p = str(tmp_path / "g")
    v = _vecs(700, 8, 1)
    with S.DescriptorStoreWriter(p, 8, shard_rows=300) as w:
        for i in range(0, 700, 130):  # appends that straddle shard boundaries
            w.append(torch.from_numpy(v[i:i + 130]))
    st = S.DescriptorStore(p)
    assert [s["rows"] for s in st.shards] == [300, 300, 100]
    assert np.array_equal(st.rows(0, 700), v)
    with pytest.raises(FileExistsError):
        S.DescriptorStoreWriter(p, 8)
    with pytest.raises(ValueError):
        S.DescriptorStoreWriter(str(tmp_path / "h"), 8).append(v[:, :4])
    # corruption is detected
    f = os.path.join(p, st.shards[1]["file"])
    raw = bytearray(open(f, "rb").read())
    raw[5] ^= 1
    open(f, "wb").write(bytes(raw))
    with pytest.raises(ValueError):
        S.DescriptorStore(p).verify()
    open(f, "wb").write(bytes(raw[:-4]))
    with pytest.raises(ValueError):
        S.DescriptorStore(p)
    meta = json.load(open(os.path.join(p, "store.json")))
    meta["version"] = 99
    json.dump(meta, open(os.path.join(p, "store.json"), "w"))
    with pytest.raises(ValueError):
        S.DescriptorStore(p)


def _worker(rank, world, port, path, q_all, k, out):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from research_image_retrieval_amd.distributed import ShardedGallery
    from test_distributed_gloo import _local_topk, _merge
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    shard, lo = S.load_gallery_shard(path, rank, world, "cpu")
    sg = ShardedGallery(shard, lo, local_topk=_local_topk, merge=_merge)
    s, i = sg.search(q_all[rank::world].contiguous(), k)
    out[rank] = (s.numpy(), i.numpy(), lo, shard.shape[0])
    dist.barrier()
    dist.destroy_process_group()


def test_store_shards_feed_sharded_search(tmp_path):
    import oracle
    from test_distributed_gloo import _free_port
    g = _vecs(901, 32, 2)
    q = _vecs(6, 32, 3)
    path = str(tmp_path / "g")
    S.write_store(path, g, shard_rows=128)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(2, _free_port(), path, torch.from_numpy(q), 15, out),
                       nprocs=2, join=True, start_method="spawn")
    for r in range(2):
        s, i, lo, rows = out[r]
        assert (lo, lo + rows) == shard_bounds(901, 2, r)
        s_ref, i_ref = oracle.cosine_topk(q[r::2], g, 15)
        assert np.array_equal(i, i_ref) and np.array_equal(s, s_ref)
