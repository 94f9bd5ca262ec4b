"""Gallery sharding across GPUs: one process per GPU,
torch.distributed over RCCL ("nccl" backend on ROCm), xGMI underneath.

Per search call, for a world of W ranks each holding B_r query descriptors and
a contiguous gallery shard [lo_r, hi_r):
  1. all-gather the query descriptors  -> every rank holds all Q = sum B_r;
  2. local fused cosine top-k of all Q queries against the shard
     (rr_cosine_topk, indices offset to global gallery rows);
  3. all-to-all of the partial top-k lists (scores fp32, idx int64): rank r
     receives, from every shard, the lists of its own B_r queries [W, B_r, k];
  4. k-way merge (rr_topk_merge), stable order (score desc, global idx asc).
The collectives move Q*D*4 and B_r*W*k*12 bytes per rank: latency-bound next
to the GEMM.

alpha-QE over the sharded gallery (config C5, ``alpha_qe_search``): after the
first search each rank holds the merged top-n of its own queries; the n
neighbour rows live on whichever shards own them.  Every rank learns all
ranks' top-n indices (all-gather, Q*n*8 bytes), sends each other rank exactly
the rows it owns for that rank's queries (one variable-split all-to-all,
about B_r*n*D*4 bytes in per rank), and the receiver puts every row back in its
(query, neighbour) slot.  The expansion then runs on copies of the very rows a
single-GPU run reads, in the same order, so the expanded queries and the second
search are bit-identical to the single-GPU path.  Ranking work per rank is Q x N/W, so the units (images embedded and
ranked against the whole gallery) scale weakly with W.

The reference has no distributed evaluation (NCCL is
training-only); this is new.  ``local_topk`` / ``merge`` are injectable so
the choreography is unit-tested on CPU with gloo against the oracle; the
product defaults are the librr kernels.
"""
import torch
import torch.distributed as dist

from . import ops


def shard_bounds(n, world, rank):
    """Contiguous row range of rank's shard (first n % world shards get +1)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _host_staged(group):
    """gloo has no all_gather / all_to_all for device tensors: rehearsal runs
    of the sharded path (several ranks on one GPU, gloo transport) stage the
    collectives through host memory.  RCCL ("nccl") moves device tensors."""
    return dist.get_backend(group) == "gloo"


def _to_comm(t, group):
    """The tensor a collective of `group` can move (host copy under gloo)."""
    return t.cpu() if _host_staged(group) else t


# device->host reads the sharded path made (size exchanges); with every
# rank's query count known (`counts`) search / gather_rows make none
HOST_READS = [0]


def _exchange_sizes(n_rows, group, device):
    """Every rank's first dim: one small all-gather and one device->host read."""
    world = dist.get_world_size(group)
    n = torch.tensor([n_rows], dtype=torch.int64, device=device)
    parts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(parts, n, group=group)
    HOST_READS[0] += 1
    return torch.cat(parts).tolist()


def _all_gather_var(t, group, sizes=None):
    """all_gather of tensors whose first dim may differ across ranks.  With
    `sizes` (every rank's first dim, known to all ranks, e.g. a fixed batch)
    no size exchange and no host sync happen; otherwise one small all-gather
    and one device->host read."""
    world = dist.get_world_size(group)
    dev = t.device
    t = _to_comm(t, group)
    if sizes is None:
        sizes = _exchange_sizes(t.shape[0], group, t.device)
    else:
        sizes = [int(x) for x in sizes]
        if len(sizes) != world or sizes[dist.get_rank(group)] != t.shape[0]:
            raise ValueError(f"_all_gather_var: sizes {sizes} do not match this rank's {t.shape[0]} rows")
    mx = max(sizes)
    pad = t.new_zeros((mx,) + tuple(t.shape[1:]))
    pad[: t.shape[0]] = t
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    return [o[:s].to(dev) for o, s in zip(outs, sizes)], sizes


class ShardedGallery:
    """This rank's shard of a gallery that is row-partitioned over the group."""

    def __init__(self, shard, global_offset, group=None, local_topk=None, merge=None, workspace=None, dtype="fp32",
                 prefilter=False, max_workspace_bytes=None):
        """dtype "fp32" ranks exactly; prefilter=True gives the same exact
        result through the bf16-bound prefilter (rr_cosine_topk_prefilter).
        max_workspace_bytes bounds the ranker workspace (rr.h "Bounded
        workspaces"; overflowed queries are re-run, results unchanged)."""
        self.max_ws = max_workspace_bytes
        self.shard = shard
        self.offset = int(global_offset)
        # rr_topk_merge keys carry 32-bit row indices (0xffffffff reserved)
        if self.offset + shard.shape[0] >= 0xffffffff:
            raise ValueError("ShardedGallery: global row indices must stay below 2^32 - 1")
        self.group = group
        self._local_topk = local_topk
        self._merge = merge
        self._ws = workspace
        self.dtype = dtype
        self.prefilter = bool(prefilter) and dtype == "fp32"
        self.shard_lp, self.shard_scale, self.bound = (None, None, None)
        if local_topk is None and (dtype != "fp32" or self.prefilter):
            self.shard_lp, self.shard_scale = ops.quantize_rows(shard, "bf16" if self.prefilter else dtype)
        if self.prefilter and local_topk is None:
            self.bound = ops.prefilter_gallery_bound(shard, self.shard_lp)

    def _local(self, q, k):
        if self._local_topk is not None:
            return self._local_topk(q, self.shard, k, self.offset)
        n, d = self.shard.shape[0], q.shape[1]
        self._ws, _ = ops._ranker_workspace("prefilter" if self.prefilter else "exact", q.shape[0], n, d, k,
                                            self._ws, self.max_ws, q.device)
        kw = dict(idx_offset=self.offset, workspace=self._ws, max_workspace_bytes=self.max_ws)
        if self.prefilter:
            return ops.cosine_topk_prefilter(q, self.shard, self.shard_lp, self.bound, k, **kw)
        if self.dtype != "fp32":
            q_lp, q_sc = ops.quantize_rows(q, self.dtype)
            return ops.cosine_topk_lp(q_lp, q_sc, self.shard_lp, self.shard_scale, k, self.dtype, **kw)
        return ops.cosine_topk(q, self.shard, k, **kw)

    def _bounds(self):
        """[lo_r, hi_r) of every rank's shard (all-gathered once)."""
        if getattr(self, "_his", None) is None:
            group = self.group
            t = torch.tensor([self.offset, self.offset + self.shard.shape[0]], dtype=torch.int64,
                             device="cpu" if _host_staged(group) else self.shard.device)
            parts = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
            dist.all_gather(parts, t, group=group)
            self._his = torch.stack(parts)[:, 1].to(self.shard.device)
        return self._his

    def _owner(self, idx):
        """Rank whose shard holds each global row index (shards are contiguous, in rank order)."""
        return torch.bucketize(idx, self._bounds(), right=True)

    def gather_rows(self, idx, counts=None):
        """Rows g[idx] of the global gallery for this rank's queries: idx
        [B_r, n] int64 (global rows; < 0 = padding -> a zero row) -> [B_r, n, D]
        fp32, each row an exact copy from the shard that owns it.

        Fixed-size exchange, no data-dependent split sizes: every rank sends
        each requester r a [B_r * n, D] block holding the rows it owns in
        their request slots (zeros elsewhere), and the requester picks every
        slot from its owner's block.  With counts (every rank's B_r) nothing
        here reads the device from the host; without, one size exchange.
        Bytes per rank: Q * n * D * 4 out and W * B_r * n * D * 4 in (W times
        the owned rows alone, which would need their counts on the host)."""
        group = self.group
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        dev = self.shard.device
        b, n = idx.shape
        d = self.shard.shape[1]
        ids, sizes = _all_gather_var(idx.contiguous(), group, counts)
        # every rank's requests, requester-major, (query, neighbour) order within
        req = torch.cat([x.reshape(-1).to(dev) for x in ids]) if ids else idx.new_empty((0,)).to(dev)
        mine = (req >= 0) & (self._owner(req.clamp_min(0)) == rank)
        if self.shard.shape[0] > 0:
            rows = self.shard.index_select(0, (req - self.offset).clamp(0, self.shard.shape[0] - 1))
            sendbuf = torch.where(mine[:, None], rows, torch.zeros((), dtype=rows.dtype, device=dev))
        else:
            sendbuf = self.shard.new_zeros((req.shape[0], d))
        recvbuf = _to_comm(self.shard.new_empty((world * b * n, d)), group)
        dist.all_to_all_single(recvbuf, _to_comm(sendbuf.contiguous(), group), [b * n] * world,
                               [sz * n for sz in sizes], group=group)
        blocks = torch.cat([recvbuf.to(dev).view(world, b * n, d), self.shard.new_zeros((1, b * n, d))])
        flat = idx.reshape(-1).to(dev)
        own = torch.where(flat >= 0, self._owner(flat.clamp_min(0)), torch.full_like(flat, world))
        out = blocks[own, torch.arange(b * n, device=dev)]  # padding slots pick the zero block
        return out.view(b, n, d)

    def alpha_qe_search(self, queries, k=100, n=2, alpha=3.0, expand=None, counts=None):
        """Search, alpha-QE this rank's queries with their top-n neighbours
        (rows fetched from their owning shards), search again (config C5).
        Returns (scores [B_r,k], global idx [B_r,k], expanded queries).
        counts: every rank's query count when known (see search)."""
        s, i = self.search(queries, max(k, n), counts)
        rows = self.gather_rows(i[:, :n].contiguous(), counts)
        top_s = s[:, :n].contiguous()
        b = queries.shape[0]
        if b == 0:  # no queries on this rank: still take part in the collectives
            q2 = queries
        elif expand is not None:
            q2 = expand(queries, rows, top_s, n, alpha)
        else:
            local = torch.arange(b * n, dtype=torch.int64, device=queries.device).view(b, n)
            q2 = ops.alpha_qe(queries.contiguous(), rows.view(b * n, rows.shape[-1]), local, top_s, n=n, alpha=alpha)
        s2, i2 = self.search(q2, k, counts)
        return s2, i2, q2

    def _merge_parts(self, ps, pi, k):
        if self._merge is not None:
            return self._merge(ps, pi, k)
        return ops.topk_merge(ps, pi, k)

    def search(self, queries, k, counts=None):
        """queries [B_r, D] (this rank's) -> (scores [B_r,k], global idx [B_r,k]).
        counts: every rank's B_r, when all ranks know them (a fixed batch):
        then the collectives and the merge make no host sync; without, one
        size all-gather + one host read.  With max_workspace_bytes set, the
        local ranker reads its 4-byte overflow count once per call
        (ops._recover_overflow), which syncs the stream."""
        group = self.group
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        qs, sizes = _all_gather_var(queries.contiguous(), group, counts)
        allq = torch.cat(qs, 0).contiguous()
        s, i = self._local(allq, k)
        # each rank needs only its own queries' partial lists: all-to-all
        # (B_r * W * k * 12 bytes in per rank instead of Q * W * k * 12)
        mine = sizes[rank]
        dev = s.device
        s, i = _to_comm(s, group), _to_comm(i, group)
        rs = s.new_empty((world * mine, k))
        ri = i.new_empty((world * mine, k))
        dist.all_to_all_single(rs, s.contiguous(), [mine] * world, sizes, group=group)
        dist.all_to_all_single(ri, i.contiguous(), [mine] * world, sizes, group=group)
        rs, ri = rs.to(dev), ri.to(dev)
        return self._merge_parts(rs.view(world, mine, k).contiguous(), ri.view(world, mine, k).contiguous(), k)


def sharded_step(sharded, desc, workload, k, counts, n=2, alpha=3.0, expand=None):
    """The rank step of bench.py's sharded workloads after embedding: C3 / C4
    rank this rank's descriptors against the whole row-sharded gallery; C5
    ranks, alpha-QE-expands with the top-n neighbour rows fetched from their
    owning shards, and ranks again.  -> (scores [B_r,k], global idx [B_r,k])."""
    if workload == "c5":
        s2, i2, _ = sharded.alpha_qe_search(desc, k, n=n, alpha=alpha, expand=expand, counts=counts)
        return s2, i2
    return sharded.search(desc, k, counts)
