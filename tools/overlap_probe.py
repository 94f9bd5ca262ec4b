"""Does the C3 ranker (bf16 prefilter sweep + exact rescoring: MFMA and
L2-bound, light on HBM) overlap with the next batch's trunk (HBM-bound
residual expansions with idle matrix cores) when the two run on separate HIP
streams?  Times embed alone, rank alone, and embed(batch i+1) || rank(batch i).
usage: overlap_probe.py [B] [reps]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from research_image_retrieval_amd import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1280
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
N = 1_600_000
gal = bench.make_gallery(N, 2048, 0, N, dev)
gbf, _ = ops.quantize_rows(gal, "bf16")
bound = ops.prefilter_gallery_bound(gal, gbf)
net = bench.build_extractor("resnet101", dev)
rs = np.random.RandomState(1234)
imgs = torch.from_numpy(rs.randint(0, 256, size=(B, 224, 224, 3), dtype=np.uint8)).to(dev)
lo_ws, full_ws = ops.ranker_workspace_bounds("prefilter", B, N, 2048, 100)
ws = torch.empty(max(lo_ws, min(full_ws, 4 << 30)), dtype=torch.uint8, device=dev)
ws2 = torch.empty_like(ws)


def embed():
    return net.forward_test_u8(imgs)


def rank(d, w):
    return ops.cosine_topk_prefilter(d, gal, gbf, bound, 100, workspace=w, max_workspace_bytes=4 << 30)


def wall(fn):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(REPS):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / REPS * 1e3


d0 = embed()
ref_s, ref_i = rank(d0, ws)
torch.cuda.synchronize()
t_embed = wall(embed)
t_rank = wall(lambda: rank(d0, ws))
s_a, s_b = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def pipelined(steps=REPS):
    """steps embeds and steps ranks; rank(i) on stream B overlaps embed(i+1) on A."""
    prev, ev_prev, outs = None, None, []
    for i in range(steps + 1):
        if i < steps:
            with torch.cuda.stream(s_a):
                d = embed()
                ev = torch.cuda.Event()
                ev.record(s_a)
        if prev is not None:
            with torch.cuda.stream(s_b):
                s_b.wait_event(ev_prev)
                prev.record_stream(s_b)  # not reused by stream A's allocations while B reads it
                outs.append(rank(prev, ws2 if (i & 1) else ws))
        if i < steps:
            prev, ev_prev = d, ev
    return outs


pipelined(2)
torch.cuda.synchronize()
t = time.perf_counter()
outs = pipelined(REPS)
torch.cuda.synchronize()
t_pipe = (time.perf_counter() - t) / REPS * 1e3
same = all(torch.equal(o[1], ref_i) and torch.equal(o[0], ref_s) for o in outs)
print(f"B={B}: embed {t_embed:.2f} ms + rank {t_rank:.2f} ms = {t_embed + t_rank:.2f} ms serial; "
      f"pipelined on two streams {t_pipe:.2f} ms per step ({B / t_pipe * 1e3:.0f} images/s vs "
      f"{B / (t_embed + t_rank) * 1e3:.0f}); results identical: {same}", flush=True)
