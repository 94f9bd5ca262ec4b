"""Interleaved A/B of the persistent split-bf16 tile (config 8) against
config 4 on every dense (1x1 stride-1) R101 layer config 8 serves, at several
round-stagger values; checks the outputs are bit-identical.
usage: s3p_ab.py [B] [stagger,...]   e.g. s3p_ab.py 1280 8,0,16"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1280
STAG = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [-1]
# (h, cin, cout, residual+relu, count in R101)
SHAPES = [(14, 256, 1024, 1, 23), (14, 1024, 256, 0, 22), (56, 64, 256, 1, 3), (28, 128, 512, 1, 4),
          (7, 512, 2048, 1, 3), (7, 2048, 512, 0, 2), (28, 512, 256, 0, 1), (14, 1024, 512, 0, 1)]
dev = torch.device("cuda:0")
tot = {}
for h, cin, cout, res, cnt in SHAPES:
    x = torch.relu(torch.randn(B, h, h, cin, device=dev))
    w = torch.randn(cout, 1, 1, cin, device=dev) * (2.0 / cin) ** 0.5
    bias = torch.randn(cout, device=dev) * 0.1
    r = torch.randn(B, h, h, cout, device=dev) if res else None
    w3 = ops.split3_bf16(w)
    variants = [(4, -1)] + [(8, st) for st in STAG]
    times = {v: [] for v in variants}
    outs = {}
    for rep in range(7):
        for v in variants:
            with ops.tuning(0, s3_cfg=v[0], s3_stagger=v[1]):
                for _ in range(2):
                    ops.conv2d_s3(x, w3, bias, 1, 0, r, bool(res))
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(5):
                    y = ops.conv2d_s3(x, w3, bias, 1, 0, r, bool(res))
                en.record()
                torch.cuda.synchronize()
                times[v].append(st.elapsed_time(en) / 5)
                outs[v] = y
    fl = 2.0 * B * h * h * cout * cin
    line = f"h{h:3d} {cin:5d}->{cout:5d} r{res} x{cnt:2d}:"
    for v in variants:
        t = statistics.median(times[v])
        tot[v] = tot.get(v, 0.0) + t * cnt
        same = torch.equal(outs[v], outs[variants[0]])
        line += f" | cfg{v[0]} st{v[1]} {t:.3f} ms ({fl / t / 1e9:.0f} TF/s){'' if same else ' DIFF'}"
    print(line, flush=True)
print("weighted total (ms): " + " | ".join(f"cfg{v[0]} st{v[1]} {t:.2f}" for v, t in tot.items()), flush=True)
