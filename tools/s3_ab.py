"""Interleaved A/B of two rr_set_tuning settings on the split-bf16 convs that
a setting affects: per shape, alternate the two settings REPS times each and
report the median ms and the max |difference| of the outputs.
usage: s3_ab.py KEY VA VB [B]   e.g. s3_ab.py s3_cfg 3 4 1280"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402

key, va, vb = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
B = int(sys.argv[4]) if len(sys.argv) > 4 else 1280
SHAPES = [(14, 256, 1024, 1, 1, 1), (14, 1024, 256, 1, 1, 0), (14, 256, 256, 3, 1, 0), (56, 64, 64, 3, 1, 0),
          (28, 128, 128, 3, 1, 0), (7, 512, 512, 3, 1, 0)]  # (h, cin, cout, k, stride, residual)
dev = torch.device("cuda:0")
for h, cin, cout, k, s, res in SHAPES:
    p = k // 2
    x = torch.relu(torch.randn(B, h, h, cin, device=dev))
    w = torch.randn(cout, k, k, cin, device=dev) * (2.0 / (k * k * cin)) ** 0.5
    bias = torch.randn(cout, device=dev) * 0.1
    oh = (h + 2 * p - k) // s + 1
    r = torch.randn(B, oh, oh, cout, device=dev) if res else None
    w3 = ops.split3_bf16(w)
    times = {va: [], vb: []}
    outs = {}
    for rep in range(7):
        for v in (va, vb):
            with ops.tuning(0, **{key: v}):
                for _ in range(2):
                    ops.conv2d_s3(x, w3, bias, s, p, r, True)
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(5):
                    y = ops.conv2d_s3(x, w3, bias, s, p, r, True)
                en.record()
                torch.cuda.synchronize()
                times[v].append(st.elapsed_time(en) / 5)
                outs[v] = y
    fl = 2.0 * B * oh * oh * cout * k * k * cin
    ma, mb = statistics.median(times[va]), statistics.median(times[vb])
    d = (outs[va] - outs[vb]).abs().max().item()
    print(f"h{h:3d} {cin:5d}->{cout:5d} k{k} s{s} r{res}: {key}={va} {ma:.3f} ms ({fl / ma / 1e9:.1f} TF/s) | "
          f"{key}={vb} {mb:.3f} ms ({fl / mb / 1e9:.1f} TF/s) | speedup {ma / mb:.3f} | max|diff| {d:.2e}", flush=True)
