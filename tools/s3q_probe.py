"""Forced s3_cfg values on the residual-expansion shape (256->1024 + residual
at 14x14): bit-identity against config 12 over repeated runs, then ms per
launch.  (Round 5 ran it on a probe build with configs 16-20 -- config 15
with sc1 output stores / nt residual loads / wait counts excluding stores,
profiles/r05j_probe*.txt; those variants were removed after it.)
usage: python tools/s3q_probe.py [B] [cfgs, default 15]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1280
CFGS = [int(c) for c in (sys.argv[2] if len(sys.argv) > 2 else "15").split(",")]
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(3)
x = torch.relu(torch.randn(B, 14, 14, 256, device=dev, generator=g))
w = torch.randn(1024, 1, 1, 256, device=dev, generator=g) * (2.0 / 256) ** 0.5
bias = torch.randn(1024, device=dev, generator=g) * 0.1
r = torch.randn(B, 14, 14, 1024, device=dev, generator=g)
wc = ops.H2Conv(w)
rec = ops.amax_records(2, dev)
ops.amax_f32(x, rec[0])
run = lambda: ops.conv2d_h2(x, rec[0], wc, bias, 1, 0, r, True, rec[1])  # noqa: E731
with ops.tuning(0, s3_cfg=12):
    ref = run()
for c in CFGS:
    bad = 0
    with ops.tuning(0, s3_cfg=c):
        for _ in range(6):
            y = run()
            bad += int((y != ref).sum())
    print(f"cfg {c}: mismatching elements over 6 runs: {bad}", flush=True)
times = {c: [] for c in CFGS}
for _ in range(5):
    for c in CFGS:
        with ops.tuning(0, s3_cfg=c):
            run()
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(5):
                run()
            en.record()
            torch.cuda.synchronize()
            times[c].append(st.elapsed_time(en) / 5)
for c in CFGS:
    print(f"cfg {c}: median {statistics.median(times[c]):.4f} ms  all {['%.4f' % v for v in times[c]]}", flush=True)
