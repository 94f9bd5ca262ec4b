"""Residual expansions (the HBM-bound 1x1 convs with a residual, 25 % of the
C3 step) on the f16x2 core: (tile config, round stagger) pairs interleaved in
one process at B images, median ms, effective GB/s of the algorithmic bytes
and bit-identity of outputs between pairs of the same config.
usage: resid_ab.py [B] [cfg:stagger,...]   (default 0:-1,11:0,11:8,11:16)
(s3_cfg 0 = the library's pick, stagger -1 = the library's default)"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1280
PAIRS = [tuple(int(v) for v in p.split(":")) for p in
         (sys.argv[2] if len(sys.argv) > 2 else "0:-1,11:0,11:8,11:16").split(",")]
dev = torch.device("cuda:0")
SHAPES = [(56, 64, 256, 2), (28, 128, 512, 3), (14, 256, 1024, 22), (7, 512, 2048, 2)]  # (h, cin, cout, count)


def timed(fn, reps=4):
    fn()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / reps


tot = {p: 0.0 for p in PAIRS}
for h, cin, cout, cnt in SHAPES:
    x = torch.relu(torch.randn(B, h, h, cin, device=dev))
    w = torch.randn(cout, 1, 1, cin, device=dev) * (2.0 / cin) ** 0.5
    bias = torch.randn(cout, device=dev) * 0.1
    r = torch.randn(B, h, h, cout, device=dev)
    wc = ops.H2Conv(w)
    rec = ops.amax_records(2, dev)
    ops.amax_f32(x, rec[0])
    times = {p: [] for p in PAIRS}
    outs = {}
    for _ in range(3):
        for p in PAIRS:
            with ops.tuning(0, s3_cfg=p[0], s3_stagger=p[1]):
                times[p].append(timed(lambda: ops.conv2d_h2(x, rec[0], wc, bias, 1, 0, r, True, rec[1])))
                outs[p] = ops.conv2d_h2(x, rec[0], wc, bias, 1, 0, r, True, rec[1]).clone()
    byts = 4.0 * B * h * h * (cin + 2 * cout)
    med = {p: statistics.median(v) for p, v in times.items()}
    for p in PAIRS:
        tot[p] += med[p] * cnt
    same = {p: torch.equal(outs[p], outs[q]) for p in PAIRS for q in PAIRS if q[0] == p[0] and q != p}
    line = " | ".join(f"{p[0]}:{p[1]} {med[p]:.3f} ms {byts / med[p] / 1e6:5.0f} GB/s" for p in PAIRS)
    print(f"h{h:3d} {cin:5d}->{cout:5d} x{cnt:2d} | {line} | same-config outputs identical: {all(same.values())}",
          flush=True)
    del x, r, outs
print("weighted sums (ms): " + "  ".join(f"{p[0]}:{p[1]} {tot[p]:.2f}" for p in PAIRS))
