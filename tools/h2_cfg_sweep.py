"""Every f16x2 tile config forced on every R101 conv shape at B images
(rr_set_tuning s3_cfg; 0 = the library's pick), interleaved rounds in one
process: median ms and TF/s per (shape, config), the fastest marked.
usage: h2_cfg_sweep.py [B] [cfgs, default 0,3,4,7,8; a trailing "i" adds conv_il=1, e.g. 0,0i]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1280
CFGS = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "3", "4", "7", "8"]


def tune(c):
    """config spec -> rr_set_tuning keys: "12" = s3_cfg 12, "12i" = with conv_il 1"""
    return {"s3_cfg": int(c.rstrip("i")), "conv_il": 1 if c.endswith("i") else 0}
dev = torch.device("cuda:0")
SHAPES = [  # (h, cin, cout, k, stride, residual, count in R101)
    (56, 64, 64, 3, 1, 0, 3), (56, 64, 256, 1, 1, 1, 2), (56, 256, 64, 1, 1, 0, 2), (56, 64, 64, 1, 1, 0, 1),
    (56, 256, 128, 1, 1, 0, 1), (56, 128, 128, 3, 2, 0, 1),
    (28, 128, 128, 3, 1, 0, 3), (28, 128, 512, 1, 1, 1, 3), (28, 512, 128, 1, 1, 0, 3), (28, 512, 256, 1, 1, 0, 1),
    (28, 256, 256, 3, 2, 0, 1),
    (14, 256, 1024, 1, 1, 1, 22), (14, 1024, 256, 1, 1, 0, 22), (14, 256, 256, 3, 1, 0, 22),
    (14, 1024, 512, 1, 1, 0, 1), (14, 512, 512, 3, 2, 0, 1),
    (7, 512, 2048, 1, 1, 1, 2), (7, 2048, 512, 1, 1, 0, 2), (7, 512, 512, 3, 1, 0, 2),
]


def timed(fn, reps=4):
    fn()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / reps


tot = {c: 0.0 for c in CFGS}
best_tot = 0.0
for h, cin, cout, k, s, res, cnt in SHAPES:
    p = k // 2
    x = torch.relu(torch.randn(B, h, h, cin, device=dev))
    w = torch.randn(cout, k, k, cin, device=dev) * (2.0 / (k * k * cin)) ** 0.5
    bias = torch.randn(cout, device=dev) * 0.1
    oh = (h + 2 * p - k) // s + 1
    r = torch.randn(B, oh, oh, cout, device=dev) if res else None
    wc = ops.H2Conv(w)
    rec = ops.amax_records(2, dev)
    ops.amax_f32(x, rec[0])
    times = {c: [] for c in CFGS}
    for _ in range(3):
        for c in CFGS:
            with ops.tuning(0, **tune(c)):
                times[c].append(timed(lambda: ops.conv2d_h2(x, rec[0], wc, bias, s, p, r, True, rec[1])))
    fl = 2.0 * B * oh * oh * cout * k * k * cin
    med = {c: statistics.median(v) for c, v in times.items()}
    bc = min(med, key=med.get)
    for c in CFGS:
        tot[c] += med[c] * cnt
    best_tot += med[bc] * cnt
    line = " | ".join(f"{c}: {med[c]:.3f}{'*' if c == bc else ' '}" for c in CFGS)
    print(f"h{h:3d} {cin:5d}->{cout:5d} k{k} s{s} r{res} x{cnt:2d} ({fl / med[bc] / 1e9:6.1f} TF/s best) | {line}",
          flush=True)
print("weighted sums (ms): " + "  ".join(f"cfg {c}: {tot[c]:.2f}" for c in CFGS) + f"  best-per-layer: {best_tot:.2f}")
