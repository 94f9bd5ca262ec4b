"""Interleaved A/B of the split-bf16 (s3) and f16x2 (h2) conv cores on the
R101 layer shapes, then the whole R101 trunk, in one process:
per shape the median ms of each core and the max |difference| of the outputs.
usage: h2_ab.py [B] [--layers-only|--trunk-only]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402
from research_image_retrieval_amd.networks import ResNet  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
B = int(args[0]) if args else 1280
dev = torch.device("cuda:0")
SHAPES = [  # (h, cin, cout, k, stride, residual, count in R101)
    (56, 64, 64, 3, 1, 0, 3), (56, 64, 256, 1, 1, 1, 3), (56, 256, 64, 1, 1, 0, 2), (28, 128, 128, 3, 1, 0, 3),
    (28, 128, 512, 1, 1, 1, 4), (28, 512, 128, 1, 1, 0, 3), (14, 256, 1024, 1, 1, 1, 23), (14, 1024, 256, 1, 1, 0, 22),
    (14, 256, 256, 3, 1, 0, 22), (7, 512, 2048, 1, 1, 1, 3), (7, 2048, 512, 1, 1, 0, 2), (7, 512, 512, 3, 1, 0, 2),
]


def timed(fn, reps=5):
    fn()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        y = fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / reps, y


if "--trunk-only" not in sys.argv:
    tot = {"s3": 0.0, "h2": 0.0}
    for h, cin, cout, k, s, res, cnt in SHAPES:
        p = k // 2
        x = torch.relu(torch.randn(B, h, h, cin, device=dev))
        w = torch.randn(cout, k, k, cin, device=dev) * (2.0 / (k * k * cin)) ** 0.5
        bias = torch.randn(cout, device=dev) * 0.1
        oh = (h + 2 * p - k) // s + 1
        r = torch.randn(B, oh, oh, cout, device=dev) if res else None
        w3, wc = ops.split3_bf16(w), ops.H2Conv(w)
        rec = ops.amax_records(2, dev)
        ops.amax_f32(x, rec[0])
        fns = {"s3": lambda: ops.conv2d_s3(x, w3, bias, s, p, r, True),
               "h2": lambda: ops.conv2d_h2(x, rec[0], wc, bias, s, p, r, True, rec[1])}
        times, outs = {"s3": [], "h2": []}, {}
        for _ in range(5):
            for kname in ("s3", "h2"):
                t, outs[kname] = timed(fns[kname])
                times[kname].append(t)
        fl = 2.0 * B * oh * oh * cout * k * k * cin
        ma, mb = statistics.median(times["s3"]), statistics.median(times["h2"])
        tot["s3"] += ma * cnt
        tot["h2"] += mb * cnt
        d = (outs["s3"] - outs["h2"]).abs().max().item()
        print(f"h{h:3d} {cin:5d}->{cout:5d} k{k} s{s} r{res} x{cnt:2d}: s3 {ma:.3f} ms ({fl / ma / 1e9:.1f} TF/s) | "
              f"h2 {mb:.3f} ms ({fl / mb / 1e9:.1f} TF/s) | speedup {ma / mb:.3f} | max|diff| {d:.2e}", flush=True)
    print(f"weighted sum of these layers: s3 {tot['s3']:.2f} ms  h2 {tot['h2']:.2f} ms", flush=True)

if "--layers-only" not in sys.argv:
    x = torch.randn(B, 224, 224, 4, device=dev)
    x[..., 3] = 0
    nets = {m: ResNet("resnet101", seed=0, device=dev, conv_math=m) for m in ("s3", "h2")}
    times, outs = {"s3": [], "h2": []}, {}
    with torch.no_grad():
        for _ in range(3):
            for m in ("s3", "h2"):
                t, outs[m] = timed(lambda: nets[m].forward(x), reps=2)
                times[m].append(t)
    ma, mb = statistics.median(times["s3"]), statistics.median(times["h2"])
    d = (outs["s3"] - outs["h2"]).abs().max().item()
    print(f"R101 trunk B={B}: s3 {ma:.2f} ms  h2 {mb:.2f} ms  speedup {ma / mb:.3f}  max|diff| {d:.2e} "
          f"(max|y| {outs['s3'].abs().max().item():.3g})", flush=True)
