"""A/B of the C3 trunk's batch split across HIP streams (networks
forward_test_u8_streams) against the one-stream batch: ms per 1280-image
embed, and bit-identity of the split schedule to the same parts run one
after another.  Usage: python tools/overlap_ab.py [reps]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda:0")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
B = int(os.environ.get("OV_BATCH", "1280"))
net = bench.build_extractor("resnet101", dev)
rs = np.random.RandomState(1234)
imgs = torch.from_numpy(rs.randint(0, 256, size=(B, 224, 224, 3), dtype=np.uint8)).to(dev)
streams = [torch.cuda.Stream(dev) for _ in range(4)]


def timed(fn):
    fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t.append((time.perf_counter() - t0) * 1e3)
    return min(t), float(np.median(t))


def serial(parts):
    cuts = [B * i // parts for i in range(parts + 1)]
    return torch.cat([net.forward_test_u8(imgs[cuts[i]:cuts[i + 1]]) for i in range(parts)])


print("one stream, whole batch  min %.2f med %.2f ms" % timed(lambda: net.forward_test_u8(imgs)), flush=True)
print("one stream, 2 parts      min %.2f med %.2f ms" % timed(lambda: serial(2)), flush=True)
ref2 = serial(2)
ref3 = serial(3)
full = net.forward_test_u8(imgs)
cases = [(2, l, 0) for l in (0, 1, 2, 3, 4, 6, 9)] + [(3, 1, 0), (3, 3, 0)]
for parts, lag, share in cases:
    f = lambda: net.forward_test_u8_streams(imgs, streams[:parts], lag=lag)  # noqa: E731
    mn, md = timed(f)
    out = f()
    ref = ref2 if parts == 2 else (ref3 if parts == 3 else serial(parts))
    same = torch.equal(out.view(torch.int32), ref.view(torch.int32))
    err = (out - full).abs().max().item()
    print(f"{parts} streams lag {lag:2d}  min {mn:.2f} med {md:.2f} ms  bit-identical to serial parts: {same}  "
          f"max |d - whole batch| {err:.2e}", flush=True)
