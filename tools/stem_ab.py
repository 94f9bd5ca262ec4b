"""The ResNet stem at B images, 224x224: f16x2 conv + ReLU then the max-pool
(two launches) vs rr_stem_pool_h2 (one launch: the halo stem by default, the
implicit-GEMM config-7 stem with s3_cfg 7), interleaved, median ms; outputs
compared bit for bit.  usage: stem_ab.py [B]"""
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1280
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
x = F.pad(torch.randn(B, 224, 224, 3, device=dev, generator=g), (0, 1)).contiguous()
w = F.pad(torch.randn(64, 7, 7, 3, device=dev, generator=g) * (2.0 / 147) ** 0.5, (0, 1)).contiguous()
bias = torch.randn(64, device=dev, generator=g) * 0.1
wc = ops.H2Conv(w)
rec = ops.amax_records(2, dev)
ops.amax_f32(x, rec[0])


def two():
    return ops.maxpool2d(ops.conv2d_h2(x, rec[0], wc, bias, 2, 3, None, True, rec[1]), 3, 2, 1)


def one():
    return ops.stem_pool_h2(x, rec[0], wc, bias, 2, 3, rec[1])


def one_cfg7():
    with ops.tuning(0, s3_cfg=7):
        return ops.stem_pool_h2(x, rec[0], wc, bias, 2, 3, rec[1])


def timed(fn, reps=5):
    fn()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / reps


t = {"conv+maxpool": [], "stem_pool (halo)": [], "stem_pool (config 7)": []}
for _ in range(5):
    t["conv+maxpool"].append(timed(two))
    t["stem_pool (halo)"].append(timed(one))
    t["stem_pool (config 7)"].append(timed(one_cfg7))
same = torch.equal(two().view(torch.int32), one().view(torch.int32)) and \
    torch.equal(two().view(torch.int32), one_cfg7().view(torch.int32))
fl = 2.0 * B * 112 * 112 * 64 * 7 * 7 * 3
for k, v in t.items():
    m = statistics.median(v)
    print(f"{k}: {m:.3f} ms ({fl / m / 1e9:.0f} TF/s on the conv's 147-deep FLOPs)")
print("bit-identical:", same)
