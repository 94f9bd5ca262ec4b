"""Stem conv (7x7/2, NHWC4, 64 out) at B images: exact-fp32 core vs the
split-bf16 core, timed in one process.  usage: stem_ab.py [B]"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 320
dev = torch.device("cuda:0")
if os.environ.get("S3_CFG"):  # force one split-bf16 tile config (rr_set_tuning)
    ops.tuning(0, s3_cfg=int(os.environ["S3_CFG"])).__enter__()
x = F.pad(torch.randn(B, 224, 224, 3, device=dev), (0, 1)).contiguous()
w = F.pad(torch.randn(64, 7, 7, 3, device=dev) * 0.1, (0, 1)).contiguous()
b = torch.randn(64, device=dev)
w3p, shp = ops.split3_stem(w)
fns = {"f32": lambda: ops.conv2d(x, w, b, 2, 3, None, True),
       "s3": lambda: ops.conv2d_s3_stem(x, w3p, shp, b, 2, 3, True)}
for rnd in range(2):
    for name, fn in fns.items():
        for _ in range(3):
            fn()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(10):
            fn()
        en.record()
        torch.cuda.synchronize()
        ms = st.elapsed_time(en) / 10
        print(f"round {rnd} stem {name}: {ms:.3f} ms ({2 * B * 112 * 112 * 64 * 147 / ms / 1e9:.1f} TF/s algorithmic)",
              flush=True)
