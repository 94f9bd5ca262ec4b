"""Run one conv shape on a split core repeatedly (rocprofv3 counter passes).
usage: s3_one.py B H W Cin Cout K stride pad [res] [reps]   (RR_CORE=h2|s3, default h2)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402

b, h, w, cin, cout, k, s, p = (int(x) for x in sys.argv[1:9])
res = len(sys.argv) > 9 and sys.argv[9] == "1"
reps = int(sys.argv[10]) if len(sys.argv) > 10 else 20
dev = torch.device("cuda:0")
x = torch.relu(torch.randn(b, h, w, cin, device=dev))
wt = torch.randn(cout, k, k, cin, device=dev) * 0.01
bias = torch.randn(cout, device=dev)
oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
r = torch.randn(b, oh, ow, cout, device=dev) if res else None
if os.environ.get("RR_CORE", "h2") == "h2":
    wc = ops.H2Conv(wt)
    rec = ops.amax_records(2, dev)
    ops.amax_f32(x, rec[0])
    run = lambda: ops.conv2d_h2(x, rec[0], wc, bias, s, p, r, True, rec[1])  # noqa: E731
else:
    w3 = ops.split3_bf16(wt)
    run = lambda: ops.conv2d_s3(x, w3, bias, s, p, r, True)  # noqa: E731
for _ in range(3):
    run()
torch.cuda.synchronize()
st = torch.cuda.Event(enable_timing=True)
en = torch.cuda.Event(enable_timing=True)
st.record()
for _ in range(reps):
    run()
en.record()
torch.cuda.synchronize()
ms = st.elapsed_time(en) / reps
print({"ms": ms, "tflops": 2.0 * b * oh * ow * cout * k * k * cin / ms / 1e9})
