"""Time the split-bf16 core on dense GEMMs with the FLOPs of the dominant R101
layers (M = 320*14*14).  usage: s3_lin.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda:0")
for m, k, n in ((62720, 2304, 256), (62720, 256, 1024), (62720, 1024, 256), (62720, 4608, 512)):
    x = torch.relu(torch.randn(m, k, device=dev))
    w3 = ops.split3_bf16(torch.randn(n, k, device=dev) * 0.02)
    for _ in range(3):
        ops.linear_s3(x, w3)
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    st.record()
    for _ in range(reps):
        ops.linear_s3(x, w3)
    en.record()
    torch.cuda.synchronize()
    ms = st.elapsed_time(en) / reps
    print(f"{m}x{k}x{n}: {ms:.3f} ms {2.0 * m * n * k / ms / 1e9:.1f} TF/s (ablate={os.environ.get('RR_S3_ABLATE', '0')}, "
          f"pipe={os.environ.get('RR_S3_PIPE', '0')})", flush=True)
