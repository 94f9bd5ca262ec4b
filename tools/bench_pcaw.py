"""Time PCA-whitening learning's GPU half (rr_pcaw_gram) on a GLDv2-scale
descriptor set: n x d fp32 rows resident in HBM (default 1.6M x 2048).
Prints one JSON line: ms, achieved TFLOP/s on the algorithmic n*d*(d+1) FLOP of
the symmetric Gram (upper triangle + diagonal), and the fraction of the fp32
MFMA peak."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import _lib, ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_600_000)
ap.add_argument("--d", type=int, default=2048)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn((a.n, a.d), generator=g, device=dev)
ops.pcaw_gram(x[:4096].contiguous())
timer = ops.KernelTimer(0)
timer.enable(True)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.reps):
    mean, gram = ops.pcaw_gram(x)
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) / a.reps * 1e3
gemm_ms = timer.collect(_lib.TIME_GEMM)[0] / a.reps
elem_ms = timer.collect(_lib.TIME_ELEM)[0] / a.reps
timer.enable(False)
flop = float(a.n) * a.d * (a.d + 1)
print(json.dumps({"what": "rr_pcaw_gram", "n": a.n, "d": a.d, "ms": round(ms, 3),
                  "gemm_ms": round(gemm_ms, 3), "elementwise_ms": round(elem_ms, 3),
                  "tflops_end_to_end": round(flop / ms / 1e9, 2), "tflops_gemm": round(flop / gemm_ms / 1e9, 2),
                  "frac_fp32_peak_gemm": round(flop / gemm_ms / 1e9 / 157.3, 4)}))
