"""One bf16 linear (the GEMM core's stored-C path, as the ViT uses it) run
REPS times, for rocprofv3 counter passes (tools/lp_pmc.sh).
usage: python tools/lp_one.py M K N act out_bf16 residual reps   (act 2 = QuickGELU)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402

m, k, n, act, obf, res, reps = (int(v) for v in sys.argv[1:8])
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
x = (torch.randn(m, k, device=dev, generator=g) * 0.5).to(torch.bfloat16)
w = (torch.randn(n, k, device=dev, generator=g) / k ** 0.5).to(torch.bfloat16)
b = torch.randn(n, device=dev, generator=g)
r = torch.randn(m, n, device=dev, generator=g) if res else None
if os.environ.get("LP_CFG"):
    ops.tuning(0, lp_cfg=int(os.environ["LP_CFG"])).__enter__()
for _ in range(reps):
    ops.linear_bf16(x, w, b, residual=r, act=act, out_bf16=bool(obf))
torch.cuda.synchronize()
print("done", m, k, n)
