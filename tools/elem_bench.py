"""Elementwise kernels of the C4 ViT step at 1280 images (M = 252160 tokens x
768): LayerNorm -> bf16 (twice per block), achieved HBM bandwidth."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402


def t_ms(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


dev = torch.device("cuda:0")
m, d = int(os.environ.get("LP_B", "1280")) * 197, 768
x = torch.randn(m, d, device=dev)
gm, bt = torch.randn(d, device=dev), torch.randn(d, device=dev)
ms = t_ms(lambda: ops.layernorm_bf16(x, gm, bt))
by = m * d * 4 + m * d * 2
print(f"layernorm_bf16 {m}x{d}: {ms:.4f} ms, {by / ms / 1e6:.0f} GB/s")
ms = t_ms(lambda: ops.layernorm(x, gm, bt))
by = m * d * 8
print(f"layernorm fp32 {m}x{d}: {ms:.4f} ms, {by / ms / 1e6:.0f} GB/s")
y = torch.empty_like(x)
ms = t_ms(lambda: y.copy_(x))
print(f"torch copy fp32 {m}x{d}: {ms:.4f} ms, {m * d * 8 / ms / 1e6:.0f} GB/s")
