"""C4 attention core timing + output dump (A/B of two librr builds via
RR_LIB_PATH).  usage: attn_ab.py OUT.pt [B]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402

out_path = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1280
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
qkv = (torch.randn(B * 197, 3 * 768, device=dev, generator=g) * 2.0).bfloat16()
for _ in range(3):
    o = ops.attention_bf16(qkv, B, 197, 12)
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
st.record()
for _ in range(10):
    o = ops.attention_bf16(qkv, B, 197, 12)
en.record()
torch.cuda.synchronize()
print(f"attention_bf16 B={B}: {st.elapsed_time(en) / 10:.3f} ms per layer", flush=True)
torch.save(o[: 64 * 197].cpu(), out_path)
