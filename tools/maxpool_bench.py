"""Time rr_maxpool2d on the R101 stem output at the bench batch (1280 x 112 x
112 x 64, 3x3/2 pad 1): algorithmic bytes 4.1 GB read + 1.03 GB write."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1280
x = torch.relu(torch.randn(B, 112, 112, 64, device="cuda"))
for _ in range(3):
    y = ops.maxpool2d(x, 3, 2, 1)
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
st.record()
for _ in range(10):
    y = ops.maxpool2d(x, 3, 2, 1)
en.record()
torch.cuda.synchronize()
ms = st.elapsed_time(en) / 10
gb = (x.numel() + y.numel()) * 4 / 1e9
print(f"maxpool {B}x112x112x64: {ms:.3f} ms, {gb / ms:.2f} TB/s algorithmic", flush=True)
