"""HBM rate of the residual expansions' read/write mix without MFMAs: at
1280 images x 14 x 14, read the 256-channel A rows and the 1024-channel
residual and write the 1024-channel output (2.31 GB per pass, 44 % writes),
as PyTorch elementwise kernels; beside it a pure stream read and a pure
copy.  Median GB/s over repeats.  usage: hbm_mix.py [B]"""
import statistics
import sys

import torch

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1280
dev = torch.device("cuda:0")
M = B * 14 * 14
a = torch.randn(M, 256, device=dev)
r = torch.randn(M, 1024, device=dev)
y = torch.empty(M, 1024, device=dev)
s = torch.empty(M, device=dev)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        fn()
        en.record()
        torch.cuda.synchronize()
        ts.append(st.elapsed_time(en))
    return statistics.median(ts)


def mix():  # y = relu(r + a (tiled to 1024 columns)): reads a + r, writes y
    torch.add(r.view(M, 4, 256), a.view(M, 1, 256), out=y.view(M, 4, 256))
    torch.relu_(y)


cases = {
    "read r (sum)": (lambda: torch.sum(r, dim=1, out=s), 4.0 * M * 1024),
    "copy r -> y": (lambda: y.copy_(r), 8.0 * M * 1024),
    "residual mix: read a + r, write y (+ in-place ReLU pass)": (mix, 4.0 * M * (256 + 1024 + 1024) + 8.0 * M * 1024),
}
for k, (fn, by) in cases.items():
    ms = timed(fn)
    print(f"{k}: {ms:.3f} ms, {by / ms / 1e6:.0f} GB/s")
