"""One layer3-shaped block seam at the bench batch, in a loop (for rocprofv3
kernel traces / PMC passes): the fused rr_bottleneck_seam_h2 and, with
SEAM_UNFUSED=1, the same two convs as rr_conv2d_h2 launches.
usage: [SEAM_P=256] [SEAM_HW=14] [SEAM_B=1280] [SEAM_REPS=10] [SEAM_UNFUSED=1] python tools/seam_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402

P = int(os.environ.get("SEAM_P", "256"))
HW = int(os.environ.get("SEAM_HW", "14"))
B = int(os.environ.get("SEAM_B", "1280"))
REPS = int(os.environ.get("SEAM_REPS", "10"))
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
y2 = torch.relu(torch.randn(B, HW, HW, P, device=dev, generator=g))
res = torch.relu(torch.randn(B, HW, HW, 4 * P, device=dev, generator=g))
c3 = ops.H2Conv(torch.randn(4 * P, 1, 1, P, device=dev, generator=g) * (2.0 / P) ** 0.5)
c1 = ops.H2Conv(torch.randn(P, 1, 1, 4 * P, device=dev, generator=g) * (2.0 / (4 * P)) ** 0.5)
b3 = torch.randn(4 * P, device=dev, generator=g) * 0.1
b1 = torch.randn(P, device=dev, generator=g) * 0.1
rec = ops.amax_records(4, dev)
ops.amax_f32(y2, rec[0])
M = B * HW * HW
byt = 4 * M * (P + 4 * P + 4 * P + P)


def fused():
    return ops.bottleneck_seam_h2(y2, rec[0], res, c3, b3, c1, b1, rec[1], rec[2])


def unfused():
    out = ops.conv2d_h2(y2, rec[0], c3, b3, 1, 0, res, True, rec[1])
    return out, ops.conv2d_h2(out, rec[1], c1, b1, 1, 0, None, True, rec[2])


if os.environ.get("SEAM_PHASES") == "1":
    import ctypes
    from research_image_retrieval_amd import _lib
    dbg = _lib.lib().rr_debug_seam_phases
    dbg.argtypes, dbg.restype = [ctypes.c_void_p], ctypes.c_int
    buf = (ctypes.c_ulonglong * 16)()
    fused()
    torch.cuda.synchronize()
    dbg(ctypes.cast(buf, ctypes.c_void_p))
    for _ in range(REPS):
        fused()
    torch.cuda.synchronize()
    dbg(ctypes.cast(buf, ctypes.c_void_p))
    names = ["conv3 mfma", "dma issue", "end wait", "barrier", "res wait+bar", "epi3", "conv1 mfma", "pro+epi1"]
    for role, nm in ((0, "residual waves"), (1, "loader waves")):
        v = [buf[8 * role + i] for i in range(8)]
        tot = sum(v)
        print(nm, " ".join(f"{names[i]} {v[i] / tot:.3f}" for i in range(8)), flush=True)
for name, fn in (("fused", fused), ("unfused", unfused)):
    if name == "unfused" and os.environ.get("SEAM_UNFUSED") != "1":
        continue
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(REPS):
        fn()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / REPS * 1e3
    print(f"{name}: P={P} {HW}x{HW} B={B}: {ms:.3f} ms per call, seam bytes {byt / 1e9:.2f} GB -> "
          f"{byt / ms / 1e6:.0f} GB/s", flush=True)
