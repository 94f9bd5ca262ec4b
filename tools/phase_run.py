"""Phase split of the f16x2 conv kernels' k-loops (diagnostic build,
tools/phase_build.sh): RR_LIB_PATH=ab/librr_phases.so python tools/phase_run.py [B]
Per R101 shape: ms, then each phase's share of the summed wave time (s_memtime
deltas): issue / MFMA part 1 / mid wait / split + MFMA part 2 / end wait /
barrier / epilogue / prologue."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import _lib, ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1280
dev = torch.device("cuda:0")
L = _lib.lib()
fn = L.rr_debug_phases
fn.argtypes = [ctypes.c_void_p]
fn.restype = ctypes.c_int
NAMES = ["issue", "mfma1", "wait_mid", "split+mfma2", "wait_end", "barrier", "epilogue", "prologue"]
# config 15 (gemm_s3q_kernel, kernel 2): its own phase map
NAMES_Q = ["issue+step0", "wait_mid", "split+step1", "wait_end+barrier", "epi_stage", "epi_res_wait", "epi_store",
           "prologue"]
# the halo tile (kernel 3)
NAMES_H = ["issue", "mfma", "wait_end", "barrier", "-", "-", "epilogue", "prologue"]
SHAPES = [(14, 256, 256, 3, 1, 0), (7, 512, 512, 3, 1, 0), (56, 64, 64, 3, 1, 0), (14, 256, 1024, 1, 1, 1),
          (14, 1024, 256, 1, 1, 0), (28, 128, 512, 1, 1, 1)]
buf = (ctypes.c_ulonglong * 32)()
for h, cin, cout, k, s, res in SHAPES:
    p = k // 2
    x = torch.relu(torch.randn(B, h, h, cin, device=dev))
    w = torch.randn(cout, k, k, cin, device=dev) * (2.0 / (k * k * cin)) ** 0.5
    bias = torch.randn(cout, device=dev) * 0.1
    oh = (h + 2 * p - k) // s + 1
    r = torch.randn(B, oh, oh, cout, device=dev) if res else None
    wc = ops.H2Conv(w)
    rec = ops.amax_records(2, dev)
    ops.amax_f32(x, rec[0])
    run = lambda: ops.conv2d_h2(x, rec[0], wc, bias, s, p, r, True, rec[1])  # noqa: E731
    run()
    torch.cuda.synchronize()
    fn(ctypes.cast(buf, ctypes.c_void_p))  # clear
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(3):
        run()
    en.record()
    torch.cuda.synchronize()
    fn(ctypes.cast(buf, ctypes.c_void_p))
    for kern in (0, 1, 2, 3):
        v = [buf[kern * 8 + i] for i in range(8)]
        tot = sum(v)
        if tot == 0:
            continue
        share = " ".join(f"{n} {x / tot:.3f}" for n, x in zip((NAMES, NAMES, NAMES_Q, NAMES_H)[kern], v))
        print(f"h{h} {cin}->{cout} k{k} r{res}: {st.elapsed_time(en) / 3:.3f} ms  "
              f"{('tile', 's3p', 's3q', 'halo')[kern]}: {share}", flush=True)
