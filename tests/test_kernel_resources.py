"""Every kernel in the built librr.so stays out of scratch memory.

The split cores run at the register file's edge (242-256 VGPRs at two waves
per SIMD) and load through inline asm whose registers the compiler does not
track (gemm_s3.hip): a spill of such a register before its counted wait would
read an unloaded value.  This reads the gfx950 code-object metadata of the
library that ships (tools/kernel_resources.py) and fails if any kernel has a
private segment (scratch) -- no GPU needed."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "research_image_retrieval_amd", "librr.so")


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-readelf"), reason="ROCm llvm tools absent")
def test_no_kernel_uses_scratch():
    if not os.path.exists(LIB):
        pytest.fail("librr.so missing: build it first (make -C research_image_retrieval_amd/csrc)")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kernel_resources.py"), "--check", LIB],
                       capture_output=True, text=True, timeout=120)
    bad = [ln for ln in r.stdout.splitlines() if " scratch " in ln and not ln.split(" scratch ")[1].strip().startswith("0 ")]
    assert r.returncode == 0, "kernels using scratch:\n" + "\n".join(bad) + "\n" + r.stderr[-500:]
    # the split-core kernels are all there (f16x2 and bf16x3, persistent and tiled)
    for name in ("gemm_s3p_kernel<", "gemm_s3_kernel<", "split2h_kernel", "amax_kernel"):
        assert name in r.stdout, name
