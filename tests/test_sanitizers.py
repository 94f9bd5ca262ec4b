"""Sanitizer checks, host code only (the GPU pool runs no GPU
AddressSanitizer): the oracle's C restatement under ASan + UBSan, and librr's
C-ABI host logic (argument validation, workspace arithmetic, handle life
cycle) in a build whose host code carries -fsanitize=address
(tests/asan/build.sh).  The GPU half (`abi_check gpu`, real device calls
through the ASan build) is test_gpu_determinism.py's sanitizer test."""
import os
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "asan")
OUT = os.path.join(HERE, "out")
SOURCES = [os.path.join(HERE, f) for f in ("abi_check.cpp", "oracle_check.c", "build.sh")]


def ensure_built():
    """Build once (about a minute: librr's nine translation units in parallel)."""
    targets = [os.path.join(OUT, f) for f in ("oracle_check", "abi_check", "librr_asan.so")]
    csrc = os.path.join(os.path.dirname(HERE), "..", "research_image_retrieval_amd", "csrc")
    srcs = SOURCES + [os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith((".hip", ".hpp"))]
    srcs.append(os.path.join(os.path.dirname(HERE), "..", "oracle", "cosine_topk.c"))
    newest = max(os.path.getmtime(s) for s in srcs)
    if all(os.path.exists(t) and os.path.getmtime(t) >= newest for t in targets):
        return
    subprocess.run(["bash", os.path.join(HERE, "build.sh")], check=True, capture_output=True, timeout=900)


def _run(args, env_extra=None):
    env = dict(os.environ, **(env_extra or {}))
    r = subprocess.run(args, capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    return out


def test_oracle_under_asan_ubsan():
    ensure_built()
    assert "oracle_check: ok" in _run([os.path.join(OUT, "oracle_check")])


def test_librr_host_abi_under_asan():
    ensure_built()
    assert "abi_check cpu: ok" in _run([os.path.join(OUT, "abi_check")])
