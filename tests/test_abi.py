"""The C-ABI library loads and exports every symbol include/rr.h declares
(no compute calls: CPU-only container)."""
import ctypes
import os
import re

from research_image_retrieval_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "rr.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(rr_[a-z0-9_]+)\s*\(", txt)))


def test_header_matches_binding_table():
    assert header_symbols() == sorted(_lib.SIGNATURES)


def test_library_exports_all_symbols():
    L = ctypes.CDLL(_lib.LIB_PATH)
    for name in header_symbols():
        assert hasattr(L, name), name
    assert b"gfx950" in _lib.lib().rr_version()


def test_library_is_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_no_device_calls_error_cleanly_without_gpu():
    # null handle -> RR_EINVAL, never a crash
    L = _lib.lib()
    assert L.rr_conv2d(None, None, 0, 0, 0, 0, None, None, 0, 0, 0, 0, 0, None, 0, None, None) == _lib.RR_EINVAL
    assert L.rr_timing_enable(None, 1) == _lib.RR_EINVAL
    assert L.rr_cosine_topk_workspace_size(256, 1_600_000, 2048, 100) >= 256 * (1_600_000 - 32768 + 100) * 8


def test_handle_entry_points_without_gpu():
    """Tuning / device queries reject a null handle; rr_create refuses a device
    that does not exist (here: any, since this container has no GPU)."""
    L = _lib.lib()
    dev = ctypes.c_int(-7)
    assert L.rr_get_device(None, ctypes.byref(dev)) == _lib.RR_EINVAL and dev.value == -7
    assert L.rr_set_tuning(None, _lib.TUNE_S3_CFG, 1) == _lib.RR_EINVAL
    out = ctypes.c_void_p()
    assert L.rr_create(-1, ctypes.byref(out)) != _lib.RR_OK and not out.value
    assert L.rr_create(1 << 20, ctypes.byref(out)) != _lib.RR_OK and not out.value


def test_bounded_workspace_arithmetic():
    """Bounded ranker workspaces (rr.h): sizes grow with the candidate cap,
    the cap a workspace affords round-trips, the worst case caps at every row,
    and below k candidates per query nothing fits (0)."""
    L = _lib.lib()
    for kind, pre in (("exact", "rr_cosine_topk"), ("prefilter", "rr_cosine_topk_prefilter")):
        size = getattr(L, pre + "_workspace_size")
        size_cap = getattr(L, pre + "_workspace_size_cap")
        cap_for = getattr(L, pre + "_cap_for")
        cnt_off = getattr(L, pre + "_counts_offset")
        ovf_off = getattr(L, pre + "_overflow_offset")
        nq, n, d, k = 1280, 1_600_000, 2048, 100
        full = size(nq, n, d, k)
        lo = size_cap(nq, n, d, k, k)
        assert 0 < lo < full and size_cap(nq, n, d, k, k - 1) == 0
        worst = cap_for(nq, n, d, k, full)
        assert worst >= n - 32768 and size_cap(nq, n, d, k, worst) == full
        for cap in (k, 4096, 65_536, 1_000_000):
            b = size_cap(nq, n, d, k, cap)
            assert cap_for(nq, n, d, k, b) == cap and cap_for(nq, n, d, k, b + 255) == cap
            assert cap_for(nq, n, d, k, b - 1) < cap
            # nq * 8 not a divisor of 256: the rounding may leave room for a few more
            c5 = cap_for(5, n, d, k, size_cap(5, n, d, k, cap))
            assert cap <= c5 < cap + 7 and size_cap(5, n, d, k, c5) == size_cap(5, n, d, k, cap)
        assert cap_for(nq, n, d, k, lo - 1) < k
        # counts and the overflow flag sit before the candidate buffer: the same
        # offsets for every cap
        assert 0 < cnt_off(nq, n, d, k) < lo and 0 < ovf_off(nq, n, d, k) < lo
        # 2 GB instead of the ~16 GB worst case at the C3 shape
        assert cap_for(nq, n, d, k, 2 << 30) > 100_000


def test_conv_algorithmic_bytes_and_flops():
    """The conv class's roofline inputs (bench.py): R101 at 224x224 is 15.6
    GFLOP and ~164 MB of algorithmic activation bytes per image (input map,
    output, residual once each, fp32), plus the split weights once per launch."""
    from research_image_retrieval_amd import weights as W
    fl = W.resnet_conv_flops("resnet101", 224, 224)
    by1 = W.resnet_conv_bytes("resnet101", 224, 224, 1)
    by2 = W.resnet_conv_bytes("resnet101", 224, 224, 2)
    assert set(fl) == set(by1) and len(fl) == 104
    assert abs(sum(fl.values()) / 1e9 - 15.60) < 0.01
    act = sum(by2.values()) - sum(by1.values())          # per image (weights cancel)
    wts = sum(by1.values()) - act
    assert 160e6 < act < 170e6
    assert abs(wts - 6 * 42.4e6) < 6 * 1.0e6             # ~42.4 M conv parameters x 3 bf16 planes
    # a residual conv3 reads its identity: 56x56, 64 -> 256 with residual
    b = W.resnet_conv_bytes("resnet101", 224, 224, 1, weight_bytes=0)["layer1.1.conv3"]
    assert b == (56 * 56 * 64 + 2 * 56 * 56 * 256) * 4
