"""ctypes binding of librr.so (include/rr.h).

The library is built in-tree (``make -C research_image_retrieval_amd/csrc``,
or ``__graft_entry__.build()``).  There is no fallback: if librr.so is missing
or cannot be loaded every op raises, so a GPU run can never silently take a
CPU or eager-PyTorch path.
"""
import ctypes
import os
import subprocess
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# RR_LIB_PATH: load an alternative build (A/B experiments on one device)
LIB_PATH = os.environ.get("RR_LIB_PATH") or os.path.join(_HERE, "librr.so")
CSRC = os.path.join(_HERE, "csrc")

RR_OK, RR_EINVAL, RR_EHIP, RR_EWORKSPACE, RR_EOVERFLOW = 0, -1, -2, -3, -4
ABI_VERSION = 6  # RR_ABI_VERSION of include/rr.h these signatures follow
AMAX_SLOTS = 64  # RR_AMAX_SLOTS

# timing classes (rr_timing_enable / rr_timing_collect)
TIME_COSINE, TIME_GEMM, TIME_SELECT, TIME_ELEM, TIME_COSINE_SEED, TIME_ATTN = 0, 1, 2, 3, 4, 5
# rr_set_tuning keys
# (6, 7 and 12 -- sweep_order, sweep_pf, lp_il -- were retired in ABI 5)
TUNE_GEMM_CFG, TUNE_GEMM_BK, TUNE_LP_CFG, TUNE_S3_CFG, TUNE_S3_STAGGER, \
    TUNE_SWEEP_MF16, TUNE_SWEEP_IL, TUNE_CONV_IL, TUNE_HALO_MF, TUNE_S3_CFG_RES, TUNE_SWEEP_FORM, TUNE_HALO_2D = \
    1, 2, 3, 4, 5, 8, 9, 10, 11, 13, 14, 15

_lib = None
_lock = threading.RLock()

_vp = ctypes.c_void_p
_i = ctypes.c_int
_ll = ctypes.c_longlong
_f = ctypes.c_float
_sz = ctypes.c_size_t

# name -> (restype, argtypes): exactly the symbols include/rr.h declares
SIGNATURES = {
    "rr_version": (ctypes.c_char_p, []),
    "rr_abi_version": (_i, []),
    "rr_create": (_i, [_i, ctypes.POINTER(_vp)]),
    "rr_destroy": (_i, [_vp]),
    "rr_last_error": (ctypes.c_char_p, [_vp]),
    "rr_timing_enable": (_i, [_vp, _i]),
    "rr_timing_collect": (_i, [_vp, _i, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_ll)]),
    "rr_get_device": (_i, [_vp, ctypes.POINTER(_i)]),
    "rr_set_tuning": (_i, [_vp, _i, _i]),
    "rr_cosine_topk_workspace_size": (_sz, [_i, _ll, _i, _i]),
    "rr_cosine_topk_workspace_size_cap": (_sz, [_i, _ll, _i, _i, _ll]),
    "rr_cosine_topk_cap_for": (_ll, [_i, _ll, _i, _i, _sz]),
    "rr_cosine_topk_counts_offset": (_sz, [_i, _ll, _i, _i]),
    "rr_cosine_topk_overflow_offset": (_sz, [_i, _ll, _i, _i]),
    "rr_cosine_topk": (_i, [_vp, _vp, _i, _vp, _ll, _i, _i, _ll, _vp, _vp, _vp, _sz, _vp]),
    "rr_cosine_scores": (_i, [_vp, _vp, _i, _vp, _ll, _i, _vp, _vp]),
    "rr_topk_merge": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp]),
    "rr_preprocess_u8": (_i, [_vp, _vp, _i, _i, _i, _vp, _vp, _vp, _vp]),
    "rr_nchw_to_nhwc": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp]),
    "rr_preprocess_u8_ex": (_i, [_vp, _vp, _i, _i, _i, _vp, _vp, _i, _vp, _vp]),
    "rr_nchw_to_nhwc_ex": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp, _vp]),
    "rr_conv2d": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _i, _i, _i, _i, _i, _vp, _i, _vp, _vp]),
    "rr_conv2d_h2": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _i, _i, _i, _i, _i, _vp, _i, _vp, _vp, _vp]),
    "rr_split2_f16": (_i, [_vp, _vp, _i, _i, _i, _vp, _vp, _vp]),
    "rr_stem_pool_h2": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _vp]),
    "rr_bottleneck_out_h2": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _i, _vp,
                                  _vp, _vp]),
    "rr_amax_f32": (_i, [_vp, _vp, _ll, _vp, _vp]),
    "rr_resize_bilinear": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _f, _f, _vp, _vp]),
    "rr_maxpool2d": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _i, _vp, _vp]),
    "rr_gem_pool": (_i, [_vp, _vp, _i, _i, _i, _f, _f, _vp, _vp]),
    "rr_linear": (_i, [_vp, _vp, _i, _i, _vp, _vp, _i, _vp, _vp]),
    "rr_l2_normalize": (_i, [_vp, _vp, _i, _i, _f, _vp, _vp]),
    "rr_linear_ex": (_i, [_vp, _vp, _i, _i, _vp, _vp, _i, _vp, _i, _vp, _vp]),
    "rr_layernorm": (_i, [_vp, _vp, _ll, _i, _i, _vp, _vp, _f, _vp, _vp]),
    "rr_patchify": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp, _vp]),
    "rr_vit_tokens": (_i, [_vp, _vp, _i, _i, _i, _vp, _vp, _vp, _vp]),
    "rr_patchify_ex": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp]),
    "rr_vit_tokens_ex": (_i, [_vp, _vp, _i, _i, _i, _vp, _vp, _vp, _vp, _f, _vp, _vp]),
    "rr_attention": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp]),
    "rr_attention_ex": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp, _vp]),
    "rr_attention_bf16": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp, _vp]),
    "rr_attention_bf16_qkv16": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp, _vp]),
    "rr_layernorm_ex": (_i, [_vp, _vp, _ll, _i, _i, _vp, _vp, _f, _i, _vp, _vp]),
    "rr_linear_bf16": (_i, [_vp, _vp, _i, _i, _vp, _vp, _i, _vp, _i, _i, _vp, _vp]),
    "rr_linear_bf16_ln": (_i, [_vp, _vp, _i, _i, _vp, _vp, _i, _vp, _i, _i, _vp, _vp, _vp, _f, _vp, _vp, _vp]),
    "rr_ln_partials_bf16": (_i, [_vp, _vp, _i, _i, _vp, _vp, _vp]),
    "rr_alpha_qe": (_i, [_vp, _vp, _i, _vp, _ll, _i, _vp, _vp, _i, _i, _f, _ll, _vp, _vp]),
    "rr_prefilter_gallery_bound": (_i, [_vp, _vp, _vp, _ll, _i, _vp, _vp]),
    "rr_cosine_topk_prefilter_workspace_size": (_sz, [_i, _ll, _i, _i]),
    "rr_cosine_topk_prefilter_counts_offset": (_sz, [_i, _ll, _i, _i]),
    "rr_cosine_topk_prefilter_overflow_offset": (_sz, [_i, _ll, _i, _i]),
    "rr_cosine_topk_prefilter_workspace_size_cap": (_sz, [_i, _ll, _i, _i, _ll]),
    "rr_cosine_topk_prefilter_cap_for": (_ll, [_i, _ll, _i, _i, _sz]),
    "rr_cosine_topk_prefilter": (_i, [_vp, _vp, _i, _vp, _vp, _vp, _ll, _i, _i, _ll, _vp, _vp, _vp, _sz, _vp]),
    "rr_pcaw_gram_workspace_size": (_sz, [_ll, _i]),
    "rr_pcaw_gram": (_i, [_vp, _vp, _ll, _i, _vp, _sz, _vp, _vp, _vp]),
    "rr_quantize_rows": (_i, [_vp, _vp, _ll, _i, _i, _vp, _vp, _vp]),
    "rr_cosine_topk_lp": (_i, [_vp, _vp, _vp, _i, _vp, _vp, _ll, _i, _i, _i, _ll, _vp, _vp, _vp, _sz, _vp]),
}


class RRError(RuntimeError):
    pass


def build(force=False):
    """Compile librr.so for gfx950 with hipcc (in-tree)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", CSRC, "-j4"], check=True)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RRError(
                    f"librr.so not found at {LIB_PATH}: build it with `make -C {CSRC}` "
                    "(there is deliberately no CPU/eager fallback)")
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                if os.environ.get("RR_LIB_PATH") and not hasattr(L, name):
                    continue  # A/B against an older build: bind what it has
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            if not os.environ.get("RR_LIB_PATH") and L.rr_abi_version() != ABI_VERSION:
                raise RRError(f"librr.so ABI {L.rr_abi_version()} != {ABI_VERSION} this binding was written "
                              f"against: rebuild it with `make -C {CSRC}`")
            _lib = L
    return _lib


_handles = {}


def handle(device_index):
    """Per-device librr handle (created once)."""
    h = _handles.get(device_index)
    if h is None:
        with _lock:
            h = _handles.get(device_index)
            if h is None:
                out = _vp()
                rc = lib().rr_create(int(device_index), ctypes.byref(out))
                if rc != RR_OK:
                    raise RRError(f"rr_create(device={device_index}) failed with {rc}")
                h = out.value
                _handles[device_index] = h
    return h


def check(rc, h, what):
    if rc != RR_OK:
        msg = lib().rr_last_error(h)
        raise RRError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
