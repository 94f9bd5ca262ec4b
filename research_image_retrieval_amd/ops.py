"""Torch-tensor wrappers over the librr C-ABI (one function per rr_* entry).

PyTorch is used only for device memory and the current HIP stream; every op
below runs a hand-written gfx950 kernel from librr.so.  Inputs must be
contiguous fp32 (uint8 for images) tensors on a ROCm device.
"""
import ctypes

import torch

from . import _lib

_NULL = None


def _dev(t):
    if not t.is_cuda:
        raise ValueError("librr ops need ROCm device tensors (got a CPU tensor)")
    return t.device.index if t.device.index is not None else torch.cuda.current_device()


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _f32(t, name):
    if t.dtype != torch.float32:
        raise TypeError(f"{name}: expected float32, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    return t


def preprocess_u8(img_nhwc, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225), out_c=3):
    """uint8 [B,H,W,3] -> fp32 NHWC normalised (ToTensor + Normalize); out_c=4
    appends a zero channel (stem-conv tap layout)."""
    if img_nhwc.dtype != torch.uint8 or img_nhwc.dim() != 4 or img_nhwc.shape[3] != 3:
        raise ValueError("preprocess_u8: expected uint8 [B,H,W,3]")
    img_nhwc = img_nhwc.contiguous()
    dev = _dev(img_nhwc)
    b, h, w, _ = img_nhwc.shape
    out = torch.empty((b, h, w, out_c), dtype=torch.float32, device=img_nhwc.device)
    m = (ctypes.c_float * 3)(*mean)
    s = (ctypes.c_float * 3)(*std)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_preprocess_u8_ex(hd, _ptr(img_nhwc), b, h, w, ctypes.cast(m, ctypes.c_void_p),
                                              ctypes.cast(s, ctypes.c_void_p), int(out_c), _ptr(out), _stream(dev)),
               hd, "rr_preprocess_u8")
    return out


def nchw_to_nhwc(x, out_c=None):
    x = _f32(x.contiguous(), "nchw_to_nhwc")
    dev = _dev(x)
    b, c, h, w = x.shape
    oc = c if out_c is None else int(out_c)
    out = torch.empty((b, h, w, oc), dtype=torch.float32, device=x.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_nchw_to_nhwc_ex(hd, _ptr(x), b, c, h, w, oc, _ptr(out), _stream(dev)), hd,
               "rr_nchw_to_nhwc")
    return out


def conv2d(x, w, bias, stride=1, pad=0, residual=None, relu=False):
    """NHWC conv with fused bias/residual/ReLU; w is [Cout,KH,KW,Cin]."""
    _f32(x, "conv2d x")
    _f32(w, "conv2d w")
    dev = _dev(x)
    b, h, wd, cin = x.shape
    cout, kh, kw, cin_w = w.shape
    if cin_w != cin:
        raise ValueError(f"conv2d: Cin mismatch {cin} vs {cin_w}")
    oh = (h + 2 * pad - kh) // stride + 1
    ow = (wd + 2 * pad - kw) // stride + 1
    y = torch.empty((b, oh, ow, cout), dtype=torch.float32, device=x.device)
    if residual is not None:
        _f32(residual, "conv2d residual")
        if tuple(residual.shape) != tuple(y.shape):
            raise ValueError("conv2d: residual shape mismatch")
    if bias is not None:
        _f32(bias, "conv2d bias")
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_conv2d(hd, _ptr(x), b, h, wd, cin, _ptr(w), _ptr(bias), cout, kh, kw, stride, pad,
                                    _ptr(residual), int(relu), _ptr(y), _stream(dev)), hd, "rr_conv2d")
    return y


AMAX_SLOTS = 64  # RR_AMAX_SLOTS: words of one tensor's max-|x| record


def amax_records(n, device):
    """n zeroed max-|x| records [n, RR_AMAX_SLOTS] (int32 words holding float
    bits) for rr_conv2d_h2's x_amax / y_amax."""
    return torch.zeros((n, AMAX_SLOTS), dtype=torch.int32, device=device)


def amax_f32(x, record):
    """Fold max |x| (finite values) into a zeroed record (rr_amax_f32)."""
    x = _f32(x.contiguous(), "amax_f32")
    if record.dtype != torch.int32 or record.numel() != AMAX_SLOTS or not record.is_contiguous():
        raise ValueError("amax_f32: record must be contiguous int32 [RR_AMAX_SLOTS]")
    dev = _dev(x)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_amax_f32(hd, _ptr(x), x.numel(), _ptr(record), _stream(dev)), hd, "rr_amax_f32")
    return record


def amax_value(record):
    """The max a record holds, as a Python float (host read: tests, tools)."""
    return float(record.view(torch.float32).max().item())


def split2_f16(w, kpad=None):
    """fp16 x2 split of the rows of w ([N, K] or [Cout, KH, KW, Cin]) at a
    per-row power-of-two scale (rr_split2_f16): returns (planes int16 [2, N,
    kpad] of fp16 bit patterns, zero past K; iscale fp32 [N] = 2^-e_n)."""
    w = _f32(w.contiguous(), "split2_f16")
    dev = _dev(w)
    rows = w.shape[0]
    k = w.numel() // max(rows, 1)
    kpad = k if kpad is None else int(kpad)
    if kpad < k:
        raise ValueError("split2_f16: kpad < K")
    planes = torch.empty((2, rows, kpad), dtype=torch.int16, device=w.device)
    iscale = torch.empty((rows,), dtype=torch.float32, device=w.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_split2_f16(hd, _ptr(w), rows, k, kpad, _ptr(planes), _ptr(iscale), _stream(dev)), hd,
               "rr_split2_f16")
    return planes, iscale


class H2Conv:
    """Weights of one conv on the f16x2 split core: planes [2, Cout, Kp],
    inverse row scales [Cout], filter (KH, KW, Cin).  Cin == 4 is the NHWC4
    stem (K = KH*KW*4 zero-padded to a multiple of 32)."""

    def __init__(self, w):
        w = _f32(w.contiguous(), "H2Conv")
        cout, kh, kw, cin = w.shape
        if cin % 32 and cin != 4:
            raise ValueError("H2Conv: Cin must be a multiple of 32, or 4 (NHWC4 stem)")
        k = kh * kw * cin
        self.kpad = (k + 31) // 32 * 32 if cin == 4 else k
        self.planes, self.iscale = split2_f16(w.reshape(cout, k), self.kpad)
        self.cout, self.kh, self.kw, self.cin = cout, kh, kw, cin


def conv2d_h2(x, x_amax, wc, bias, stride=1, pad=0, residual=None, relu=False, y_amax=None):
    """conv2d on the f16x2 split core (rr_conv2d_h2): fp32-accurate, wc an
    H2Conv, x_amax the max-|x| record of x; y_amax (optional, zeroed) gets
    max |y| for the next conv."""
    _f32(x, "conv2d_h2 x")
    if not isinstance(wc, H2Conv):
        raise TypeError("conv2d_h2: wc must be an ops.H2Conv")
    dev = _dev(x)
    b, h, wd, cin = x.shape
    if cin != wc.cin:
        raise ValueError(f"conv2d_h2: Cin mismatch {cin} vs {wc.cin}")
    for r, nm in ((x_amax, "x_amax"), (y_amax, "y_amax")):
        if r is not None and (r.dtype != torch.int32 or r.numel() != AMAX_SLOTS or not r.is_contiguous()):
            raise ValueError(f"conv2d_h2: {nm} must be a contiguous int32 [RR_AMAX_SLOTS] record")
    oh = (h + 2 * pad - wc.kh) // stride + 1
    ow = (wd + 2 * pad - wc.kw) // stride + 1
    y = torch.empty((b, oh, ow, wc.cout), dtype=torch.float32, device=x.device)
    if residual is not None:
        _f32(residual, "conv2d_h2 residual")
        if tuple(residual.shape) != tuple(y.shape):
            raise ValueError("conv2d_h2: residual shape mismatch")
    if bias is not None:
        _f32(bias, "conv2d_h2 bias")
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_conv2d_h2(hd, _ptr(x), _ptr(x_amax), b, h, wd, cin, _ptr(wc.planes), _ptr(wc.iscale),
                                       _ptr(bias), wc.cout, wc.kh, wc.kw, stride, pad, _ptr(residual), int(relu),
                                       _ptr(y), _ptr(y_amax), _stream(dev)), hd, "rr_conv2d_h2")
    return y


def stem_pool_h2(x, x_amax, wc, bias, stride=2, pad=3, y_amax=None):
    """The NHWC4 stem conv + bias + ReLU with the 3x3/2 padding-1 max-pool
    fused (rr_stem_pool_h2): [B,H,W,4] -> pooled [B,PH,PW,64], the same bits
    as conv2d_h2(..., relu=True) followed by maxpool2d for finite inputs."""
    _f32(x, "stem_pool_h2 x")
    if not isinstance(wc, H2Conv) or wc.cin != 4 or wc.cout != 64:
        raise TypeError("stem_pool_h2: wc must be an ops.H2Conv with Cin 4 and Cout 64")
    dev = _dev(x)
    b, h, wd, cin = x.shape
    if cin != 4:
        raise ValueError("stem_pool_h2: x must be NHWC4")
    oh = (h + 2 * pad - wc.kh) // stride + 1
    ow = (wd + 2 * pad - wc.kw) // stride + 1
    y = torch.empty((b, (oh - 1) // 2 + 1, (ow - 1) // 2 + 1, 64), dtype=torch.float32, device=x.device)
    if bias is not None:
        _f32(bias, "stem_pool_h2 bias")
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_stem_pool_h2(hd, _ptr(x), _ptr(x_amax), b, h, wd, _ptr(wc.planes), _ptr(wc.iscale),
                                          _ptr(bias), 64, wc.kh, wc.kw, stride, pad, _ptr(y), _ptr(y_amax),
                                          _stream(dev)), hd, "rr_stem_pool_h2")
    return y


class H2Bottleneck:
    """Weights of a stage-entry bottleneck's conv3 + downsample projection as
    one f16x2 GEMM (rr_bottleneck_out_h2): rows [W3 | Wd] split together,
    bias = b3 + bd."""

    def __init__(self, w3, b3, wd, bd):
        w3, wd = _f32(w3.contiguous(), "H2Bottleneck w3"), _f32(wd.contiguous(), "H2Bottleneck wd")
        cout, planes = w3.shape[0], w3.numel() // w3.shape[0]
        cin = wd.numel() // wd.shape[0]
        if wd.shape[0] != cout or tuple(w3.shape[1:3]) != (1, 1) or tuple(wd.shape[1:3]) != (1, 1):
            raise ValueError("H2Bottleneck: 1x1 conv3 and downsample with the same Cout")
        self.planes, self.cin, self.cout = planes, cin, cout
        self.planes2, self.iscale = split2_f16(torch.cat([w3.reshape(cout, planes), wd.reshape(cout, cin)], 1))
        self.bias = (b3.double() + bd.double()).float().contiguous() if b3 is not None else bd.contiguous()


def bottleneck_out_h2(y, y_amax, x, x_amax, wb, stride, out_amax=None):
    """ReLU(conv3(y) + downsample(x)) of a stage-entry bottleneck as one f16x2
    GEMM (rr_bottleneck_out_h2): y [B,OH,OW,planes], x [B,H,W,cin]."""
    _f32(y, "bottleneck_out_h2 y")
    _f32(x, "bottleneck_out_h2 x")
    if not isinstance(wb, H2Bottleneck):
        raise TypeError("bottleneck_out_h2: wb must be an ops.H2Bottleneck")
    b, oh, ow, planes = y.shape
    bx, hx, wx, cin = x.shape
    if planes != wb.planes or cin != wb.cin or bx != b:
        raise ValueError("bottleneck_out_h2: shape mismatch")
    dev = _dev(y)
    out = torch.empty((b, oh, ow, wb.cout), dtype=torch.float32, device=y.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_bottleneck_out_h2(hd, _ptr(y), _ptr(y_amax), b, oh, ow, planes, _ptr(x), _ptr(x_amax),
                                               hx, wx, cin, int(stride), _ptr(wb.planes2), _ptr(wb.iscale),
                                               _ptr(wb.bias), wb.cout, _ptr(out), _ptr(out_amax), _stream(dev)),
               hd, "rr_bottleneck_out_h2")
    return out


def resize_bilinear(x_nhwc, out_h, out_w, scale_factor=None):
    """NHWC bilinear resize, align_corners=False.  With ``scale_factor`` the
    source index uses 1/scale_factor, as F.interpolate(scale_factor=s) does."""
    _f32(x_nhwc, "resize_bilinear")
    dev = _dev(x_nhwc)
    b, h, w, c = x_nhwc.shape
    y = torch.empty((b, out_h, out_w, c), dtype=torch.float32, device=x_nhwc.device)
    inv = 0.0 if scale_factor is None else float(1.0 / scale_factor)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_resize_bilinear(hd, _ptr(x_nhwc), b, h, w, c, int(out_h), int(out_w), inv, inv, _ptr(y),
                                             _stream(dev)), hd, "rr_resize_bilinear")
    return y


def maxpool2d(x, k=3, stride=2, pad=1):
    _f32(x, "maxpool2d")
    dev = _dev(x)
    b, h, w, c = x.shape
    oh = (h + 2 * pad - k) // stride + 1
    ow = (w + 2 * pad - k) // stride + 1
    y = torch.empty((b, oh, ow, c), dtype=torch.float32, device=x.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_maxpool2d(hd, _ptr(x), b, h, w, c, k, stride, pad, _ptr(y), _stream(dev)), hd,
               "rr_maxpool2d")
    return y


def gem_pool(x_nhwc, p=3.0, eps=1e-6):
    """[B,H,W,C] (or [B,HW,C]) -> [B,C] GeM."""
    _f32(x_nhwc, "gem_pool")
    dev = _dev(x_nhwc)
    b, c = x_nhwc.shape[0], x_nhwc.shape[-1]
    hw = x_nhwc.numel() // (b * c) if b * c else 0
    out = torch.empty((b, c), dtype=torch.float32, device=x_nhwc.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_gem_pool(hd, _ptr(x_nhwc), b, hw, c, float(p), float(eps), _ptr(out), _stream(dev)), hd,
               "rr_gem_pool")
    return out


def linear(x, w, bias=None):
    """y = x @ w.T + bias, x [M,K], w [N,K]."""
    _f32(x, "linear x")
    _f32(w, "linear w")
    dev = _dev(x)
    m, k = x.shape
    n = w.shape[0]
    y = torch.empty((m, n), dtype=torch.float32, device=x.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_linear(hd, _ptr(x), m, k, _ptr(w), _ptr(bias), n, _ptr(y), _stream(dev)), hd,
               "rr_linear")
    return y


def l2_normalize(x, eps=1e-12, out=None):
    _f32(x, "l2_normalize")
    dev = _dev(x)
    m, d = x.shape
    y = torch.empty_like(x) if out is None else out
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_l2_normalize(hd, _ptr(x), m, d, float(eps), _ptr(y), _stream(dev)), hd,
               "rr_l2_normalize")
    return y


def cosine_topk_workspace_size(nq, n, d, k):
    return int(_lib.lib().rr_cosine_topk_workspace_size(int(nq), int(n), int(d), int(k)))


# ---- bounded ranker workspaces (rr.h "Bounded workspaces") ----------------
# kind -> C functions: worst-case size, size for a cap, cap for a size,
# per-query counts offset, overflow-count offset
_WS_FUNCS = {
    "exact": ("rr_cosine_topk_workspace_size", "rr_cosine_topk_workspace_size_cap", "rr_cosine_topk_cap_for",
              "rr_cosine_topk_counts_offset", "rr_cosine_topk_overflow_offset"),
    "prefilter": ("rr_cosine_topk_prefilter_workspace_size", "rr_cosine_topk_prefilter_workspace_size_cap",
                  "rr_cosine_topk_prefilter_cap_for", "rr_cosine_topk_prefilter_counts_offset",
                  "rr_cosine_topk_prefilter_overflow_offset"),
}


def _wsf(kind, i):
    return getattr(_lib.lib(), _WS_FUNCS[kind][i])


def ranker_workspace_bounds(kind, nq, n, d, k):
    """(minimum bytes = a cap of k candidates per query, worst-case bytes) of
    a ranker workspace; kind 'exact' (cosine_topk / cosine_topk_lp) or
    'prefilter'."""
    a = (int(nq), int(n), int(d), int(k))
    return int(_wsf(kind, 1)(*a, int(k))), int(_wsf(kind, 0)(*a))


def _ranker_workspace(kind, nq, n, d, k, workspace, max_workspace_bytes, device):
    """The workspace a ranker call runs with: the caller's if large enough,
    else a new one of the worst-case size or, with max_workspace_bytes, of at
    most that many bytes (never below the k-candidate minimum).  Returns
    (workspace, bounded)."""
    lo, full = ranker_workspace_bounds(kind, nq, n, d, k)
    budget = full if max_workspace_bytes is None else max(lo, min(full, int(max_workspace_bytes)))
    if workspace is None or workspace.numel() < budget:
        workspace = torch.empty(budget, dtype=torch.uint8, device=device)
    return workspace, workspace.numel() < full


def _recover_overflow(kind, nq, n, d, k, workspace, rerun, os_, oi):
    """After a bounded-workspace call: re-run every query whose candidates
    overflowed the buffer (rr.h) with a worst-case workspace for just those
    queries, in chunks that fit the same workspace, and write their rows.
    rerun(query_index_tensor, workspace) -> (scores, idx).  One device->host
    read of the overflow count (a stream sync); returns the re-run count."""
    a = (int(nq), int(n), int(d), int(k))
    ovf_off = int(_wsf(kind, 4)(*a))
    if int(workspace[ovf_off:ovf_off + 4].view(torch.int32).item()) == 0:
        return 0
    cap = int(_wsf(kind, 2)(*a, workspace.numel()))
    cnt_off = int(_wsf(kind, 3)(*a))
    bad = torch.nonzero(workspace[cnt_off:cnt_off + 4 * int(nq)].view(torch.int32) > cap).flatten()
    c = max(1, bad.numel())
    while c > 1 and int(_wsf(kind, 0)(c, int(n), int(d), int(k))) > workspace.numel():
        c = (c + 1) // 2
    need = int(_wsf(kind, 0)(c, int(n), int(d), int(k)))
    ws = workspace if need <= workspace.numel() else torch.empty(need, dtype=torch.uint8, device=workspace.device)
    for part in bad.split(c):
        s_, i_ = rerun(part, ws)
        os_[part] = s_
        oi[part] = i_
    return int(bad.numel())


def cosine_topk(queries, gallery, k, idx_offset=0, workspace=None, max_workspace_bytes=None):
    """Exact stable top-k of queries [nq,D] against gallery [N,D] -> (scores [nq,k] fp32, idx [nq,k] int64).
    max_workspace_bytes: run with a bounded candidate buffer (rr.h) and re-run
    overflowed queries; results are identical either way."""
    _f32(queries, "cosine_topk queries")
    _f32(gallery, "cosine_topk gallery")
    dev = _dev(queries)
    nq, d = queries.shape
    n = gallery.shape[0]
    if gallery.shape[1] != d:
        raise ValueError("cosine_topk: descriptor dims differ")
    workspace, bounded = _ranker_workspace("exact", nq, n, d, k, workspace, max_workspace_bytes, queries.device)
    os_ = torch.empty((nq, k), dtype=torch.float32, device=queries.device)
    oi = torch.empty((nq, k), dtype=torch.int64, device=queries.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_cosine_topk(hd, _ptr(queries), nq, _ptr(gallery), n, d, k, int(idx_offset), _ptr(os_),
                                         _ptr(oi), _ptr(workspace), workspace.numel(), _stream(dev)), hd,
               "rr_cosine_topk")
    if bounded and nq > 0:
        _recover_overflow("exact", nq, n, d, k, workspace,
                          lambda r, ws: cosine_topk(queries[r].contiguous(), gallery, k, idx_offset, ws), os_, oi)
    return os_, oi


def cosine_scores(queries, gallery):
    """Dense scores, gallery-major [N, nq] (= similarity.T of iris_evaluate.py:383)."""
    _f32(queries, "cosine_scores queries")
    _f32(gallery, "cosine_scores gallery")
    dev = _dev(queries)
    nq, d = queries.shape
    n = gallery.shape[0]
    out = torch.empty((n, nq), dtype=torch.float32, device=queries.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_cosine_scores(hd, _ptr(queries), nq, _ptr(gallery), n, d, _ptr(out), _stream(dev)), hd,
               "rr_cosine_scores")
    return out


def topk_merge(part_scores, part_idx, k_out):
    """[P,nq,kin] partial lists -> stable top-k_out per query."""
    _f32(part_scores, "topk_merge scores")
    if part_idx.dtype != torch.int64 or not part_idx.is_contiguous():
        raise TypeError("topk_merge: idx must be contiguous int64")
    dev = _dev(part_scores)
    p, nq, kin = part_scores.shape
    os_ = torch.empty((nq, k_out), dtype=torch.float32, device=part_scores.device)
    oi = torch.empty((nq, k_out), dtype=torch.int64, device=part_scores.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_topk_merge(hd, _ptr(part_scores), _ptr(part_idx), p, nq, kin, k_out, _ptr(os_), _ptr(oi),
                                        _stream(dev)), hd, "rr_topk_merge")
    return os_, oi


_TUNE_KEYS = {"gemm_cfg": _lib.TUNE_GEMM_CFG, "gemm_bk": _lib.TUNE_GEMM_BK, "lp_cfg": _lib.TUNE_LP_CFG,
              "s3_cfg": _lib.TUNE_S3_CFG, "s3_stagger": _lib.TUNE_S3_STAGGER, "sweep_mf16": _lib.TUNE_SWEEP_MF16,
              "sweep_il": _lib.TUNE_SWEEP_IL, "conv_il": _lib.TUNE_CONV_IL,
              "halo_mf": _lib.TUNE_HALO_MF, "s3_cfg_res": _lib.TUNE_S3_CFG_RES,
              "sweep_form": _lib.TUNE_SWEEP_FORM, "halo_2d": _lib.TUNE_HALO_2D}
_TUNE_DEFAULT = {"s3_stagger": -1, "sweep_mf16": -1, "sweep_il": -1,
                 "conv_il": -1, "halo_mf": -1, "sweep_form": -1, "halo_2d": -1}  # the library's own pick (0 elsewhere)


class tuning:
    """Force kernel tile configs on a device's handle for the duration of a
    ``with`` block (rr_set_tuning; tests and tuning tools only):
    ``with ops.tuning(0, s3_cfg=6): ...``.  Values revert to the library's
    own pick on exit."""

    def __init__(self, device_index, **kw):
        for k in kw:
            if k not in _TUNE_KEYS:
                raise ValueError(f"unknown tuning key {k!r}")
        self.h = _lib.handle(device_index)
        self.kw = kw

    def __enter__(self):
        for k, v in self.kw.items():
            _lib.check(_lib.lib().rr_set_tuning(self.h, _TUNE_KEYS[k], int(v)), self.h, "rr_set_tuning")
        return self

    def __exit__(self, *exc):
        for k in self.kw:
            _lib.lib().rr_set_tuning(self.h, _TUNE_KEYS[k], _TUNE_DEFAULT.get(k, 0))
        return False


class KernelTimer:
    """HIP-event timing of librr kernel classes on their launch stream."""

    def __init__(self, device_index):
        self.h = _lib.handle(device_index)

    def enable(self, on=True):
        _lib.check(_lib.lib().rr_timing_enable(self.h, int(on)), self.h, "rr_timing_enable")

    def collect(self, cls):
        ms = ctypes.c_double()
        n = ctypes.c_longlong()
        _lib.check(_lib.lib().rr_timing_collect(self.h, cls, ctypes.byref(ms), ctypes.byref(n)), self.h,
                   "rr_timing_collect")
        return ms.value, n.value


def linear_ex(x, w, bias=None, residual=None, act=0):
    """y = act(x @ w.T + bias + residual); act 0 none, 1 ReLU, 2 QuickGELU."""
    _f32(x, "linear_ex x")
    _f32(w, "linear_ex w")
    dev = _dev(x)
    m, k = x.shape
    n = w.shape[0]
    y = torch.empty((m, n), dtype=torch.float32, device=x.device)
    if residual is not None:
        _f32(residual, "linear_ex residual")
        if tuple(residual.shape) != (m, n):
            raise ValueError("linear_ex: residual shape mismatch")
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_linear_ex(hd, _ptr(x), m, k, _ptr(w), _ptr(bias), n, _ptr(residual), int(act), _ptr(y),
                                       _stream(dev)), hd, "rr_linear_ex")
    return y


def layernorm(x, gamma, beta, eps=1e-5, rows=None, row_stride=None):
    """LayerNorm over the last dim of x [..., D]; with rows/row_stride, LN of
    ``rows`` rows spaced ``row_stride`` floats apart (e.g. the CLS tokens)."""
    _f32(x, "layernorm")
    dev = _dev(x)
    d = x.shape[-1]
    m = x.numel() // d if rows is None else int(rows)
    ld = d if row_stride is None else int(row_stride)
    y = torch.empty((m, d), dtype=torch.float32, device=x.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_layernorm(hd, _ptr(x), ld, m, d, _ptr(gamma), _ptr(beta), float(eps), _ptr(y),
                                       _stream(dev)), hd, "rr_layernorm")
    return y


def patchify(x_nhwc, patch, out_bf16=False):
    """NHWC image -> patch rows (fp32, or bf16 RNE for the bf16 patch GEMM)."""
    _f32(x_nhwc, "patchify")
    dev = _dev(x_nhwc)
    b, h, w, c = x_nhwc.shape
    y = torch.empty((b * (h // patch) * (w // patch), patch * patch * c),
                    dtype=torch.bfloat16 if out_bf16 else torch.float32, device=x_nhwc.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_patchify_ex(hd, _ptr(x_nhwc), b, h, w, c, patch, int(out_bf16), _ptr(y), _stream(dev)),
               hd, "rr_patchify_ex")
    return y


def vit_tokens(patches, b, cls, pos, ln=None, eps=1e-5):
    """[cls; patches] + pos per image; with ln = (gamma, beta), ln_pre fused."""
    _f32(patches, "vit_tokens")
    dev = _dev(patches)
    width = patches.shape[1]
    npatch = patches.shape[0] // b
    y = torch.empty((b * (npatch + 1), width), dtype=torch.float32, device=patches.device)
    hd = _lib.handle(dev)
    gamma, beta = ln if ln is not None else (None, None)
    _lib.check(_lib.lib().rr_vit_tokens_ex(hd, _ptr(patches), b, npatch, width, _ptr(cls), _ptr(pos), _ptr(gamma),
                                           _ptr(beta), float(eps), _ptr(y), _stream(dev)), hd, "rr_vit_tokens_ex")
    return y


def attention(qkv, b, seq, heads, head_dim=64):
    _f32(qkv, "attention")
    dev = _dev(qkv)
    out = torch.empty((b * seq, heads * head_dim), dtype=torch.float32, device=qkv.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_attention(hd, _ptr(qkv), b, seq, heads, head_dim, _ptr(out), _stream(dev)), hd,
               "rr_attention")
    return out


# ---- low precision (C4 bf16 / C5 fp8) --------------------------------------
DT_BF16, DT_FP8 = 1, 2
_LP = {"bf16": DT_BF16, "fp8": DT_FP8}


def quantize_rows(x, dtype):
    """fp32 [rows, d] -> (bf16 tensor, None) or (fp8-e4m3 bytes as uint8, per-row fp32 scales)."""
    _f32(x, "quantize_rows")
    dev = _dev(x)
    dt = _LP[dtype]
    rows, d = x.shape
    if dt == DT_BF16:
        y = torch.empty((rows, d), dtype=torch.bfloat16, device=x.device)
        sc = None
    else:
        y = torch.empty((rows, d), dtype=torch.uint8, device=x.device)
        sc = torch.empty(rows, dtype=torch.float32, device=x.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_quantize_rows(hd, _ptr(x), rows, d, dt, _ptr(y), _ptr(sc), _stream(dev)), hd,
               "rr_quantize_rows")
    return y, sc


def _lp_rows(t, sc, dtype, name):
    """Validate quantised rows as quantize_rows makes them: bf16 [rows, d]
    (no scales) or fp8-e4m3 bytes uint8 [rows, d] + fp32 scales [rows]."""
    if t.dim() != 2 or not t.is_contiguous():
        raise ValueError(f"{name}: expected contiguous [rows, d]")
    if dtype == "bf16":
        if t.dtype != torch.bfloat16:
            raise TypeError(f"{name}: bf16 rows must be torch.bfloat16, got {t.dtype}")
    else:
        if t.dtype not in (torch.uint8, torch.float8_e4m3fn):
            raise TypeError(f"{name}: fp8 rows must be uint8 (e4m3 bytes), got {t.dtype}")
        if sc is None or sc.dtype != torch.float32 or not sc.is_contiguous() or sc.numel() != t.shape[0]:
            raise ValueError(f"{name}: fp8 rows need contiguous fp32 scales, one per row")


def cosine_topk_lp(q, q_scale, g, g_scale, k, dtype, idx_offset=0, workspace=None, max_workspace_bytes=None):
    """Fused top-k on bf16 / fp8 rows (fp32 accumulate); scores dequantised.
    max_workspace_bytes: bounded candidate buffer, as in cosine_topk."""
    if dtype not in _LP:
        raise ValueError("cosine_topk_lp: dtype must be 'bf16' or 'fp8'")
    _lp_rows(q, q_scale, dtype, "cosine_topk_lp queries")
    _lp_rows(g, g_scale, dtype, "cosine_topk_lp gallery")
    if q.shape[1] != g.shape[1]:
        raise ValueError("cosine_topk_lp: descriptor dims differ")
    dev = _dev(q)
    dt = _LP[dtype]
    nq, d = q.shape
    n = g.shape[0]
    workspace, bounded = _ranker_workspace("exact", nq, n, d, k, workspace, max_workspace_bytes, q.device)
    os_ = torch.empty((nq, k), dtype=torch.float32, device=q.device)
    oi = torch.empty((nq, k), dtype=torch.int64, device=q.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_cosine_topk_lp(hd, _ptr(q), _ptr(q_scale), nq, _ptr(g), _ptr(g_scale), n, d, dt, k,
                                            int(idx_offset), _ptr(os_), _ptr(oi), _ptr(workspace), workspace.numel(),
                                            _stream(dev)), hd, "rr_cosine_topk_lp")
    if bounded and nq > 0:
        _recover_overflow("exact", nq, n, d, k, workspace,
                          lambda r, ws: cosine_topk_lp(q[r].contiguous(), None if q_scale is None else
                                                       q_scale[r].contiguous(), g, g_scale, k, dtype, idx_offset, ws),
                          os_, oi)
    return os_, oi


def linear_bf16(x, w, bias=None, residual=None, act=0, out_bf16=False):
    """bf16 x [M,K] . bf16 w [N,K]^T -> fp32 (or bf16) with fused epilogue."""
    if x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        raise TypeError("linear_bf16: x and w must be bfloat16")
    if x.dim() != 2 or w.dim() != 2 or not x.is_contiguous() or not w.is_contiguous() or x.shape[1] != w.shape[1]:
        raise ValueError("linear_bf16: contiguous x [M,K] and w [N,K] with matching K")
    dev = _dev(x)
    m, k = x.shape
    n = w.shape[0]
    if bias is not None and (_f32(bias, "linear_bf16 bias").numel() != n):
        raise ValueError("linear_bf16: bias must have N entries")
    if residual is not None and tuple(_f32(residual, "linear_bf16 residual").shape) != (m, n):
        raise ValueError("linear_bf16: residual shape mismatch")
    y = torch.empty((m, n), dtype=torch.bfloat16 if out_bf16 else torch.float32, device=x.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_linear_bf16(hd, _ptr(x), m, k, _ptr(w), _ptr(bias), n, _ptr(residual), int(act),
                                         int(out_bf16), _ptr(y), _stream(dev)), hd, "rr_linear_bf16")
    return y


def linear_bf16_ln_produce(x, w, bias, residual):
    """The residual GEMM of a ViT block with the next LayerNorm's inputs
    produced in its epilogue (rr_linear_bf16_ln, stats_out): returns (y fp32
    [M,N] = x.w^T + bias + residual, bf16(y - mean_t) with mean_t the mean of
    the row's 256-column tile, the per-row tile LayerNorm partials
    [M, N/256, 2] = (mean_t, M2_t))."""
    if x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        raise TypeError("linear_bf16_ln_produce: x and w must be bfloat16")
    if x.dim() != 2 or w.dim() != 2 or not x.is_contiguous() or not w.is_contiguous() or x.shape[1] != w.shape[1]:
        raise ValueError("linear_bf16_ln_produce: contiguous x [M,K] and w [N,K] with matching K")
    dev = _dev(x)
    m, k = x.shape
    n = w.shape[0]
    if n % 256:
        raise ValueError("linear_bf16_ln_produce: N % 256 == 0")
    if _f32(bias, "bias").numel() != n or tuple(_f32(residual, "residual").shape) != (m, n):
        raise ValueError("linear_bf16_ln_produce: bias [N] and residual [M,N]")
    y = torch.empty((m, n), dtype=torch.float32, device=x.device)
    yb = torch.empty((m, n), dtype=torch.bfloat16, device=x.device)
    st = torch.empty((m, n // 256, 2), dtype=torch.float32, device=x.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_linear_bf16_ln(hd, _ptr(x), m, k, _ptr(w), _ptr(bias), n, _ptr(residual), 0, 0, _ptr(y),
                                            None, None, 0.0, _ptr(st), _ptr(yb), _stream(dev)), hd, "rr_linear_bf16_ln")
    return y, yb, st


# widest K the fold's consumer serves: rr_linear_bf16_ln stages LN_TMAX = 3
# column-sum tiles of 256 (csrc/gemm_epilogue.hpp; rr.h: stats_in needs k <= 768)
LN_FOLD_MAX_K = 768


def ln_fold_supported(width, dtype):
    """Whether the ViT LayerNorm fold (rr_linear_bf16_ln) serves a width:
    bf16, 256-column tiles, and K = width within the consumer's limit."""
    return dtype == "bf16" and width % 256 == 0 and width <= LN_FOLD_MAX_K


def linear_bf16_ln_fold(xb, stats, w_folded, colsum, bias_folded, act=0, eps=1e-5):
    """act(LayerNorm(x) . W^T + b) -> bf16 with the LayerNorm folded into the
    GEMM (rr_linear_bf16_ln, stats_in): xb = the tile-centred bf16 rows of x
    and their partials (linear_bf16_ln_produce / ln_partials_bf16), w_folded =
    bf16(W o gamma), colsum = its fp32 row sums per 256-deep k tile
    [ceil(K/256), N], bias_folded = b + W beta (ln_fold_weights); K <= 768."""
    if xb.dtype != torch.bfloat16 or w_folded.dtype != torch.bfloat16:
        raise TypeError("linear_bf16_ln_fold: xb and w_folded must be bfloat16")
    dev = _dev(xb)
    m, k = xb.shape
    n = w_folded.shape[0]
    t = (k + 255) // 256
    if tuple(stats.shape) != (m, t, 2) or w_folded.shape[1] != k or tuple(colsum.shape) != (t, n):
        raise ValueError("linear_bf16_ln_fold: stats [M, ceil(K/256), 2], w_folded [N, K], colsum [ceil(K/256), N]")
    y = torch.empty((m, n), dtype=torch.bfloat16, device=xb.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_linear_bf16_ln(hd, _ptr(xb), m, k, _ptr(w_folded), _ptr(bias_folded), n, None, int(act),
                                            1, _ptr(y), _ptr(stats), _ptr(colsum), float(eps), None, None,
                                            _stream(dev)), hd, "rr_linear_bf16_ln")
    return y


def ln_partials_bf16(x):
    """(bf16(x - mean_t), the LayerNorm partials [M, D/256, 2]) of fp32 rows x
    [M, D], each 256-column tile t centred on its own mean mean_t
    (rr_ln_partials_bf16): the first block's ln_1 input, which no GEMM wrote."""
    _f32(x, "ln_partials_bf16")
    dev = _dev(x)
    d = x.shape[-1]
    m = x.numel() // d
    xb = torch.empty((m, d), dtype=torch.bfloat16, device=x.device)
    st = torch.empty((m, d // 256, 2), dtype=torch.float32, device=x.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_ln_partials_bf16(hd, _ptr(x), m, d, _ptr(xb), _ptr(st), _stream(dev)), hd,
               "rr_ln_partials_bf16")
    return xb, st


def ln_fold_weights(w, b, gamma, beta):
    """Fold a LayerNorm (gamma, beta) into the following linear (w [N,K] fp32,
    b [N]): (bf16(w o gamma), the fp32 row sums of that bf16 matrix per
    256-deep k tile [ceil(K/256), N], b + w beta)."""
    wf = (w.float() * gamma.float()[None, :]).to(torch.bfloat16).contiguous()
    n, k = wf.shape
    t = (k + 255) // 256
    colsum = torch.nn.functional.pad(wf.float(), (0, 256 * t - k)).view(n, t, 256).sum(dim=2).t().contiguous()
    bf = (b.double() + w.double() @ beta.double()).float().contiguous()
    return wf, colsum, bf


def layernorm_bf16(x, gamma, beta, eps=1e-5):
    _f32(x, "layernorm_bf16")
    dev = _dev(x)
    d = x.shape[-1]
    m = x.numel() // d
    y = torch.empty((m, d), dtype=torch.bfloat16, device=x.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_layernorm_ex(hd, _ptr(x), d, m, d, _ptr(gamma), _ptr(beta), float(eps), 1, _ptr(y),
                                          _stream(dev)), hd, "rr_layernorm_ex")
    return y


def attention_bf16(qkv, b, seq, heads, head_dim=64, bf16_math=True):
    """Attention core for the bf16 ViT: bf16 output; bf16 MFMA with fp32
    softmax (rr_attention_bf16; bf16 qkv rows: rr_attention_bf16_qkv16), or
    fp32 MFMA (bf16_math=False, fp32 qkv)."""
    dev = _dev(qkv)
    if qkv.dtype == torch.bfloat16 and bf16_math:
        if not qkv.is_contiguous():
            raise ValueError("attention_bf16: qkv must be contiguous")
        fn = _lib.lib().rr_attention_bf16_qkv16
    else:
        _f32(qkv, "attention_bf16")
        fn = _lib.lib().rr_attention_bf16 if bf16_math else _lib.lib().rr_attention_ex
    out = torch.empty((b * seq, heads * head_dim), dtype=torch.bfloat16, device=qkv.device)
    hd = _lib.handle(dev)
    _lib.check(fn(hd, _ptr(qkv), b, seq, heads, head_dim, 1, _ptr(out), _stream(dev)), hd, "rr_attention_bf16")
    return out


def alpha_qe(queries, gallery, top_idx, top_scores, n=2, alpha=3.0, idx_offset=0):
    """alpha-QE new queries (see include/rr.h rr_alpha_qe)."""
    _f32(queries, "alpha_qe queries")
    _f32(gallery, "alpha_qe gallery")
    dev = _dev(queries)
    nq, d = queries.shape
    k = top_idx.shape[1]
    out = torch.empty_like(queries)
    hd = _lib.handle(dev)
    if gallery.shape[1] != d or top_idx.dtype != torch.int64 or top_scores.dtype != torch.float32:
        raise TypeError("alpha_qe: gallery [N, d] fp32, top_idx int64, top_scores fp32")
    _lib.check(_lib.lib().rr_alpha_qe(hd, _ptr(queries), nq, _ptr(gallery), gallery.shape[0], d,
                                      _ptr(top_idx.contiguous()),
                                      _ptr(top_scores.contiguous()), k, int(n), float(alpha), int(idx_offset),
                                      _ptr(out), _stream(dev)), hd, "rr_alpha_qe")
    return out


def pcaw_gram(x):
    """Column mean and centred Gram sum_i (x_i - m)(x_i - m)^T of fp32 rows
    x [n, d] on the device (include/rr.h rr_pcaw_gram) -> (mean fp64 [d],
    gram fp64 [d, d])."""
    _f32(x, "pcaw_gram")
    dev = _dev(x)
    n, d = x.shape
    if n == 0:
        raise ValueError("pcaw_gram: empty descriptor set")
    L = _lib.lib()
    ws = torch.empty(L.rr_pcaw_gram_workspace_size(n, d), dtype=torch.uint8, device=dev)
    mean = torch.empty(d, dtype=torch.float64, device=dev)
    gram = torch.empty((d, d), dtype=torch.float64, device=dev)
    hd = _lib.handle(dev)
    _lib.check(L.rr_pcaw_gram(hd, _ptr(x), n, d, _ptr(ws), ws.numel(), _ptr(mean), _ptr(gram), _stream(dev)),
               hd, "rr_pcaw_gram")
    return mean, gram


def prefilter_gallery_bound(gallery, gallery_bf16):
    """Row-norm maxima (|g|, |g - bf16(g)|, |bf16(g)|) as fp64 [3] on the device."""
    _f32(gallery, "prefilter_gallery_bound")
    dev = _dev(gallery)
    n, d = gallery.shape
    out = torch.empty(3, dtype=torch.float64, device=gallery.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_prefilter_gallery_bound(hd, _ptr(gallery), _ptr(gallery_bf16), n, d, _ptr(out),
                                                     _stream(dev)), hd, "rr_prefilter_gallery_bound")
    return out


def cosine_topk_prefilter_workspace_size(nq, n, d, k):
    return int(_lib.lib().rr_cosine_topk_prefilter_workspace_size(nq, n, d, k))


def prefilter_survivors(workspace, nq, n, d, k):
    """Per-query count of rows that passed the bf16 filter in the last
    cosine_topk_prefilter call on this workspace (int32 [nq], device)."""
    off = int(_lib.lib().rr_cosine_topk_prefilter_counts_offset(int(nq), int(n), int(d), int(k)))
    return workspace[off:off + 4 * int(nq)].view(torch.int32)


def cosine_topk_prefilter(q, g, g_bf16, bound3, k, idx_offset=0, workspace=None, max_workspace_bytes=None):
    """Exact top-k (bit-identical to cosine_topk) via the bf16 prefilter.
    max_workspace_bytes: bounded candidate buffer + re-run of overflowed
    queries, as in cosine_topk."""
    _f32(q, "cosine_topk_prefilter q")
    _f32(g, "cosine_topk_prefilter g")
    dev = _dev(q)
    nq, d = q.shape
    n = g.shape[0]
    workspace, bounded = _ranker_workspace("prefilter", nq, n, d, k, workspace, max_workspace_bytes, q.device)
    s = torch.empty((nq, k), dtype=torch.float32, device=q.device)
    i = torch.empty((nq, k), dtype=torch.int64, device=q.device)
    hd = _lib.handle(dev)
    _lib.check(_lib.lib().rr_cosine_topk_prefilter(hd, _ptr(q), nq, _ptr(g), _ptr(g_bf16), _ptr(bound3), n, d, k,
                                                   int(idx_offset), _ptr(s), _ptr(i), _ptr(workspace),
                                                   workspace.numel(), _stream(dev)), hd, "rr_cosine_topk_prefilter")
    if bounded and nq > 0:
        _recover_overflow("prefilter", nq, n, d, k, workspace,
                          lambda r, ws: cosine_topk_prefilter(q[r].contiguous(), g, g_bf16, bound3, k, idx_offset, ws),
                          s, i)
    return s, i
