"""oracle/ — TEST INFRASTRUCTURE: the CPU restatement of the reference hot path.

Used ONLY by tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline``
leg, always as the checker / baseline and never as the thing measured or
shipped.  The product package (research_image_retrieval_amd) never imports it.

* ``cosine_topk.c`` (-> liboracle.so): the ranker of iris_evaluate.py:383-386
  (torch.mm + argsort), scores as the exact fmaf chain of librr's MFMA kernel,
  stable (score desc, index asc) ranking.  Pinned by tests/golden fixtures made
  from the reference's own op sequence.
* ``embed_ref.py``: torch-CPU restatement of the extractor (torchvision-layout
  ResNet, gem / GeMPooling, whiten / Linear projection, PCA-whitening apply,
  F.normalize).  GeM, projection, PCA-w and normalisation are pinned by golden
  fixtures generated from the reference's own functions; the ResNet trunk
  mirrors torchvision 0.22.1 resnet50/101 (not installed here) and is
  "parity unpinned" at that boundary.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
        i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
        c_int, c_ll = ctypes.c_int, ctypes.c_longlong
        L.rr_oracle_scores.argtypes = [f32p, c_int, f32p, c_ll, c_int, c_int, f32p]
        L.rr_oracle_topk_rows.argtypes = [f32p, c_int, c_ll, c_int, c_ll, f32p, i64p]
        L.rr_oracle_cosine_topk.argtypes = [f32p, c_int, f32p, c_ll, c_int, c_int, c_ll, c_int, f32p, i64p]
        L.rr_oracle_topk_merge.argtypes = [f32p, i64p, c_int, c_int, c_int, c_int, f32p, i64p]
        for fn in (L.rr_oracle_scores, L.rr_oracle_topk_rows, L.rr_oracle_cosine_topk, L.rr_oracle_topk_merge):
            fn.restype = None
        _LIB = L
    return _LIB


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def cosine_scores(q, g, order=0):
    """[nq][n] fp32 scores in librr's MFMA fmaf order (order 0)."""
    q, g = _f32(q), _f32(g)
    nq, d = q.shape
    n = g.shape[0]
    out = np.empty((nq, n), np.float32)
    lib().rr_oracle_scores(q, nq, g, n, d, order, out)
    return out


def topk_rows(scores, k, idx_offset=0):
    """Stable top-k (score desc, index asc) of every row of scores [nq][n]."""
    s = _f32(scores)
    nq, n = s.shape
    os_ = np.empty((nq, k), np.float32)
    oi = np.empty((nq, k), np.int64)
    lib().rr_oracle_topk_rows(s, nq, n, k, idx_offset, os_, oi)
    return os_, oi


def cosine_topk(q, g, k, idx_offset=0, order=0):
    q, g = _f32(q), _f32(g)
    nq, d = q.shape
    n = g.shape[0]
    os_ = np.empty((nq, k), np.float32)
    oi = np.empty((nq, k), np.int64)
    lib().rr_oracle_cosine_topk(q, nq, g, n, d, k, idx_offset, order, os_, oi)
    return os_, oi


def topk_merge(ps, pi, kout):
    ps = _f32(ps)
    pi = np.ascontiguousarray(pi, dtype=np.int64)
    nparts, nq, kin = ps.shape
    os_ = np.empty((nq, kout), np.float32)
    oi = np.empty((nq, kout), np.int64)
    lib().rr_oracle_topk_merge(ps, pi, nparts, nq, kin, kout, os_, oi)
    return os_, oi


def argsort_stable_desc(scores):
    """Full stable ranking of each row (the reference's np.argsort(-S, axis=1),
    iris_evaluate.py:386, with a stable tie-break)."""
    return np.argsort(-np.asarray(scores), axis=1, kind="stable")


def alpha_qe(q, g, top_idx, top_scores, n=2, alpha=3.0, idx_offset=0):
    """alpha-QE restatement (float64 accumulate, then fp32): q + sum max(s,0)^a g_r, L2-normalised."""
    q = np.asarray(q, np.float64)
    out = q.copy()
    for i in range(q.shape[0]):
        for r in range(n):
            j = int(top_idx[i, r]) - idx_offset
            if j < 0:
                continue
            w = max(float(top_scores[i, r]), 0.0) ** alpha
            out[i] += w * np.asarray(g[j], np.float64)
    out /= np.maximum(np.linalg.norm(out, axis=1, keepdims=True), 1e-12)
    return out.astype(np.float32)
