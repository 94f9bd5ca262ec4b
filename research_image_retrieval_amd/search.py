"""search — the reference ranker (iris_evaluate.py:378-386) on librr.

Reference lines:
    query_features = F.normalize(query_features, p=2, dim=1)      # :379
    gallery_features = F.normalize(gallery_features, p=2, dim=1)  # :380
    similarity = torch.mm(query_features, gallery_features.t())   # :383
    ranks = np.argsort(-similarity, axis=1)                        # :386
Here: descriptors are L2-normalised on the GPU, the cosine GEMM + top-k run
fused in rr_cosine_topk (fp32 MFMA, stable order score desc / index asc), and
ranks come back in the layout ``compute_map`` consumes:
    k=None -> int64 ndarray [N, Q]   (compute_map(..., li=False), utils/evaluate.py:79-80)
    k=int  -> list of Q int64 arrays (compute_map(..., li=True),  utils/evaluate.py:75-77)
(the reference's own driver passes a [Q,N] array with li=False, a layout bug —
SURVEY.md Appendix A.2 — which this API does not reproduce).
"""
import numpy as np
import torch

from . import ops

MAX_FULL_RANK = 16384  # full ranking sorts one query's scores in LDS


def _dev_f32(x, device):
    if isinstance(x, np.ndarray):
        x = torch.from_numpy(x)
    return x.to(device=device, dtype=torch.float32).contiguous()


class GallerySearcher:
    """A gallery resident in HBM plus a reusable top-k workspace.

    ``normalize=True`` applies F.normalize to the gallery once at load (as
    iris_evaluate.py:380); pass False for descriptors that are already unit
    norm (extractor outputs are)."""

    def __init__(self, gallery, device="cuda", normalize=True, idx_offset=0, dtype="fp32", prefilter=False):
        """dtype "fp32" (exact, default), or "bf16" / "fp8" (configs C4 / C5:
        the gallery is quantised once; parity vs fp32 is recall@k).
        prefilter=True (fp32, D % 8 == 0): same exact result, bit for bit,
        through the bf16-bound prefilter (rr_cosine_topk_prefilter); keeps a
        bf16 copy of the gallery beside the fp32 one."""
        if dtype not in ("fp32", "bf16", "fp8"):
            raise ValueError("dtype must be fp32, bf16 or fp8")
        self.device = torch.device(device)
        g = _dev_f32(gallery, self.device)
        self.gallery = ops.l2_normalize(g, 1e-12) if normalize else g
        self.idx_offset = int(idx_offset)
        self.dtype = dtype
        self.prefilter = bool(prefilter) and dtype == "fp32" and self.gallery.shape[1] % 8 == 0
        self.gallery_lp, self.gallery_scale, self.bound = (None, None, None)
        if dtype != "fp32" or self.prefilter:
            self.gallery_lp, self.gallery_scale = ops.quantize_rows(self.gallery, "bf16" if self.prefilter else dtype)
        if self.prefilter:
            self.bound = ops.prefilter_gallery_bound(self.gallery, self.gallery_lp)
        self._ws = None

    @property
    def n(self):
        return self.gallery.shape[0]

    def topk(self, queries, k, normalize=True):
        """-> (scores [Q,k] fp32, idx [Q,k] int64) on the device."""
        q = _dev_f32(queries, self.device)
        if normalize:
            q = ops.l2_normalize(q, 1e-12)
        size = ops.cosine_topk_prefilter_workspace_size if self.prefilter else ops.cosine_topk_workspace_size
        need = size(q.shape[0], self.n, q.shape[1], k)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        if self.prefilter:
            return ops.cosine_topk_prefilter(q.contiguous(), self.gallery, self.gallery_lp, self.bound, k,
                                             idx_offset=self.idx_offset, workspace=self._ws)
        if self.dtype != "fp32":
            q_lp, q_sc = ops.quantize_rows(q.contiguous(), self.dtype)
            return ops.cosine_topk_lp(q_lp, q_sc, self.gallery_lp, self.gallery_scale, k, self.dtype,
                                      idx_offset=self.idx_offset, workspace=self._ws)
        return ops.cosine_topk(q, self.gallery, k, idx_offset=self.idx_offset, workspace=self._ws)


def search(qvecs, vecs, k=None, return_scores=False, device="cuda", normalize=True):
    """Rank gallery ``vecs`` [N,D] for every query in ``qvecs`` [Q,D].

    k=None: full ranking, int64 [N, Q] (N <= 16384 per call).
    k=int : list of Q int64 arrays of the top-k gallery indices."""
    g = GallerySearcher(vecs, device=device, normalize=normalize)
    n = g.n
    kk = n if k is None else min(int(k), n)
    if k is None and n > MAX_FULL_RANK:
        raise ValueError(f"full ranking supports N <= {MAX_FULL_RANK}; pass k for larger galleries")
    if kk == 0:
        ranks = np.zeros((0, len(qvecs)), np.int64)
        return (ranks, None) if return_scores else ranks
    s, i = g.topk(qvecs, kk, normalize=normalize)
    s, i = s.cpu().numpy(), i.cpu().numpy()
    ranks = i.T.copy() if k is None else [row for row in i]
    return (ranks, s) if return_scores else ranks


def alpha_qe_search(searcher, queries, k=100, n=2, alpha=3.0, normalize=True):
    """Search, alpha-QE the queries with their top-n, search again (config C5).
    Returns (scores, idx) of the second search and the expanded queries."""
    q = _dev_f32(queries, searcher.device)
    if normalize:
        q = ops.l2_normalize(q, 1e-12)
    s, i = searcher.topk(q, max(k, n), normalize=False)
    q2 = ops.alpha_qe(q, searcher.gallery, i, s, n=n, alpha=alpha, idx_offset=searcher.idx_offset)
    s2, i2 = searcher.topk(q2, k, normalize=False)
    return s2, i2, q2
