"""Prefilter diagnostics at the bench scale: pass-1 candidates per query,
rescored survivors per query and eps, read back from the workspace
(layout of csrc/prefilter.hip prefilter_layout)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402

n, d, nq, k = 1_600_000, 2048, 320, 100
dev = torch.device("cuda:0")
g = torch.empty((n, d), device=dev)
gen = torch.Generator(device=dev).manual_seed(0)
for b in range(0, n, 65536):
    g[b:b + 65536] = torch.randn((min(65536, n - b), d), generator=gen, device=dev)
g = ops.l2_normalize(g, 1e-12, out=g)
q = ops.l2_normalize(torch.randn((nq, d), generator=gen, device=dev), 1e-12)
gb, _ = ops.quantize_rows(g, "bf16")
bound = ops.prefilter_gallery_bound(g, gb)
print("bound (G, E, H):", bound.cpu().numpy())
ws = torch.empty(ops.cosine_topk_prefilter_workspace_size(nq, n, d, k), dtype=torch.uint8, device=dev)
s, i = ops.cosine_topk_prefilter(q, g, gb, bound, k, workspace=ws)
torch.cuda.synchronize()
al = lambda x: (x + 255) & ~255  # noqa: E731
smax = max(32768, k)
s_rows = min(n, smax)
ld = (s_rows + 3) & ~3
o = al(nq * ld * 4)
off_tau = o
o = al(o + nq * 4)
off_cnt = o
o = al(o + nq * 4)
o = al(o + 4)
off_eps = o
o = al(o + nq * 4)
o = al(o + nq * d * 2)
off_cand = o
cap = max(n, k)
cnt = ws[off_cnt:off_cnt + nq * 4].view(torch.int32).cpu().numpy()
eps2 = ws[off_eps:off_eps + nq * 4].view(torch.float32).cpu().numpy()
surv = []
for qi in range(0, nq, 32):
    keys = ws[off_cand + qi * cap * 8: off_cand + qi * cap * 8 + int(cnt[qi]) * 8].view(torch.int64)
    surv.append(int((keys != 0).sum().item()))
print("pass-1 candidates per query: mean %.0f min %d max %d" % (cnt.mean(), cnt.min(), cnt.max()))
print("rescored survivors (sampled queries):", surv)
print("eps2 mean %.5f min %.5f max %.5f" % (eps2.mean(), eps2.min(), eps2.max()))
# timing of the whole call
t0 = torch.cuda.Event(enable_timing=True)
t1 = torch.cuda.Event(enable_timing=True)
t0.record()
for _ in range(5):
    ops.cosine_topk_prefilter(q, g, gb, bound, k, workspace=ws)
t1.record()
torch.cuda.synchronize()
print("prefilter call ms: %.3f" % (t0.elapsed_time(t1) / 5))
