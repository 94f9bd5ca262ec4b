"""Interleaved A/B of the low-precision filter sweep configs (rr_set_tuning
lp_cfg: 0 = the pick, 5 = the 8-phase 256x256 pipeline of gemm_8p.hip) on the
C5 shape (Q fp8 queries x 1.6 M fp8 rows x 2048, top-100) or the C4 bf16
shape (LP_DT=bf16, d = 512): the sweep launch's HIP-event time, its fraction
of the dtype's dense peak, and the ranker's top-k compared between configs
(the accumulation order differs, so scores within 1e-5 and index sets).
usage: [LP_KEY=lp_cfg|sweep_form|...] LP_CFGS="0 5" LP_Q=1280 LP_DT=fp8 python tools/fp8_ab.py"""
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
Q = int(os.environ.get("LP_Q", "1280"))
DT = os.environ.get("LP_DT", "fp8")
cfgs = [int(c) for c in os.environ.get("LP_CFGS", "0 5").split()]
KEY = os.environ.get("LP_KEY", "lp_cfg")
N = int(os.environ.get("LP_N", "1600000"))
D = int(os.environ.get("LP_D", "2048" if DT == "fp8" else "512"))
K = 100
PEAK = {"fp8": 5000.0, "bf16": 2500.0}[DT]
g = torch.Generator(device=dev).manual_seed(0)
gal = F.normalize(torch.randn(N, D, device=dev, generator=g), dim=1)
q = F.normalize(torch.randn(Q, D, device=dev, generator=g), dim=1)
q = F.normalize(q[:1] + 0.3 * q, dim=1)  # correlated queries: a realistic survivor count
gq, gs = ops.quantize_rows(gal, DT)
qq, qs = ops.quantize_rows(q, DT)
del gal
timer = ops.KernelTimer(0)


def run(cfg, iters=3):
    with ops.tuning(0, **{KEY: cfg}):
        ops.cosine_topk_lp(qq, qs, gq, gs, K, DT)
        torch.cuda.synchronize()
        timer.enable(True)
        for _ in range(iters):
            s, i = ops.cosine_topk_lp(qq, qs, gq, gs, K, DT)
        torch.cuda.synchronize()
        ms = timer.collect(_lib.TIME_COSINE)[0] / iters
        timer.enable(False)
    return ms, s.clone(), i.clone()


res = {c: [] for c in cfgs}
outs = {}
for _ in range(3):
    for c in cfgs:
        ms, s, i = run(c)
        res[c].append(ms)
        outs[c] = (s, i)
fl = 2.0 * Q * N * D
base = cfgs[0]
for c in cfgs:
    ms = statistics.median(res[c])
    ds = (outs[c][0] - outs[base][0]).abs().max().item()
    same_sets = sum(len(set(a.tolist()) & set(b.tolist())) for a, b in zip(outs[c][1].cpu(), outs[base][1].cpu())) / (Q * K)
    print(json.dumps({KEY: c, "dtype": DT, "Q": Q, "N": N, "D": D, "sweep_ms": round(ms, 3),
                      "tflops": round(fl / ms / 1e9, 1), "frac_peak": round(fl / ms / 1e9 / PEAK, 4),
                      "max_score_diff_vs_cfg_%d" % base: ds, "topk_overlap_vs_cfg_%d" % base: round(same_sets, 5)}),
          flush=True)
