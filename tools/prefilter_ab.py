"""Interleaved A/B of the exact prefilter ranker's bf16 filter sweep configs
(rr_set_tuning lp_cfg: 0 = the pick, 4 / 5 forced; or another key with PF_KEY, e.g.
sweep_il / sweep_mf16) on the C3 shape
(Q queries x 1.6 M x 2048, top-100): the sweep launch's HIP-event time, its
fraction of the bf16 dense peak, and the whole ranker's results compared bit
for bit between configs.
usage: [PF_KEY=lp_cfg|sweep_il|...] [PF_EXTRA="key=value ..."] PF_CFGS="0 5" PF_Q=1280
       python tools/prefilter_ab.py"""
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
Q = int(os.environ.get("PF_Q", "1280"))
cfgs = [int(c) for c in os.environ.get("PF_CFGS", "0 5").split()]
KEY = os.environ.get("PF_KEY", "lp_cfg")
# fixed extra tuning for every config, e.g. PF_EXTRA="sweep_mf16=1"
EXTRA = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in os.environ.get("PF_EXTRA", "").split()}
N, D, K = int(os.environ.get("PF_N", "1600000")), 2048, 100
g = torch.Generator(device=dev).manual_seed(0)
gal = F.normalize(torch.randn(N, D, device=dev, generator=g), dim=1)
q = F.normalize(torch.randn(Q, D, device=dev, generator=g), dim=1)
if os.environ.get("PF_QKIND") == "corr":  # near-parallel queries (cosine ~0.999 to each other)
    q = F.normalize(q[:1] + 0.05 * q, dim=1)
elif os.environ.get("PF_QKIND") == "same":  # the C3 bench's own descriptors: one vector to ~1e-6
    q = F.normalize(q[:1] + 1e-6 * q, dim=1)
gbf, _ = ops.quantize_rows(gal, "bf16")
bound = ops.prefilter_gallery_bound(gal, gbf)
ws = torch.empty(ops.cosine_topk_prefilter_workspace_size(Q, N, D, K), dtype=torch.uint8, device=dev)
timer = ops.KernelTimer(0)
CLS = (_lib.TIME_COSINE, _lib.TIME_COSINE_SEED, _lib.TIME_SELECT, _lib.TIME_ELEM, _lib.TIME_GEMM)


def run(cfg, iters=3):
    with ops.tuning(0, **{KEY: cfg}, **EXTRA):
        ops.cosine_topk_prefilter(q, gal, gbf, bound, K, workspace=ws)
        torch.cuda.synchronize()
        timer.enable(True)
        for _ in range(iters):
            s, i = ops.cosine_topk_prefilter(q, gal, gbf, bound, K, workspace=ws)
        torch.cuda.synchronize()
        out = {c: timer.collect(c) for c in CLS}
        timer.enable(False)
    return out[_lib.TIME_COSINE][0] / iters, s.clone(), i.clone()


res = {c: [] for c in cfgs}
outs = {}
for r in range(3):
    for c in cfgs:
        ms, s, i = run(c)
        res[c].append(ms)
        outs[c] = (s, i)
fl = 2.0 * Q * N * D
base = cfgs[0]
for c in cfgs:
    ms = statistics.median(res[c])
    same = torch.equal(outs[c][1], outs[base][1]) and torch.equal(outs[c][0].view(torch.int32),
                                                                  outs[base][0].view(torch.int32))
    print(json.dumps({KEY: c, "Q": Q, "N": N, "sweep_ms": round(ms, 3), "tflops": round(fl / ms / 1e9, 1),
                      "frac_bf16_peak": round(fl / ms / 1e9 / 2500.0, 4), "identical_to_cfg_%d" % base: same}),
          flush=True)
