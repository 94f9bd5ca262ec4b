"""The ViT-B/16 block's four fold-path linears (networks.VisionTransformer
bf16 with ln_fold: in-proj LN-fold -> bf16, out-proj + residual + LayerNorm
partials, c_fc LN-fold + QuickGELU -> bf16, c_proj + residual + partials) at
B images, each under the given lp_cfg values, rounds interleaved: median ms.
usage: python tools/vit_lin_ab.py [B] [cfgs, default 0,6]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1280
CFGS = [int(c) for c in (sys.argv[2] if len(sys.argv) > 2 else "0,6").split(",")]
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
M, D = B * 197, 768
x = torch.randn(M, D, device=dev, generator=g)
r = torch.randn(M, D, device=dev, generator=g)
gam, bet = 1 + 0.1 * torch.randn(D, device=dev, generator=g), 0.1 * torch.randn(D, device=dev, generator=g)
xb, st = ops.ln_partials_bf16(x)
w_in, b_in = torch.randn(3 * D, D, device=dev, generator=g) * D ** -0.5, torch.zeros(3 * D, device=dev)
w_fc, b_fc = torch.randn(4 * D, D, device=dev, generator=g) * D ** -0.5, torch.zeros(4 * D, device=dev)
wf_in, cs_in, bf_in = ops.ln_fold_weights(w_in, b_in, gam, bet)
wf_fc, cs_fc, bf_fc = ops.ln_fold_weights(w_fc, b_fc, gam, bet)
w_out = (torch.randn(D, D, device=dev, generator=g) * D ** -0.5).bfloat16()
w_pr = (torch.randn(D, 4 * D, device=dev, generator=g) * (4 * D) ** -0.5).bfloat16()
h = torch.randn(M, 4 * D, device=dev, generator=g).bfloat16()
bias = torch.zeros(D, device=dev)
ops_ = {
    "in_proj (fold)": lambda: ops.linear_bf16_ln_fold(xb, st, wf_in, cs_in, bf_in),
    "out_proj (+res, partials)": lambda: ops.linear_bf16_ln_produce(xb, w_out, bias, r),
    "c_fc (fold, gelu)": lambda: ops.linear_bf16_ln_fold(xb, st, wf_fc, cs_fc, bf_fc, act=2),
    "c_proj (+res, partials)": lambda: ops.linear_bf16_ln_produce(h, w_pr, bias, r),
}


def t_ms(fn, reps=5):
    fn()
    st_, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st_.record()
    for _ in range(reps):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st_.elapsed_time(en) / reps


res = {(n, c): [] for n in ops_ for c in CFGS}
for _ in range(4):
    for n, fn in ops_.items():
        for c in CFGS:
            with ops.tuning(0, lp_cfg=c):
                res[(n, c)].append(t_ms(fn))
tot = {c: 0.0 for c in CFGS}
for n in ops_:
    line = " | ".join(f"lp_cfg {c}: {statistics.median(res[(n, c)]):.3f} ms" for c in CFGS)
    for c in CFGS:
        tot[c] += statistics.median(res[(n, c)])
    print(f"{n:28s} {line}", flush=True)
print("per block (x12 per step): " + " | ".join(f"lp_cfg {c}: {tot[c]:.3f} ms" for c in CFGS))
