"""Low-precision GEMM configs on the shapes that matter (the ViT-B/16 block's
linears with their epilogues at LP_B images (default 320), the bf16 prefilter
sweep, the fp8 C5 sweep; LP_SWEEPS=0 skips the sweeps).  Run once per forced
config: LP_CFG=1..5 python tools/lp_bench.py  -> JSON lines (rr_set_tuning
RR_TUNE_LP_CFG: 1 = 128x128, 2 = 256x64, 3 = 256x256, 4 = 256x320 sweep tile,
5 = 8-phase 256x256 sweep; unset = the
library's pick)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import _lib, ops  # noqa: E402


def t_ms(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    st = torch.cuda.Event(enable_timing=True)
    en = torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters


cfg = os.environ.get("LP_CFG", "auto")
dev = torch.device("cuda:0")
if cfg != "auto":
    ops.tuning(0, lp_cfg=int(cfg)).__enter__()
g = torch.Generator(device=dev).manual_seed(0)
M = int(os.environ.get("LP_B", "320")) * 197
SWEEPS = os.environ.get("LP_SWEEPS", "1") == "1"
# the ViT-B/16 block's four linears with their epilogues (networks.VisionTransformer bf16):
# QKV -> bf16, out-proj + residual, fc1 QuickGELU -> bf16, fc2 + residual
VIT = [(768, 2304, 0, True, False), (768, 768, 0, False, True), (768, 3072, 2, True, False),
       (3072, 768, 0, False, True)]
for (k, n, act, obf, resid) in VIT:
    res = torch.randn(M, n, device=dev, generator=g) if resid else None
    x = (torch.randn(M, k, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    w = (torch.randn(n, k, device=dev, generator=g) / k ** 0.5).to(torch.bfloat16)
    b = torch.randn(n, device=dev, generator=g)
    y = ops.linear_bf16(x, w, b, residual=res, act=act, out_bf16=obf)
    ref = torch.addmm(b, x[:4096].float(), w.float().t()) + (0 if res is None else res[:4096])
    if act == 2:
        ref = ref * torch.sigmoid(1.702 * ref)
    err = ((y[:4096].float() - ref).abs().max() / ref.abs().max()).item()
    ms = t_ms(lambda: ops.linear_bf16(x, w, b, residual=res, act=act, out_bf16=obf))
    tag = (" +res" if resid else "") + (" gelu" if act == 2 else "") + (" ->bf16" if obf else "")
    print(json.dumps({"cfg": cfg, "op": f"linear_bf16 {M}x{k}->{n}" + tag, "ms": round(ms, 4),
                      "tflops": round(2.0 * M * k * n / ms / 1e9, 1), "rel_err": err}), flush=True)
# cosine sweeps: bf16 d=2048 (prefilter), bf16 d=512 (C4), fp8 d=2048 (C5)
N = 1_600_000
for dt, d in ([("bf16", 2048), ("bf16", 512), ("fp8", 2048)] if SWEEPS else []):
    gal = torch.nn.functional.normalize(torch.randn(N, d, device=dev, generator=g), dim=1)
    q = torch.nn.functional.normalize(torch.randn(320, d, device=dev, generator=g), dim=1)
    gl, gs = ops.quantize_rows(gal, dt)
    ql, qs = ops.quantize_rows(q, dt)
    ws = torch.empty(ops.cosine_topk_workspace_size(320, N, d, 100), dtype=torch.uint8, device=dev)
    timer = ops.KernelTimer(0)
    timer.enable(True)
    ms = t_ms(lambda: ops.cosine_topk_lp(ql, qs, gl, gs, 100, dt, workspace=ws), iters=5, warm=2)
    f_ms, f_n = timer.collect(_lib.TIME_COSINE)
    timer.collect(_lib.TIME_COSINE_SEED), timer.collect(_lib.TIME_SELECT), timer.collect(_lib.TIME_ELEM)
    timer.enable(False)
    s, i = ops.cosine_topk_lp(ql, qs, gl, gs, 100, dt, workspace=ws)
    # reference on the dequantised rows for 8 queries
    if dt == "bf16":
        gd, qd = gl.float(), ql.float()
    else:
        gd = gl.view(torch.float8_e4m3fn).float() * gs[:, None]
        qd = ql.view(torch.float8_e4m3fn).float() * qs[:, None]
    ref = torch.topk(qd[:8] @ gd.t(), 100, dim=1).indices
    rec = sum(len(set(ref[r].tolist()) & set(i[r].tolist())) for r in range(8)) / 800.0
    fl = 2.0 * 320 * (N - 32768) * d
    print(json.dumps({"cfg": cfg, "op": f"cosine_topk_lp {dt} 320x{N}x{d}", "call_ms": round(ms, 4),
                      "filter_ms": round(f_ms / max(1, f_n), 4), "filter_tflops": round(fl / (f_ms / max(1, f_n)) / 1e9, 1),
                      "recall_vs_dequant_ref": rec}), flush=True)
    del gal, gl, gs, ws
