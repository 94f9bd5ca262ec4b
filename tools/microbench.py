"""Quick kernel microbenchmarks (development aid, not the contract bench)."""
import argparse
import json
import time

import torch

from research_image_retrieval_amd import ops, _lib


def t_ms(fn, iters=5, warm=2):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_600_000)
    ap.add_argument("--d", type=int, default=2048)
    ap.add_argument("--q", type=int, default=256)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--conv", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    gal = torch.randn(a.n, a.d, device=dev, generator=g)
    gal = torch.nn.functional.normalize(gal, dim=1)
    q = torch.nn.functional.normalize(torch.randn(a.q, a.d, device=dev, generator=g), dim=1)
    ws = torch.empty(ops.cosine_topk_workspace_size(a.q, a.n, a.d, a.k), dtype=torch.uint8, device=dev)
    timer = ops.KernelTimer(0)
    timer.enable(True)
    ms = t_ms(lambda: ops.cosine_topk(q, gal, a.k, workspace=ws), iters=5)
    cos_ms, cos_n = timer.collect(_lib.TIME_COSINE)
    sel_ms, sel_n = timer.collect(_lib.TIME_SELECT)
    flop = 2.0 * a.q * a.n * a.d
    out = {"rank_ms": ms, "rank_tflops": flop / ms / 1e9, "gemm_ms_per_call": cos_ms / 7, "select_ms_per_call": sel_ms / 7,
           "gemm_tflops": flop / (cos_ms / 7) / 1e9}
    # dense-only GEMM rate
    sc_ms = t_ms(lambda: ops.cosine_scores(q, gal[:200000]), iters=5)
    out["dense_scores_tflops_200k"] = 2.0 * a.q * 200000 * a.d / sc_ms / 1e9
    print(json.dumps(out))
    if a.conv:
        shapes = [(256, 56, 56, 64, 64, 3, 1, 1), (256, 56, 56, 256, 64, 1, 1, 0), (256, 56, 56, 64, 256, 1, 1, 0),
                  (256, 28, 28, 128, 128, 3, 1, 1), (256, 14, 14, 256, 256, 3, 1, 1), (256, 7, 7, 512, 512, 3, 1, 1),
                  (256, 7, 7, 512, 2048, 1, 1, 0), (256, 224, 224, 3, 64, 7, 2, 3)]
        for (b, h, w, cin, cout, k, s, p) in shapes:
            x = torch.randn(b, h, w, cin, device=dev)
            wt = torch.randn(cout, k, k, cin, device=dev) * 0.01
            bias = torch.randn(cout, device=dev)
            oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
            ms = t_ms(lambda: ops.conv2d(x, wt, bias, s, p, None, True))
            fl = 2.0 * b * oh * ow * cout * k * k * cin
            print(json.dumps({"conv": [b, h, w, cin, cout, k, s, p], "ms": ms, "tflops": fl / ms / 1e9}))
            del x, wt


if __name__ == "__main__":
    main()
