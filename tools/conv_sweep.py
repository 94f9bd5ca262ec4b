"""Time every distinct ResNet conv launch of networks.ResNet.forward (B images
at 224^2) and report TF/s, effective GB/s and weighted share of the trunk."""
import argparse
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402
from research_image_retrieval_amd import weights as W  # noqa: E402


def conv_launches(arch, b, h=224, w=224):
    out = lambda x, k, s, p: (x + 2 * p - k) // s + 1  # noqa: E731
    L = collections.Counter()
    H, Wd = h, w
    L[(b, H, Wd, 4, 64, 7, 2, 3, False, True)] += 1  # stem on NHWC4
    H, Wd = out(out(H, 7, 2, 3), 3, 2, 1), out(out(Wd, 7, 2, 3), 3, 2, 1)
    inpl = 64
    for li, nb in enumerate(W.RESNET_LAYERS[arch]):
        pl = 64 * 2 ** li
        for bi in range(nb):
            s = 2 if (bi == 0 and li > 0) else 1
            Ho, Wo = out(H, 3, s, 1), out(Wd, 3, s, 1)
            if bi == 0:
                L[(b, H, Wd, inpl, pl * 4, 1, s, 0, False, False)] += 1
            L[(b, H, Wd, inpl, pl, 1, 1, 0, False, True)] += 1
            L[(b, H, Wd, pl, pl, 3, s, 1, False, True)] += 1
            L[(b, Ho, Wo, pl, pl * 4, 1, 1, 0, True, True)] += 1
            H, Wd, inpl = Ho, Wo, pl * 4
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--arch", default="resnet101")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    rows = []
    tot_ms = 0.0
    for (b, h, w, cin, cout, k, s, p, res, relu), mult in conv_launches(a.arch, a.batch).items():
        x = torch.randn(b, h, w, cin, device=dev)
        wt = torch.randn(cout, k, k, cin, device=dev) * (2.0 / (k * k * cin)) ** 0.5
        bias = torch.randn(cout, device=dev)
        oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
        r = torch.randn(b, oh, ow, cout, device=dev) if res else None
        f = lambda: ops.conv2d(x, wt, bias, s, p, r, relu)  # noqa: E731
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        fl = 2.0 * b * oh * ow * cout * k * k * cin
        by = 4.0 * (x.numel() + b * oh * ow * cout * (2 if res else 1) + wt.numel())
        rows.append({"shape": [b, h, w, cin, cout, k, s, p], "res": res, "mult": mult, "ms": round(ms, 4),
                     "tflops": round(fl / ms / 1e9, 1), "gbs": round(by / ms / 1e6, 0),
                     "weighted_ms": round(ms * mult, 3)})
        tot_ms += ms * mult
        del x, wt, r
    for r in sorted(rows, key=lambda r: -r["weighted_ms"]):
        r["share"] = round(r["weighted_ms"] / tot_ms, 3)
        print(json.dumps(r))
    print(json.dumps({"trunk_conv_ms": round(tot_ms, 3)}))


if __name__ == "__main__":
    main()
