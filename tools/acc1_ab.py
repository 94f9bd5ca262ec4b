"""f16x2 conv with the plane-1 products in their own accumulator (config 4)
vs in the a0b0 accumulator (config 10, ACC1): error vs float64 next to the
exact-fp32 core on small batches, then interleaved timing at B images.
usage: acc1_ab.py [B]"""
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1280
dev = torch.device("cuda:0")
SHAPES = [(14, 256, 256, 3, 1, 0), (14, 1024, 256, 1, 1, 0), (14, 256, 1024, 1, 1, 1), (7, 512, 512, 3, 1, 0),
          (28, 128, 512, 1, 1, 1), (7, 2048, 512, 1, 1, 0), (56, 64, 256, 1, 1, 1)]


def run(x, rec, wc, bias, s, p, r, cfg):
    with ops.tuning(0, s3_cfg=cfg):
        return ops.conv2d_h2(x, rec, wc, bias, s, p, r, True)


def err(y, ref, scale):
    live = ref > 0
    e = ((y.double() - ref).abs() / scale)[live]
    return float(e.max()), float(e.mean())


for h, cin, cout, k, s, res in SHAPES:
    p = k // 2
    g = torch.Generator(device=dev).manual_seed(h * cin + cout)
    b = 8
    x = torch.relu(torch.randn(b, h, h, cin, device=dev, generator=g))
    w = torch.randn(cout, k, k, cin, device=dev, generator=g) * (2.0 / (k * k * cin)) ** 0.5
    bias = torch.randn(cout, device=dev, generator=g) * 0.1
    oh = (h + 2 * p - k) // s + 1
    r = torch.randn(b, oh, oh, cout, device=dev, generator=g) if res else None
    xn, wn = x.permute(0, 3, 1, 2).double(), w.permute(0, 3, 1, 2).double()
    ref = F.conv2d(xn, wn, None, s, p).permute(0, 2, 3, 1) + bias.double()
    scale = F.conv2d(xn.abs(), wn.abs(), None, s, p).permute(0, 2, 3, 1) + 1e-30
    if res:
        ref = ref + r.double()
        scale = scale + r.double().abs()
    ref = torch.relu(ref)
    wc = ops.H2Conv(w)
    rec = ops.amax_records(1, dev)
    ops.amax_f32(x, rec[0])
    e4 = err(run(x, rec[0], wc, bias, s, p, r, 4), ref, scale)
    e10 = err(run(x, rec[0], wc, bias, s, p, r, 10), ref, scale)
    ef = err(ops.conv2d(x, w, bias, s, p, r, True), ref, scale)
    # timing at B images
    xb = torch.relu(torch.randn(B, h, h, cin, device=dev, generator=g))
    rb = torch.randn(B, oh, oh, cout, device=dev, generator=g) if res else None
    recb = ops.amax_records(1, dev)
    ops.amax_f32(xb, recb[0])
    t = {4: [], 10: []}
    for _ in range(3):
        for c in (4, 10):
            run(xb, recb[0], wc, bias, s, p, rb, c)
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(4):
                run(xb, recb[0], wc, bias, s, p, rb, c)
            en.record()
            torch.cuda.synchronize()
            t[c].append(st.elapsed_time(en) / 4)
    fl = 2.0 * B * oh * oh * cout * k * k * cin
    m4, m10 = statistics.median(t[4]), statistics.median(t[10])
    print(f"h{h} {cin}->{cout} k{k} r{res}: err max/mean cfg4 {e4[0]:.3g}/{e4[1]:.3g} acc1 {e10[0]:.3g}/{e10[1]:.3g} "
          f"f32 {ef[0]:.3g}/{ef[1]:.3g} | ms cfg4 {m4:.3f} acc1 {m10:.3f} ({fl / m10 / 1e9:.0f} TF/s)", flush=True)
