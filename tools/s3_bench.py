"""Per-layer timing of the R101 trunk convs at B images: exact-fp32 core vs
the split-bf16 core.  usage: [S3_CFG=1..6] [S3_ONLY=1] s3_bench.py [B] [reps]
(S3_CFG forces one s3 tile config through rr_set_tuning, S3_STAGGER the
first-round stagger in ~1 us sleeps; default: the library's picks)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 320
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 10
# (h, cin, cout, k, stride, residual, count in R101)
SHAPES = [(56, 64, 64, 1, 1, 0, 1), (56, 64, 64, 3, 1, 0, 3), (56, 64, 256, 1, 1, 1, 3), (56, 256, 64, 1, 1, 0, 2),
          (56, 64, 256, 1, 1, 0, 1),
          (56, 256, 128, 1, 1, 0, 1), (56, 128, 128, 3, 2, 0, 1), (28, 128, 512, 1, 1, 1, 4), (28, 512, 128, 1, 1, 0, 3),
          (28, 128, 128, 3, 1, 0, 3), (56, 256, 512, 1, 2, 0, 1),
          (28, 512, 256, 1, 1, 0, 1), (28, 256, 256, 3, 2, 0, 1), (14, 256, 1024, 1, 1, 1, 23),
          (14, 1024, 256, 1, 1, 0, 22), (14, 256, 256, 3, 1, 0, 22), (28, 512, 1024, 1, 2, 0, 1),
          (14, 1024, 512, 1, 1, 0, 1), (14, 512, 512, 3, 2, 0, 1), (7, 512, 2048, 1, 1, 1, 3),
          (7, 2048, 512, 1, 1, 0, 2), (7, 512, 512, 3, 1, 0, 2), (14, 1024, 2048, 1, 2, 0, 1)]
dev = torch.device("cuda:0")
CFG = int(os.environ.get("S3_CFG", "0"))
STAGGER = int(os.environ.get("S3_STAGGER", "-1"))  # rr_set_tuning(RR_TUNE_S3_STAGGER); -1 = the library's pick
ops.tuning(0, s3_cfg=CFG, s3_stagger=STAGGER).__enter__()
tot = {"f32": 0.0, "s3": 0.0}
flops_tot = 0.0
for h, cin, cout, k, s, res, cnt in SHAPES:
    p = k // 2
    x = torch.relu(torch.randn(B, h, h, cin, device=dev))
    w = torch.randn(cout, k, k, cin, device=dev) * (2.0 / (k * k * cin)) ** 0.5
    bias = torch.randn(cout, device=dev) * 0.1
    oh = (h + 2 * p - k) // s + 1
    r = torch.randn(B, oh, oh, cout, device=dev) if res else None
    w3 = ops.split3_bf16(w)
    fl = 2.0 * B * oh * oh * cout * k * k * cin
    out = {}
    for math in (("s3",) if os.environ.get("S3_ONLY") else ("f32", "s3")):
        fn = (lambda: ops.conv2d(x, w, bias, s, p, r, True)) if math == "f32" else \
             (lambda: ops.conv2d_s3(x, w3, bias, s, p, r, True))
        for _ in range(3):
            fn()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        st.record()
        for _ in range(REPS):
            y = fn()
        en.record()
        torch.cuda.synchronize()
        ms = st.elapsed_time(en) / REPS
        out[math] = (ms, y)
        tot[math] += ms * cnt
    flops_tot += fl * cnt
    if "f32" not in out:
        print(f"h{h:3d} {cin:5d}->{cout:5d} k{k} s{s} r{res} x{cnt:2d}: s3 {out['s3'][0]:7.3f} ms "
              f"({fl / out['s3'][0] / 1e9:6.1f} TF/s)", flush=True)
        continue
    d = (out["s3"][1] - out["f32"][1]).abs().max().item()
    print(f"h{h:3d} {cin:5d}->{cout:5d} k{k} s{s} r{res} x{cnt:2d}: f32 {out['f32'][0]:7.3f} ms "
          f"({fl / out['f32'][0] / 1e9:6.1f} TF/s)  s3 {out['s3'][0]:7.3f} ms ({fl / out['s3'][0] / 1e9:6.1f} TF/s) "
          f"speedup {out['f32'][0] / out['s3'][0]:.2f}  max|diff| {d:.2e}", flush=True)
print(f"TOTAL trunk convs (weighted): f32 {tot['f32']:.2f} ms ({flops_tot / max(tot['f32'], 1e-9) / 1e9:.1f} TF/s)  "
      f"s3 {tot['s3']:.2f} ms ({flops_tot / tot['s3'] / 1e9:.1f} TF/s) cfg={CFG or 'auto'}")
