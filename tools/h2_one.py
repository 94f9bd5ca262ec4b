"""One f16x2 layer of the C3 trunk in a loop (rocprofv3 --pmc passes, one
launch shape per process).
usage: h2_one.py conv B H W Cin Cout k stride pad res [reps]
       h2_one.py stem B [reps]          (the halo stem + max-pool)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
if os.environ.get("H2_TUNE"):  # e.g. H2_TUNE=halo_mf=2 (rr_set_tuning keys, A/Bs)
    ops.tuning(0, **{k: int(v) for k, v in (kv.split("=") for kv in os.environ["H2_TUNE"].split(","))}).__enter__()
g = torch.Generator(device=dev).manual_seed(0)
mode = sys.argv[1]
if mode == "stem":
    b = int(sys.argv[2])
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    x = torch.zeros(b, 224, 224, 4, device=dev)
    x[..., :3] = torch.randn(b, 224, 224, 3, device=dev, generator=g)
    wc = ops.H2Conv(torch.nn.functional.pad(torch.randn(64, 7, 7, 3, device=dev, generator=g) * 0.05, (0, 1)))
    bias = torch.randn(64, device=dev, generator=g) * 0.1
    rin = ops.amax_records(1, dev)[0]
    ops.amax_f32(x, rin)

    def run():
        rout = ops.amax_records(1, dev)[0]
        return ops.stem_pool_h2(x, rin, wc, bias, 2, 3, rout)
    flop = 2.0 * b * 112 * 112 * 64 * 147
else:
    b, h, w, cin, cout, k, s, p, res = (int(v) for v in sys.argv[2:11])
    reps = int(sys.argv[11]) if len(sys.argv) > 11 else 10
    x = torch.relu(torch.randn(b, h, w, cin, device=dev, generator=g))
    wc = ops.H2Conv(torch.randn(cout, k, k, cin, device=dev, generator=g) * (1.0 / (k * k * cin) ** 0.5))
    bias = torch.randn(cout, device=dev, generator=g) * 0.1
    oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    r = torch.randn(b, oh, ow, cout, device=dev, generator=g) if res else None
    rin = ops.amax_records(1, dev)[0]
    ops.amax_f32(x, rin)

    def run():
        rout = ops.amax_records(1, dev)[0]
        return ops.conv2d_h2(x, rin, wc, bias, s, p, r, True, rout)
    flop = 2.0 * b * oh * ow * cout * k * k * cin
for _ in range(2):
    run()
torch.cuda.synchronize()
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
st.record()
for _ in range(reps):
    run()
en.record()
torch.cuda.synchronize()
ms = st.elapsed_time(en) / reps
print({"ms": round(ms, 4), "fp32_equiv_tflops": round(flop / ms / 1e9, 1)}, flush=True)
