"""Dump the C3 bench's own query descriptors (bench.py's rank-0 images through
its R101-GeM + PCA-w extractor) to gpurun_out/bench_q.npy with summary
statistics, plus the prefilter's per-query survivor counts for each
sweep_form, so sweep A/Bs can be reproduced off the bench.
usage: python tools/bench_queries.py [B]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from research_image_retrieval_amd import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1280
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
net = bench.build_extractor("resnet101", dev)
rs = np.random.RandomState(1234)  # bench.py's rank-0 images
imgs = torch.from_numpy(rs.randint(0, 256, size=(B, 224, 224, 3), dtype=np.uint8)).to(dev)
d = net.forward_test_u8(imgs)
q = d.cpu().numpy()
os.makedirs("gpurun_out", exist_ok=True)
np.save("gpurun_out/bench_q.npy", q)
g = q @ q.T
off = g[~np.eye(B, dtype=bool)]
print(f"queries {q.shape}: mean cos to each other {off.mean():.5f} (min {off.min():.5f}); "
      f"mean vector norm {np.linalg.norm(q.mean(0)):.4f}; per-dim std min/median/max "
      f"{q.std(0).min():.2e}/{np.median(q.std(0)):.2e}/{q.std(0).max():.2e}; "
      f"|q| max per dim {np.abs(q).max():.3f}; fraction |x| < 1e-3: {(np.abs(q) < 1e-3).mean():.3f}", flush=True)
N = 1_600_000
gal = bench.make_gallery(N, 2048, 0, N, dev)
gbf, _ = ops.quantize_rows(gal, "bf16")
bound = ops.prefilter_gallery_bound(gal, gbf)
ws = torch.empty(ops.cosine_topk_prefilter_workspace_size(B, N, 2048, 100), dtype=torch.uint8, device=dev)
for form in (0, 1):
    with ops.tuning(0, sweep_form=form):
        ops.cosine_topk_prefilter(d, gal, gbf, bound, 100, workspace=ws)
        torch.cuda.synchronize()
        cnt = ops.prefilter_survivors(ws, B, N, 2048, 100).cpu().numpy()
    print(f"sweep_form {form}: survivors per query mean {cnt.mean():.0f} min {cnt.min()} max {cnt.max()}", flush=True)
