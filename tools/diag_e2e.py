"""Per-image / per-stage error of the C3 extractor at the bench batch vs the
oracle (diagnostic for tests/test_gpu_e2e.py)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import embed_ref  # noqa: E402
from research_image_retrieval_amd import ops  # noqa: E402
from research_image_retrieval_amd import weights as W  # noqa: E402
from research_image_retrieval_amd.networks import GeM, ConvDimReduction, GeMPCAw  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1280
dev = torch.device("cuda:0")
sd = W.synthetic_resnet_state_dict("resnet101", 0)
ww, wb = W.synthetic_linear(2048, 2048, 1)
pw, pb = W.synthetic_linear(2048, 2048, 5, scale=1.0 / np.sqrt(2048))
net = GeM(2048, backbone="resnet101", state_dict=sd, whiten=(ww, wb), device=dev)
pca = ConvDimReduction(2048, 2048, device=dev)
pca.set_params(pw, pb)
rs = np.random.RandomState(1234)
imgs = torch.from_numpy(rs.randint(0, 256, size=(B, 224, 224, 3), dtype=np.uint8))
x = ops.preprocess_u8(imgs.to(dev), out_c=4)
f = net.backbone(x)
g = net.pooling(f)
h = ops.l2_normalize(ops.linear(g, net.whiten_w, net.whiten_b))
p = ops.l2_normalize(pca(h))
pick = np.unique(np.linspace(0, B - 1, 8).astype(np.int64))
L = W.RESNET_LAYERS["resnet101"]
torch.set_num_threads(16)
for i in pick:
    xi = embed_ref.normalize_u8(imgs[i:i + 1])
    with torch.no_grad():
        tr = embed_ref.resnet_trunk(xi, sd, L)
        gr = embed_ref.gem(tr)
        hr = torch.nn.functional.normalize(torch.nn.functional.conv2d(gr, ww.view(2048, 2048, 1, 1), wb).flatten(1),
                                           dim=-1)
        pr = embed_ref.pcaw_apply(hr, pw, pb)
    e_t = (f[i].cpu().permute(2, 0, 1) - tr[0]).abs().max().item()
    e_g = (g[i].cpu() - gr.flatten()).abs().max().item()
    e_h = (h[i].cpu() - hr[0]).abs().max().item()
    e_p = (p[i].cpu() - pr[0]).abs().max().item()
    # PCA-w alone on the oracle's input (isolates the last linear)
    p_only = ops.l2_normalize(pca(hr.to(dev))).cpu()
    e_po = (p_only[0] - pr[0]).abs().max().item()
    print(f"img {i:5d}: trunk {e_t:.2e} (max {tr.abs().max():.3f}) gem {e_g:.2e} (max {gr.abs().max():.3f}) "
          f"whiten+L2 {e_h:.2e} pcaw+L2 {e_p:.2e} | pcaw on oracle input {e_po:.2e} | |pre-L2 pcaw| "
          f"{torch.nn.functional.linear(hr, pw, pb).norm():.3f}", flush=True)
