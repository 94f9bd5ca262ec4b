import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
t0 = time.time()
def p(*a):
    print(f"[{time.time()-t0:7.2f}s]", *a, flush=True)
import torch
p("torch imported", torch.__version__)
p("cuda avail", torch.cuda.is_available(), torch.cuda.get_device_name(0))
x = torch.ones(10, device="cuda"); torch.cuda.synchronize(); p("tensor ok", x.sum().item())
from research_image_retrieval_amd import ops, _lib
p("lib", _lib.lib().rr_version())
import numpy as np
which = sys.argv[1] if len(sys.argv) > 1 else "all"
q = torch.nn.functional.normalize(torch.randn(37, 96, device="cuda"), dim=1)
g = torch.nn.functional.normalize(torch.randn(1000, 96, device="cuda"), dim=1)
p("inputs ready")
s = ops.cosine_scores(q, g); p("launched scores"); torch.cuda.synchronize(); p("scores done", s.shape, float((s.T - q @ g.T).abs().max()))
q2 = torch.nn.functional.normalize(torch.randn(200, 96, device="cuda"), dim=1)
s = ops.cosine_scores(q2, g); torch.cuda.synchronize(); p("scores 2x2 cfg done", float((s.T - q2 @ g.T).abs().max()))
si, ii = ops.cosine_topk(q, g, 10); torch.cuda.synchronize(); p("topk small done", ii[0, :5].tolist())
g2 = torch.nn.functional.normalize(torch.randn(50000, 96, device="cuda"), dim=1)
si, ii = ops.cosine_topk(q, g2, 10); torch.cuda.synchronize(); p("topk filter-path done", ii[0, :5].tolist())
ref = torch.topk(q @ g2.T, 10, dim=1)
p("matches torch.topk idx:", bool((ref.indices == ii).all()), float((ref.values - si).abs().max()))
