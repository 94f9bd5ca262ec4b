"""Prefilter survivor counts on independent Gaussian queries vs bench.py's
descriptors: reuse of one workspace across query sets (debug aid)."""
import sys, torch
sys.path.insert(0, "/root/repo")
import bench
from research_image_retrieval_amd import ops
dev = torch.device("cuda:0")
n, d, k, nq = 1_600_000, 2048, 100, 1280
g = bench.make_gallery(n, d, 0, n, dev)
gb, _ = ops.quantize_rows(g, "bf16")
bound = ops.prefilter_gallery_bound(g, gb)
lo_ws, full_ws = ops.ranker_workspace_bounds("prefilter", nq, n, d, k)
ws = torch.empty(full_ws, dtype=torch.uint8, device=dev)
print("ws", full_ws, ops.cosine_topk_prefilter_workspace_size(nq, n, d, k), flush=True)
qa = ops.l2_normalize(torch.randn(nq, d, generator=torch.Generator().manual_seed(4321)).to(dev))
qb = ops.l2_normalize(torch.randn(nq, d, generator=torch.Generator().manual_seed(7)).to(dev))
qc = ops.l2_normalize((torch.randn(1, d, generator=torch.Generator().manual_seed(9)) +
                       1e-3 * torch.randn(nq, d, generator=torch.Generator().manual_seed(10))).to(dev))
for name, q in (("A", qa), ("B", qb), ("C", qc), ("A", qa)):
    s, i = ops.cosine_topk_prefilter(q, g, gb, bound, k, workspace=ws)
    sv = ops.prefilter_survivors(ws, nq, n, d, k).float()
    print(name, sv.mean().item(), sv.min().item(), sv.max().item(), sv[:4].tolist(), flush=True)
net = bench.build_extractor("resnet101", dev)
imgs = torch.randint(0, 256, (64, 224, 224, 3), dtype=torch.uint8, device=dev)
f = net.forward_test_u8(imgs)
torch.cuda.synchronize()
print("tuning", ops.get_tuning(0) if hasattr(ops, "get_tuning") else None, flush=True)
for name, q in (("A", qa), ("B", qb)):
    s, i = ops.cosine_topk_prefilter(q, g, gb, bound, k, workspace=ws)
    sv = ops.prefilter_survivors(ws, nq, n, d, k).float()
    print("after trunk", name, sv.mean().item(), sv.min().item(), sv.max().item(), sv[:4].tolist(), flush=True)
