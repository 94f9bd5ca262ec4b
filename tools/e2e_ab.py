"""Interleaved A/B of tuning keys on the C3 bench's own work (bench.py's
images, extractor, gallery and prefilter ranker on its real descriptors), in
one process: the embed's wall time per config and the ranker's filter-sweep
HIP-event time per config, rounds interleaved, medians.  Rankings are checked
bit for bit between the ranker configs.
usage: E2E_EMBED="conv_il=0 conv_il=1" E2E_RANK="sweep_il=0,sweep_mf16=0 sweep_il=1,sweep_mf16=1"
       [E2E_WORKLOAD=c4: the ViT-B/16 bf16 embed instead (E2E_RANK unsupported)] python tools/e2e_ab.py [B] [rounds]"""
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from research_image_retrieval_amd import _lib, ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1280
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 4
parse = lambda spec: {k: int(v) for k, v in (kv.split("=") for kv in spec.split(",") if kv)}  # noqa: E731
EMB = os.environ.get("E2E_EMBED", "").split()
RNK = os.environ.get("E2E_RANK", "").split()
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
N = 1_600_000
if os.environ.get("E2E_WORKLOAD") == "c4":  # bench.py --workload c4's ViT-B/16 bf16 extractor
    from research_image_retrieval_amd import weights as W  # noqa: E402
    from research_image_retrieval_amd.networks import VisionTransformer  # noqa: E402
    net = VisionTransformer(224, 16, 768, 12, 12, 512, dtype="bf16", state_dict=W.synthetic_vit_state_dict(out_dim=512, seed=0),
                            device=dev)
else:
    net = bench.build_extractor("resnet101", dev)
rs = np.random.RandomState(1234)  # bench.py's rank-0 images
imgs = torch.from_numpy(rs.randint(0, 256, size=(B, 224, 224, 3), dtype=np.uint8)).to(dev)


def wall(fn, reps=2):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def split(c):
    """spec -> (rr_set_tuning keys, extractor attributes: keys that are not
    tuning keys, e.g. ln_fold=0 on the ViT)"""
    kv = parse(c)
    return ({k: v for k, v in kv.items() if k in ops._TUNE_KEYS},
            {k: v for k, v in kv.items() if k not in ops._TUNE_KEYS})


def owner(k):
    """the extractor object holding attribute k: the extractor itself or a
    nested part (GeMPCAw.net, GeM.backbone: e.g. fuse_stem_pool on the trunk)"""
    o = net
    while not hasattr(o, k):
        o = getattr(o, "net", None) or getattr(o, "backbone", None)
        if o is None:
            raise AttributeError(k)
    return o


if EMB:
    res = {c: [] for c in EMB}
    for _ in range(ROUNDS):
        for c in EMB:
            tk, attrs = split(c)
            saved = {k: getattr(owner(k), k) for k in attrs}
            for k, v in attrs.items():
                setattr(owner(k), k, bool(v) if isinstance(saved[k], bool) else v)
            with ops.tuning(0, **tk):
                res[c].append(wall(lambda: net.forward_test_u8(imgs)))
            for k, v in saved.items():
                setattr(owner(k), k, v)
    for c in EMB:
        print(f"embed {c:40s} median {statistics.median(res[c]):8.3f} ms  all {['%.2f' % v for v in res[c]]}",
              flush=True)
if RNK:
    d = net.forward_test_u8(imgs)
    gal = bench.make_gallery(N, 2048, 0, N, dev)
    gbf, _ = ops.quantize_rows(gal, "bf16")
    bound = ops.prefilter_gallery_bound(gal, gbf)
    lo_ws, full_ws = ops.ranker_workspace_bounds("prefilter", B, N, 2048, 100)
    ws = torch.empty(max(lo_ws, min(full_ws, 4 << 30)), dtype=torch.uint8, device=dev)
    timer = ops.KernelTimer(0)
    res, outs = {c: [] for c in RNK}, {}
    for _ in range(ROUNDS):
        for c in RNK:
            with ops.tuning(0, **parse(c)):
                ops.cosine_topk_prefilter(d, gal, gbf, bound, 100, workspace=ws, max_workspace_bytes=4 << 30)
                torch.cuda.synchronize()
                timer.enable(True)
                for _ in range(2):
                    s, i = ops.cosine_topk_prefilter(d, gal, gbf, bound, 100, workspace=ws, max_workspace_bytes=4 << 30)
                torch.cuda.synchronize()
                ms = timer.collect(_lib.TIME_COSINE)[0] / 2
                timer.enable(False)
            res[c].append(ms)
            outs[c] = (s, i)
    base = RNK[0]
    for c in RNK:
        same = torch.equal(outs[c][1], outs[base][1]) and torch.equal(outs[c][0].view(torch.int32),
                                                                      outs[base][0].view(torch.int32))
        print(f"sweep {c:40s} median {statistics.median(res[c]):8.3f} ms  all {['%.3f' % v for v in res[c]]}  "
              f"identical: {same}", flush=True)
