"""bench.py — images embedded + ranked per second against a 1.6M x 2048 gallery
(BASELINE.json metric), on librr's gfx950 kernels.

Workload (config C3 of BASELINE.json, the one the metric is quoted on; it fits
one MI355X: the 1.6M x 2048 fp32 gallery is 13.1 GB of the 288 GB HBM):
  per GPU and step: B synthetic uint8 224x224x3 images (resident in HBM) ->
  ToTensor+Normalize -> ResNet-101 (BN folded) -> GeM(p=3) -> whiten 1x1 conv
  -> L2 -> PCA-whitening (2048 -> 2048) -> L2 -> exact stable top-100 cosine
  search against the WHOLE gallery.
  N GPUs: one process per GPU (torch.distributed.run), gallery row-sharded
  (1.6M/N rows each), query descriptors all-gathered over RCCL, per-shard
  fused top-k, partial lists exchanged by all-to-all, k-way merge.  Per-GPU
  work is fixed as N grows ("weak" scaling): value = N * B * K / max-over-ranks time.

One JSON line on rank 0 with the contract keys plus `roofline` (dominant
kernel by measured time, HIP events on the launch stream), `roofline_by_kernel`
and `cpu_baseline` (oracle CPU restatement of the reference path, rank 0, N=1).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from research_image_retrieval_amd import _lib, ops  # noqa: E402
from research_image_retrieval_amd import weights as W  # noqa: E402
from research_image_retrieval_amd.distributed import ShardedGallery, shard_bounds, sharded_step  # noqa: E402
from research_image_retrieval_amd.networks import GeM, ConvDimReduction, GeMPCAw, VisionTransformer  # noqa: E402
from research_image_retrieval_amd.extract import _rescale  # noqa: E402

METRIC = "images embedded+ranked/sec on 1.6M×2048 gallery; mAP on ROxf/RPar"
# MI355X_MICROARCH.md: dense MFMA peaks (TFLOP/s) per input dtype, HBM3E peak.
# "h2": three fp16 MFMA products per fp32 product (the f16x2 split), so its
# ceiling in algorithmic fp32 FLOP/s is the fp16 dense peak (= bf16's) / 3;
# "s3": the ceiling of round 2's retired six-product bf16 split (the bf16
# peak / 6), kept only as the frac_of_bf16x3_ceiling comparison.
PEAK_TFLOPS = {"fp32": 157.3, "bf16": 2500.0, "fp8": 5000.0, "s3": 2500.0 / 6, "h2": 2500.0 / 3}
SPLIT_MATH = {
    "h2": (3, "fp32-accurate f16x2 split at power-of-two scales: 3 fp16 MFMA products per fp32 product "
              "(a0b0 + a0b1 + a1b0), fp32 accumulation; tested bar vs float64 (tests/test_gpu_h2.py): per conv "
              "mean error <= 1.05x the exact-fp32 core's and max <= 1.25x (1.5x for the fused stage-entry "
              "bottleneck), descriptors <= 2x the exact-fp32 trunk's and <= 1e-6; peak = fp16 dense peak / 3"),
}
WEIGHT_BYTES = {"h2": 4, "f32": 4}
PEAK_HBM_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


GLDV2_CLASSES = 81313  # GLDv2-clean: 1,580,470 images of 81,313 landmarks (dataset/configdataset.py:443)


def make_gallery(n_total, d, lo, hi, device, seed=0, kind="gaussian"):
    """Rows [lo, hi) of a seeded gallery, L2-normalised, generated on the GPU
    in 64k-row blocks keyed by global block index (shard-invariant).
    kind "gaussian": isotropic rows.  kind "clustered": landmark-like rows,
    normalize(centre[c] + noise) with |noise| = |centre| (cosine ~0.7 to the
    class centre, ~0.5 between members of a class), the class of each row drawn
    from GLDV2_CLASSES seeded centres: the prefilter's worst case, many rows
    crowding near a query's top-k threshold."""
    g = torch.empty((hi - lo, d), dtype=torch.float32, device=device)
    blk = 65536
    gen = torch.Generator(device=device)
    centres = None
    if kind == "clustered":
        gen.manual_seed(seed * 1_000_003 + 999_983)
        centres = torch.randn((GLDV2_CLASSES, d), generator=gen, device=device)
        centres = ops.l2_normalize(centres, 1e-12, out=centres)
    b0 = lo // blk
    for b in range(b0, (hi + blk - 1) // blk):
        gen.manual_seed(seed * 1_000_003 + b)
        rows = torch.randn((blk, d), generator=gen, device=device)
        if centres is not None:
            cls = torch.randint(0, GLDV2_CLASSES, (blk,), generator=gen, device=device)
            rows = centres[cls] + rows / d ** 0.5
        s, e = max(lo, b * blk), min(hi, (b + 1) * blk)
        g[s - lo:e - lo] = rows[s - b * blk:e - b * blk]
    ops.l2_normalize(g, 1e-12, out=g)
    return g


def build_extractor(arch, device, seed=0, conv_math="h2"):
    net = GeM(2048, backbone=arch, seed=seed, device=device, conv_math=conv_math)
    pw = ConvDimReduction(2048, 2048, device=device)
    w, b = W.synthetic_linear(2048, 2048, seed + 5, scale=1.0 / np.sqrt(2048))
    pw.set_params(w, b)
    return GeMPCAw(net, pw)


def host_threads():
    """torch.set_num_threads(len(os.sched_getaffinity(0))) --
    capped by the CPU share the job is actually granted: a cgroup CPU quota, or
    the OMP_NUM_THREADS the GPU box exports (its affinity mask shows the whole
    machine, 256 CPUs, of which the box grants 16; 256 threads on 16 cores ran
    the batch-1 R50 embed 60x slower).  Returns (affinity, cap, threads)."""
    affinity = len(os.sched_getaffinity(0))
    cap = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            cap = max(1, int(int(q) // int(p)))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        cap = int(omp) if cap is None else min(cap, int(omp))
    return affinity, cap, (min(affinity, cap) if cap else affinity)


def cpu_baseline(arch, n_total, d, k, seed=0):
    """The reference's CPU path, timed on a bounded sample on this host:
    batch-1 extraction (utils/helpfunc.py:18-48 semantics) through the oracle's
    torch-CPU restatement of ResNet->GeM->whiten->L2->PCA-w->L2, then the
    ranker of iris_evaluate.py:383-386 (torch.mm + full np.argsort) against a
    400k-row gallery sample, scaled to the full gallery.  The same extraction
    is also timed at batch 32 ("timed at batch 1 ... and
    batch 32"): value_b32 / embed_s_per_image_b32."""
    from oracle import embed_ref
    affinity, quota, threads = host_threads()
    default_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    n_img, n_q, n_g = 160, 64, 400_000  # ~10-15 s of CPU work on the box's 16-core share
    n_b32 = 2  # timed batches of 32 images (after one untimed batch)
    sd = W.synthetic_resnet_state_dict(arch, seed)
    ww, wb = W.synthetic_linear(2048, 2048, seed + 1)
    pw, pb = W.synthetic_linear(2048, 2048, seed + 5, scale=1.0 / np.sqrt(2048))
    rs = np.random.RandomState(1234)
    imgs = torch.from_numpy(rs.randint(0, 256, size=(n_img, 224, 224, 3), dtype=np.uint8))
    layers = W.RESNET_LAYERS[arch]
    with torch.no_grad():
        x = embed_ref.normalize_u8(imgs[:1])
        embed_ref.gem_net_forward_test(x, sd, layers, ww, wb)  # warm-up
        t0 = time.perf_counter()
        for i in range(n_img):
            x = embed_ref.normalize_u8(imgs[i:i + 1])
            f = embed_ref.gem_net_forward_test(x, sd, layers, ww, wb)
            embed_ref.pcaw_apply(f, pw, pb)
        t_embed = (time.perf_counter() - t0) / n_img
        imgs32 = torch.from_numpy(rs.randint(0, 256, size=(32, 224, 224, 3), dtype=np.uint8))
        for it in range(n_b32 + 1):
            if it == 1:
                t0 = time.perf_counter()
            f = embed_ref.gem_net_forward_test(embed_ref.normalize_u8(imgs32), sd, layers, ww, wb)
            embed_ref.pcaw_apply(f, pw, pb)
        t_embed32 = (time.perf_counter() - t0) / (32 * n_b32)
        gen = torch.Generator().manual_seed(7)
        gal = torch.nn.functional.normalize(torch.randn(n_g, d, generator=gen), dim=1)
        q = torch.nn.functional.normalize(torch.randn(n_q, d, generator=gen), dim=1)
        t0 = time.perf_counter()
        sim = torch.mm(q, gal.t()).numpy()
        t_mm = time.perf_counter() - t0
        t0 = time.perf_counter()
        np.argsort(-sim, axis=1)
        t_sort = time.perf_counter() - t0
        t0 = time.perf_counter()
        torch.topk(torch.from_numpy(sim), k, dim=1)
        t_topk = time.perf_counter() - t0
    scale = n_total / n_g
    t_rank = (t_mm + t_sort) * scale / n_q  # per query, full gallery, reference argsort
    t_rank_topk = (t_mm + t_topk) * scale / n_q
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    torch.set_num_threads(default_threads)
    return {"value": 1.0 / (t_embed + t_rank), "unit": "images/s", "cores": threads, "kind": "port",
            "affinity_cpus": affinity, "granted_cpus": quota, "torch_default_threads": default_threads,
            "sample": f"{n_img} images embedded at batch 1 (224x224, {arch}-GeM+PCA-w, fp32) + {n_q} queries "
                      f"ranked against a {n_g}-row x {d} gallery sample (torch.mm + full np.argsort), "
                      f"rank time scaled x{scale:.0f} to {n_total} rows; batch-32 figures: {n_b32} timed batches "
                      f"of 32 images after one untimed batch, same ranker time",
            "embed_s_per_image": t_embed, "rank_s_per_query_argsort": t_rank, "rank_s_per_query_topk": t_rank_topk,
            "value_with_topk": 1.0 / (t_embed + t_rank_topk),
            "embed_s_per_image_b32": t_embed32, "value_b32": 1.0 / (t_embed32 + t_rank), "cpu_model": model}


# ---- config C2: ResNet50-GeM 512-d at imsize 1024 over a ROxford5k-shaped set ----
# (H, W) after thumbnail(1024) and the share of the gallery at that size
C2_SIZES = ((768, 1024, 0.70), (1024, 768, 0.22), (683, 1024, 0.06), (1024, 683, 0.02))
C2_BATCH = 128  # same-size gallery images per extractor call (the reference runs batch 1; 16 -> 128: +15 %)


def c2_layout(n_gallery, n_query, seed=1234):
    """Sizes of the gallery groups and of the query crops (bbox crops of
    1024-px images, dataset/ImageFromList.py:40-57: kept at their crop size)."""
    counts = [int(round(n_gallery * f)) for _, _, f in C2_SIZES]
    counts[0] += n_gallery - sum(counts)
    rs = np.random.RandomState(seed)
    qs = [(int(rs.randint(200, 769)), int(rs.randint(200, 1025))) for _ in range(n_query)]
    return [(h, w, c) for (h, w, _), c in zip(C2_SIZES, counts)], qs


def cpu_baseline_c2(sets, d=512, seed=0):
    """The reference CPU path for C2, timed on a bounded sample: batch-1
    extraction of 50 gallery images at 768x1024 (utils/helpfunc.py:18-48
    through the oracle's R50-GeM-512 restatement), and the full ranking of
    every set's queries against its whole gallery (torch.mm + np.argsort,
    iris_evaluate.py:383-386); the job time = all images x per-image embed +
    the rankings.  sets: [(n_gallery, n_query), ...]."""
    from oracle import embed_ref
    affinity, granted, threads = host_threads()
    default_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    sd = W.synthetic_resnet_state_dict("resnet50", seed)
    pw, pb = W.synthetic_linear(d, 2048, seed + 2)
    rs = np.random.RandomState(1234)
    n_img = 50  # ~10 s of CPU work (0.2 s per image on the box's 16-core share)
    imgs = torch.from_numpy(rs.randint(0, 256, size=(n_img + 1, 768, 1024, 3), dtype=np.uint8))
    with torch.no_grad():
        embed_ref.gem_model_descriptor(embed_ref.normalize_u8(imgs[:1]), sd, W.RESNET_LAYERS["resnet50"], pw, pb)
        t0 = time.perf_counter()
        for i in range(1, n_img + 1):
            embed_ref.gem_model_descriptor(embed_ref.normalize_u8(imgs[i:i + 1]), sd, W.RESNET_LAYERS["resnet50"],
                                           pw, pb)
        t_embed = (time.perf_counter() - t0) / n_img
        gen = torch.Generator().manual_seed(7)
        t_rank = 0.0
        for n_gallery, n_query in sets:
            g = torch.nn.functional.normalize(torch.randn(n_gallery, d, generator=gen), dim=1)
            q = torch.nn.functional.normalize(torch.randn(n_query, d, generator=gen), dim=1)
            t0 = time.perf_counter()
            np.argsort(-torch.mm(q, g.t()).numpy(), axis=1)
            t_rank += time.perf_counter() - t0
    torch.set_num_threads(default_threads)
    n_all = sum(g_ + q_ for g_, q_ in sets)
    total = n_all * t_embed + t_rank
    return {"value": n_all / total, "unit": "images/s", "cores": threads, "kind": "port",
            "affinity_cpus": affinity, "granted_cpus": granted,
            "sample": f"{n_img} images embedded at batch 1 (768x1024, resnet50-GeM 512-d, fp32) and the full ranking of "
                      + " + ".join(f"{q_} queries x {g_} rows" for g_, q_ in sets)
                      + f" (torch.mm + np.argsort); job time = {n_all} x per-image embed + rankings",
            "embed_s_per_image": t_embed, "rank_s": t_rank, "torch_default_threads": default_threads}


# RR_FORCE_SHARDED=1 (with torch.distributed.run --nproc-per-node 1): run the
# multi-GPU path — process group (RCCL), ShardedGallery, collectives — on a
# world of one, so its RCCL calls execute on a 1-GPU box
DIST_ON = False


C2_SETS = {"roxford5k": (4993, 70), "rparis6k": (6322, 70)}  # revisitop sizes (dataset/configdataset.py:27-57)


def run_c2(a, world, rank, dev):
    """C2: ResNet50-GeM 512-d fp32 (Table-1 GeMModel) over full ROxford5k- and
    RParis6k-shaped sets at imsize 1024 -- 4,993 + 6,322 gallery images and
    70 + 70 query crops, every image embedded (gallery images in same-size
    batches, queries one by one at their own crop size), full ranks of each
    dataset's queries against its gallery and the revisited mAP
    (utils/evaluate.py:153-194) on the host.  One step = both sets (or the one
    --c2-dataset names); N ranks split the images (strong scaling),
    descriptors are all-gathered over RCCL and rank 0 ranks and scores.

    Conv-class time for the roofline: the gallery phases run on one stream,
    so their per-launch HIP events do not overlap and are summed; the query
    phases run batch-1 crops on concurrent streams, whose event spans overlap,
    so each query phase counts with its whole wall time on the main stream
    (an upper bound on its conv time).  The sum never exceeds the step."""
    from research_image_retrieval_amd.distributed import _all_gather_var
    from research_image_retrieval_amd.evaluate import compute_map_and_print
    from research_image_retrieval_amd.models import get_model
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import inputs as I  # noqa: E402  (synthetic revisitop-shaped ground truth)
    names = list(C2_SETS) if a.c2_dataset == "both" else [a.c2_dataset]
    net = get_model("gem_r50", 1000, feature_dim=512, seed=0, device=dev, conv_math=a.conv_math)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234)
    sets = []
    for si, name in enumerate(names):
        n_g, n_q = C2_SETS[name]
        if a.c2_gallery:
            n_g = a.c2_gallery
        if a.c2_queries:
            n_q = a.c2_queries
        groups, qsizes = c2_layout(n_g, n_q, seed=1234 + si)
        # this rank's images (contiguous share of the gallery order, and of the queries)
        glo, ghi = shard_bounds(n_g, world, rank)
        qlo, qhi = shard_bounds(n_q, world, rank)
        batches, start = [], 0
        for h, w, c in groups:
            lo, hi = max(start, glo), min(start + c, ghi)
            for b0 in range(lo, hi, a.c2_batch):
                nb = min(a.c2_batch, hi - b0)
                batches.append(torch.randint(0, 256, (nb, h, w, 3), dtype=torch.uint8, device=dev, generator=gen))
            start += c
        queries = [torch.randint(0, 256, (1, h, w, 3), dtype=torch.uint8, device=dev, generator=gen)
                   for (h, w) in qsizes[qlo:qhi]]
        gnd, _ = I.map_inputs(31 + si, nq=n_q, n=n_g)
        img_flops = sum(c_ * (sum(W.resnet_conv_flops("resnet50", h, w).values()) + 2 * 2048 * 512)
                        for (h, w, c_) in [(h, w, max(0, min(s0 + c, ghi) - max(s0, glo)))
                                           for (h, w, c), s0 in zip(groups, np.cumsum([0] + [g[2] for g in groups]))])
        img_flops += sum(sum(W.resnet_conv_flops("resnet50", h, w).values()) + 2 * 2048 * 512
                         for (h, w) in qsizes[qlo:qhi])
        sets.append({"name": name, "n_g": n_g, "n_q": n_q, "batches": batches, "queries": queries, "gnd": gnd,
                     "flops": img_flops})
    torch.cuda.synchronize()
    # batch-1 query crops (all sizes differ): small grids, so C2_QSTREAMS of them
    # run concurrently on side streams
    qstreams = [torch.cuda.Stream(dev) for _ in range(a.c2_qstreams)] if a.c2_qstreams > 1 else []
    timer = ops.KernelTimer(dev.index)
    acct = {"conv_ms": 0.0, "conv_n": 0, "qphase_ms": 0.0, "on": False}

    def embed_queries(queries):
        if not queries:
            return torch.empty((0, 512), device=dev)
        if not qstreams:
            return torch.cat([net.forward_test_u8(q) for q in queries], 0)
        cur = torch.cuda.current_stream(dev)
        for st in qstreams:
            st.wait_stream(cur)
        outs = []
        for j, q in enumerate(queries):
            with torch.cuda.stream(qstreams[j % len(qstreams)]):
                outs.append(net.forward_test_u8(q))
        for st in qstreams:
            cur.wait_stream(st)
        for o in outs:
            o.record_stream(cur)
        return torch.cat(outs, 0)

    def step(marks=None):
        def mark(name):
            if marks is not None:
                torch.cuda.synchronize()
                marks.append((name, time.perf_counter()))
        mark("start")
        maps, qev = {}, []
        for st in sets:
            if acct["on"]:
                timer.enable(True)
            gd = torch.cat([net.forward_test_u8(b) for b in st["batches"]], 0) if st["batches"] else \
                torch.empty((0, 512), device=dev)
            if acct["on"]:  # gallery phase: one stream, events do not overlap
                ms, n = timer.collect(_lib.TIME_GEMM)
                acct["conv_ms"] += ms
                acct["conv_n"] += n
                timer.enable(False)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            mark(st["name"] + "_gallery_embed")
            qd = embed_queries(st["queries"])
            if acct["on"]:  # query phase: concurrent streams, counted by its wall time
                e1.record()
                qev.append((e0, e1))
            mark(st["name"] + "_query_embed")
            if DIST_ON:
                gd = torch.cat(_all_gather_var(gd.contiguous(), None)[0], 0)
                qd = torch.cat(_all_gather_var(qd.contiguous(), None)[0], 0)
            mark(st["name"] + "_all_gather")
            if rank != 0:
                continue
            s, i = ops.cosine_topk(qd.contiguous(), gd.contiguous(), st["n_g"])  # full ranks (k = N)
            ranks = i.cpu().numpy().T.copy()
            mark(st["name"] + "_rank")
            import contextlib
            with contextlib.redirect_stdout(sys.stderr):  # stdout carries only the JSON line
                maps[st["name"]] = compute_map_and_print(st["name"], "c2", "global", ranks, st["gnd"])
            mark(st["name"] + "_map")
        for e0, e1 in qev:
            e1.synchronize()
            acct["qphase_ms"] += e0.elapsed_time(e1)
        return maps

    for _ in range(a.warmup):
        step()
    marks = []
    step(marks)  # one more untimed step with a sync at every phase boundary
    phases = {b[0]: round((b[1] - a_[1]) * 1e3, 2) for a_, b in zip(marks, marks[1:])}
    log(f"[rank {rank}] c2 phases (ms, synchronised step): {phases}")
    acct["on"] = True
    if DIST_ON:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        maps = step()
    if DIST_ON:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if DIST_ON:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    units = sum(st["n_g"] + st["n_q"] for st in sets)
    value = units * a.steps / elapsed
    # algorithmic FLOPs of this rank's share: every image's trunk convs + the 2048->512 projection
    img_flops = sum(st["flops"] for st in sets)
    rk = {}
    conv_ms = acct["conv_ms"] + acct["qphase_ms"]
    if acct["conv_n"]:
        sec = conv_ms / 1e3 / a.steps
        dt = a.conv_math if a.conv_math in SPLIT_MATH else "fp32"
        ach = img_flops / sec / 1e12
        rk["conv_gemm"] = {"bound": "mfma", "achieved": round(ach, 2), "peak": PEAK_TFLOPS[dt], "unit": "TFLOP/s",
                           "frac": round(ach / PEAK_TFLOPS[dt], 4), "dtype": "fp32",
                           "ms_per_step": round(conv_ms / a.steps, 3),
                           "gallery_conv_kernel_ms_per_step": round(acct["conv_ms"] / a.steps, 3),
                           "query_phase_wall_ms_per_step": round(acct["qphase_ms"] / a.steps, 3),
                           "timing": "gallery phases: summed per-launch HIP events (one stream); query phases "
                                     "(8 concurrent streams): whole phase wall time on the main stream",
                           "gallery_launches_per_step": acct["conv_n"] / a.steps,
                           "algorithmic_flop_per_step": img_flops, "algorithmic_bytes_per_launch": None,
                           "traffic": None}
        if dt in SPLIT_MATH:
            rk["conv_gemm"]["math"] = SPLIT_MATH[dt][1]
            rk["conv_gemm"]["mfma_flop_per_step"] = SPLIT_MATH[dt][0] * img_flops
            if dt == "h2":
                rk["conv_gemm"]["frac_of_bf16x3_ceiling"] = round(ach / PEAK_TFLOPS["s3"], 4)
    roof = dict(rk.get("conv_gemm", {}))
    roof["kernel"] = "conv_gemm"
    desc = " + ".join(f"{st['name']} ({st['n_g']} gallery + {st['n_q']} query images)" for st in sets)
    res = {"metric": METRIC, "value": round(value, 2), "unit": "images/s", "n_gpus": world, "steps": a.steps,
           "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
           "scaling": "strong", "vs_baseline": None, "dtype": "fp32",
           "data": "synthetic: uint8 images at ROxford5k's post-thumbnail(1024) sizes (768x1024 / 1024x768 / 683x1024 / "
                   "1024x683, the same mix for RParis6k) and random 200-768 x 200-1024 query crops, "
                   "torch.Generator(1234); synthetic revisitop-shaped gnd (mAP is pipeline parity, not accuracy); "
                   "seeded weights",
           "config": {"workload": f"C2: resnet50-GeM 512-d fp32 (Table-1 GeMModel), {desc} at imsize 1024, "
                                  f"full ranks + revisited mAP per dataset",
                      "global_batch": units, "datasets": [st["name"] for st in sets],
                      "gallery_rows": [st["n_g"] for st in sets], "queries": [st["n_q"] for st in sets], "dim": 512,
                      "gallery_batch": a.c2_batch, "parallelism": f"image-dp{world}", "conv_math": a.conv_math},
           "map_easy_medium_hard": {k: list(v) for k, v in maps.items()} if maps else None,
           "phases_ms_synchronised_step": phases,
           "roofline": roof, "roofline_by_kernel": rk}
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        t = time.time()
        res["cpu_baseline"] = cpu_baseline_c2([(st["n_g"], st["n_q"]) for st in sets])
        log(f"cpu baseline {time.time() - t:.1f}s")
    if rank == 0:
        print(json.dumps(res, default=_json_scalar), flush=True)
    if DIST_ON:
        dist.barrier()
        dist.destroy_process_group()


def seed_rows(n, k):
    """Rows of the rankers' threshold-seeding sample (librr seed_sample_rows)."""
    return min(n, max(k, 4096, min(32768, n // 48)))


def load_traffic():
    """Per-launch HBM bytes measured by rocprofv3 --pmc (profiles/traffic.json),
    corrected per MI355X_MICROARCH.md §HBM; None if not collected."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(p):
        try:
            return json.load(open(p))
        except (OSError, ValueError):
            return None
    return None


def _json_scalar(o):
    """numpy scalars (dataset sizes, FLOP counts) in the JSON line."""
    if hasattr(o, "item"):
        return o.item()
    raise TypeError(f"not JSON serializable: {type(o).__name__}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1280,
                    help="images per GPU per step (1280 = the BASELINE C3 batch; a larger batch amortises the "
                         "gallery sweep over more queries and fills the conv grids' last rounds better: round 2's "
                         "sweep on one box, profiles/r02l_batch_sweep.jsonl, was flat above 1280)")
    ap.add_argument("--gallery", type=int, default=1_600_000)
    ap.add_argument("--gallery-kind", choices=("gaussian", "clustered"), default="gaussian",
                    help="gaussian: isotropic rows; clustered: 81,313 landmark-like classes (the prefilter's "
                         "harder case: many rows near each query's top-k threshold)")
    ap.add_argument("--dim", type=int, default=2048)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--arch", default="resnet101")
    ap.add_argument("--workload", choices=("c2", "c3", "c4", "c5"), default="c3",
                    help="c2: ResNet50-GeM 512-d fp32 over ROxford5k- + RParis6k-shaped sets at imsize 1024 (full ranks + mAP); "
                         "c3: ResNet101-GeM 2048-d + PCA-w, fp32 (BASELINE metric config); "
                         "c4: ViT-B/16 CLS 512-d, bf16 GEMMs + bf16 cosine; "
                         "c5: c3 extractor at 3 scales + fp8 cosine + alpha-QE re-rank (sharded: neighbour rows fetched from their shards)")
    ap.add_argument("--dtype", choices=("fp32", "bf16", "fp8"), default=None,
                    help="GEMM input dtype (default: fp32 for c3, bf16 for c4)")
    ap.add_argument("--ranker", choices=("exhaustive", "prefilter"), default="prefilter",
                    help="fp32 exact ranking: exhaustive fp32 MFMA sweep, or the bf16-bound prefilter + exact "
                         "fp32 rescoring (bit-identical results)")
    ap.add_argument("--conv-math", choices=("h2", "f32"), default="h2",
                    help="ResNet trunk convs: h2 = fp32-accurate f16x2 split on the fp16 matrix cores, 3 MFMA "
                         "products per fp32 product (tested bar vs float64, tests/test_gpu_h2.py: per conv mean "
                         "error <= 1.05x and max <= 1.25x the exact-fp32 core's); f32 = exact fp32 MFMA")
    ap.add_argument("--ws-budget-gb", type=float, default=4.0,
                    help="ranker workspace budget per rank (bounded candidate buffers, overflowed queries re-run; "
                         "0 = the worst-case size, ~Q*N*8 bytes)")
    ap.add_argument("--pipeline", type=int, choices=(0, 1), default=None,
                    help="1: rank batch i on a second HIP stream while batch i+1 is embedded (n embeds + n rankings "
                         "per n steps either way)")
    ap.add_argument("--embed-streams", type=int, default=None,
                    help="C3: the trunk's batch cut into this many parts, each on its own HIP stream, part i+1 one "
                         "conv behind part i (networks forward_test_u8_streams; bit-identical to serial parts); "
                         "default 1; C3 also reports the overlapped schedule (2 streams + pipelined ranker)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the side measurements after the timed loop (the decorrelated-query sweep and the "
                         "overlapped schedule): tools/profile.sh, so that the profile holds the timed loop's launches")
    ap.add_argument("--c2-dataset", choices=("both", "roxford5k", "rparis6k"), default="both",
                    help="C2 sets per step (BASELINE C2: full ROxford5k + RParis6k)")
    ap.add_argument("--c2-gallery", type=int, default=0, help="override every C2 set's gallery size (0: revisitop's)")
    ap.add_argument("--c2-queries", type=int, default=0, help="override every C2 set's query count (0: 70)")
    ap.add_argument("--c2-batch", type=int, default=C2_BATCH, help="same-size gallery images per extractor call")
    ap.add_argument("--c2-qstreams", type=int, default=8, help="HIP streams for the batch-1 query crops (1: serial)")
    ap.add_argument("--tune", default="",
                    help="A/B only: rr_set_tuning keys for the whole run, e.g. sweep_il=0,conv_il=0 (ops._TUNE_KEYS)")
    a = ap.parse_args()
    if a.workload == "c4":
        if a.dim == 2048:
            a.dim = 512
        a.arch = "vit_b16"
    if a.dtype is None:
        a.dtype = {"c2": "fp32", "c3": "fp32", "c4": "bf16", "c5": "fp8"}[a.workload]
    if a.workload in ("c2", "c3") and a.dtype != "fp32":
        raise SystemExit(f"{a.workload} is defined in fp32 (the reference's arithmetic)")

    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # started bare with --gpus N: run ourselves under torch.distributed.run
        # as a child (nothing has touched the GPU yet in this process)
        import socket
        import subprocess
        sock = socket.socket()
        sock.bind(("127.0.0.1", 0))
        port = sock.getsockname()[1]
        sock.close()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.run(cmd).returncode)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        log(f"note: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    # one process per GPU; ranks beyond the visible devices share them (rehearsal)
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    global DIST_ON
    DIST_ON = world > 1 or os.environ.get("RR_FORCE_SHARDED") == "1"
    if DIST_ON:
        backend = os.environ.get("RR_DIST_BACKEND", "nccl")  # "gloo" only for 1-GPU rehearsals
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    if a.tune:  # held for the rest of the process (A/B runs; the default line sets nothing)
        ops.tuning(dev.index, **{k: int(v) for k, v in (kv.split("=") for kv in a.tune.split(","))}).__enter__()
    if a.workload == "c2":
        return run_c2(a, world, rank, dev)
    t_setup = time.time()
    lo, hi = shard_bounds(a.gallery, world, rank)
    gallery = make_gallery(a.gallery, a.dim, lo, hi, dev, kind=a.gallery_kind)
    if a.workload == "c4":
        net = VisionTransformer(224, 16, 768, 12, 12, a.dim, dtype="bf16" if a.dtype != "fp32" else "fp32",
                                state_dict=W.synthetic_vit_state_dict(out_dim=a.dim, seed=0), device=dev)
    else:
        net = build_extractor(a.arch, dev, conv_math=a.conv_math)
    rs = np.random.RandomState(1234 + rank)
    imgs = torch.from_numpy(rs.randint(0, 256, size=(a.batch, 224, 224, 3), dtype=np.uint8)).to(dev)
    q_total = a.batch * world
    pre = a.ranker == "prefilter" and a.dtype == "fp32"
    # ranker workspace: the worst case (every row a candidate, ~Q*N*8 bytes), or
    # --ws-budget-gb of bounded candidate buffers (overflowed queries re-run)
    ws_max = int(a.ws_budget_gb * (1 << 30)) if a.ws_budget_gb > 0 else None
    ws_lo, ws_full = ops.ranker_workspace_bounds("prefilter" if pre else "exact", q_total, hi - lo, a.dim, a.k)
    ws = torch.empty(ws_full if ws_max is None else max(ws_lo, min(ws_full, ws_max)), dtype=torch.uint8, device=dev)
    counts = [a.batch] * world  # every rank's query count: the sharded search needs no size exchange
    sharded = ShardedGallery(gallery, lo, workspace=ws, dtype=a.dtype, prefilter=pre,
                             max_workspace_bytes=ws_max) if DIST_ON else None
    gal_bf, gal_bound = (None, None)
    if pre and not DIST_ON:
        gal_bf, _ = ops.quantize_rows(gallery, "bf16")
        gal_bound = ops.prefilter_gallery_bound(gallery, gal_bf)
    gal_lp, gal_sc = ops.quantize_rows(gallery, a.dtype) if (a.dtype != "fp32" and not DIST_ON) else (None, None)
    torch.cuda.synchronize()
    log(f"[rank {rank}] setup {time.time() - t_setup:.1f}s: shard [{lo},{hi}) x {a.dim}, batch {a.batch}")

    scales = (1.0, 1.0 / np.sqrt(2.0), 0.5)  # C5 multi-scale set

    # the schedule of the timed steps (--embed-streams / --pipeline): one
    # stream by default, so that every kernel's HIP-event duration (the
    # rooflines) is its own.  C3 also times the overlapped schedule after the
    # main loop -- the trunk's batch in two parts on two HIP streams, batch i's
    # ranking on a third beside batch i+1's embed -- and reports it as
    # `overlapped_schedule` (its kernels co-run, so its per-launch durations
    # include the other streams' work).
    c3 = a.workload == "c3"
    n_es = a.embed_streams if a.embed_streams is not None else 1
    pipe = bool(a.pipeline) if a.pipeline is not None else False
    sched = {"streams": n_es if c3 else 1, "pipeline": pipe}
    e_streams = [torch.cuda.Stream(dev) for _ in range(max(2, n_es))] if c3 else None

    def embed():
        if sched["streams"] > 1:
            return net.forward_test_u8_streams(imgs, e_streams[:sched["streams"]], lag=1)
        if a.workload != "c5":
            return net.forward_test_u8(imgs)
        # multi-scale extraction (utils/helpfunc.py:30-46): rescale, embed, average, renormalise
        x = ops.preprocess_u8(imgs, out_c=4)
        acc = None
        for sc in scales:
            xs = x if sc == 1.0 else _rescale(x, sc)
            f = net.forward_test_nhwc(xs)
            acc = f.clone() if acc is None else acc.add_(f)
        acc.div_(len(scales))
        return ops.l2_normalize(acc, 1e-12, out=acc)

    def step():
        return rank_step(embed())

    def rank_step(desc):
        if sharded is not None:
            # C3 / C4: sharded search; C5: + alpha-QE with neighbour rows fetched
            # from their owning shards (bit-identical to 1 GPU); tests/test_distributed_gloo.py
            # drives this same sharded_step at world 2 and 4
            return sharded_step(sharded, desc, a.workload, a.k, counts, n=2, alpha=3.0)
        if a.workload == "c5":
            q_lp, q_sc = ops.quantize_rows(desc, a.dtype)
            s1, i1 = ops.cosine_topk_lp(q_lp, q_sc, gal_lp, gal_sc, a.k, a.dtype, idx_offset=lo, workspace=ws,
                                        max_workspace_bytes=ws_max)
            q2 = ops.alpha_qe(desc, gallery, i1, s1, n=2, alpha=3.0, idx_offset=lo)
            q_lp, q_sc = ops.quantize_rows(q2, a.dtype)
            return ops.cosine_topk_lp(q_lp, q_sc, gal_lp, gal_sc, a.k, a.dtype, idx_offset=lo, workspace=ws,
                                      max_workspace_bytes=ws_max)
        if sharded is not None:
            return sharded.search(desc, a.k, counts)
        if gal_lp is not None:
            q_lp, q_sc = ops.quantize_rows(desc, a.dtype)
            return ops.cosine_topk_lp(q_lp, q_sc, gal_lp, gal_sc, a.k, a.dtype, idx_offset=lo, workspace=ws,
                                      max_workspace_bytes=ws_max)
        if gal_bf is not None:
            return ops.cosine_topk_prefilter(desc, gallery, gal_bf, gal_bound, a.k, idx_offset=lo, workspace=ws,
                                             max_workspace_bytes=ws_max)
        return ops.cosine_topk(desc, gallery, a.k, idx_offset=lo, workspace=ws, max_workspace_bytes=ws_max)

    s_rank = torch.cuda.Stream(dev)

    def run_steps(n):
        """n steps.  --pipeline: batch i's ranking runs on its own HIP stream
        (after an event on batch i's descriptors) while batch i+1 is embedded
        on the current stream -- the ranker's MFMA / L2-bound sweep beside the
        trunk's HBM-bound layers; still exactly n embeds and n rankings, the
        last ranking joined before returning."""
        if not sched["pipeline"]:
            out = None
            for _ in range(n):
                out = step()
            return out
        prev, ev_prev, out = None, None, None
        for i in range(n + 1):
            if i < n:
                d = embed()
                ev = torch.cuda.Event()
                ev.record()
            if prev is not None:
                with torch.cuda.stream(s_rank):
                    s_rank.wait_event(ev_prev)
                    prev.record_stream(s_rank)  # not reused by the embed stream's allocations meanwhile
                    out = rank_step(prev)
            if i < n:
                prev, ev_prev = d, ev
        torch.cuda.current_stream(dev).wait_stream(s_rank)
        return out

    out = run_steps(a.warmup) if a.warmup > 0 else None
    torch.cuda.synchronize()
    prefilter_stats = None
    if gal_bf is not None:  # the prefilter must reproduce the exhaustive fp32 ranking bit for bit
        d0 = embed()
        s_p, i_p = ops.cosine_topk_prefilter(d0, gallery, gal_bf, gal_bound, a.k, idx_offset=lo, workspace=ws,
                                             max_workspace_bytes=ws_max)
        s_p, i_p = s_p.clone(), i_p.clone()
        s_x, i_x = ops.cosine_topk(d0, gallery, a.k, idx_offset=lo, workspace=ws, max_workspace_bytes=ws_max)
        assert torch.equal(i_p, i_x) and torch.equal(s_p.view(torch.int32), s_x.view(torch.int32)), \
            "prefilter ranking differs from the exhaustive fp32 ranking"
        log("[rank 0] prefilter == exhaustive fp32 ranking on this batch (bit-exact)")
        # (the timed loop's bounded workspace: the survivor counts are read from it)
        ops.cosine_topk_prefilter(d0, gallery, gal_bf, gal_bound, a.k, idx_offset=lo, workspace=ws,
                                  max_workspace_bytes=ws_max)
        surv = ops.prefilter_survivors(ws, q_total, hi - lo, a.dim, a.k).float()
        prefilter_stats = {"bf16_filter_survivors_per_query": {"mean": round(surv.mean().item(), 1),
                                                               "min": int(surv.min().item()),
                                                               "max": int(surv.max().item())}}
    # sanity: a gallery row used as a query must come back first
    chk_s, chk_i = ops.cosine_topk(gallery[:2].contiguous(), gallery, 1, idx_offset=lo, workspace=ws)
    assert chk_i[:, 0].tolist() == [lo, lo + 1], chk_i
    if sharded is not None:  # the full sharded path: all-gather -> shard top-k -> all-to-all -> merge
        ss, si = sharded.search(gallery[:2].contiguous(), a.k, [2] * world)
        assert si[:, 0].tolist() == [lo, lo + 1], si[:, :3]

    timer = ops.KernelTimer(dev.index)
    timer.enable(True)
    if DIST_ON:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = run_steps(a.steps)
    if DIST_ON:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    cls = {name: timer.collect(c) for name, c in (("cosine_filter", _lib.TIME_COSINE), ("conv_gemm", _lib.TIME_GEMM),
                                                   ("select", _lib.TIME_SELECT), ("elementwise", _lib.TIME_ELEM),
                                                   ("cosine_seed", _lib.TIME_COSINE_SEED),
                                                   ("attention", _lib.TIME_ATTN))}
    timer.enable(False)
    if DIST_ON:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = world * a.batch * a.steps / elapsed

    exhaustive = None
    if gal_bf is not None:  # the same step with the exhaustive fp32 ranker, for comparison
        timer.enable(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            ops.cosine_topk(embed(), gallery, a.k, idx_offset=lo, workspace=ws, max_workspace_bytes=ws_max)
        torch.cuda.synchronize()
        el_x = time.perf_counter() - t0
        f_ms, f_n = timer.collect(_lib.TIME_COSINE)
        timer.collect(_lib.TIME_GEMM), timer.collect(_lib.TIME_SELECT), timer.collect(_lib.TIME_ELEM)
        timer.collect(_lib.TIME_COSINE_SEED)
        timer.enable(False)
        s_rows_x = seed_rows(hi - lo, a.k)
        fl = 2.0 * q_total * max(0, (hi - lo) - s_rows_x) * a.dim
        ach = fl / (f_ms / 1e3 / max(1, f_n)) / 1e12 if f_n else 0.0
        exhaustive = {"value": round(a.batch * a.steps / el_x, 2), "ms_per_step": round(el_x / a.steps * 1e3, 3),
                      "cosine_filter": {"bound": "mfma", "dtype": "fp32", "achieved": round(ach, 2),
                                        "peak": PEAK_TFLOPS["fp32"], "unit": "TFLOP/s",
                                        "frac": round(ach / PEAK_TFLOPS["fp32"], 4),
                                        "ms_per_step": round(f_ms / a.steps, 3)},
                      "bit_identical_to_prefilter": True}

    alt_sched, alt_cls = None, None
    if c3 and not DIST_ON and not a.no_extras:
        # the other schedule: one stream if the timed loop overlapped, else the
        # overlapped one; same steps, after one untimed step
        main_sched = dict(sched)
        one = (sched["streams"], sched["pipeline"]) != (1, False)
        sched.update(streams=1, pipeline=False) if one else sched.update(streams=2, pipeline=True)
        run_steps(1)
        timer.enable(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run_steps(a.steps)
        torch.cuda.synchronize()
        el_o = time.perf_counter() - t0
        alt_cls = {name: timer.collect(c) for name, c in (("cosine_filter", _lib.TIME_COSINE),
                                                          ("conv_gemm", _lib.TIME_GEMM), ("select", _lib.TIME_SELECT),
                                                          ("elementwise", _lib.TIME_ELEM),
                                                          ("cosine_seed", _lib.TIME_COSINE_SEED),
                                                          ("attention", _lib.TIME_ATTN))}
        timer.enable(False)
        alt_sched = {"embed_streams": sched["streams"], "pipeline": sched["pipeline"],
                     "value": round(a.batch * a.steps / el_o, 2), "ms_per_step": round(el_o / a.steps * 1e3, 3),
                     "detail": ("the same steps on one HIP stream, each kernel alone on the chip: its rooflines "
                                "are single-kernel durations" if one else
                                "the same steps with the trunk's batch in two parts on two HIP streams (part 2 one "
                                "conv behind) and the ranking of batch i on a third stream beside the embed of "
                                "batch i+1")
                               + "; descriptors bit-identical between the schedules (tests/test_gpu_overlap.py)"}
        sched.update(main_sched)

    decorrelated = None
    if gal_bf is not None and not a.no_extras:
        # The seeded random-weight trunk maps every image to nearly the same
        # descriptor (pairwise cosine ~1.0), so the timed queries are one
        # direction repeated.  The same ranker on q_total independent Gaussian
        # unit queries reports the sweep under decorrelated traffic (its own
        # survivors, its own bit-exactness check); not part of `value`.
        gq = torch.Generator().manual_seed(4321)
        qd = ops.l2_normalize(torch.randn(q_total, a.dim, generator=gq).to(dev))
        s_p, i_p = ops.cosine_topk_prefilter(qd, gallery, gal_bf, gal_bound, a.k, idx_offset=lo, workspace=ws,
                                             max_workspace_bytes=ws_max)
        s_p, i_p = s_p.clone(), i_p.clone()
        surv_d = ops.prefilter_survivors(ws, q_total, hi - lo, a.dim, a.k).float()
        s_x, i_x = ops.cosine_topk(qd, gallery, a.k, idx_offset=lo, workspace=ws, max_workspace_bytes=ws_max)
        assert torch.equal(i_p, i_x) and torch.equal(s_p.view(torch.int32), s_x.view(torch.int32)), \
            "prefilter ranking differs from the exhaustive fp32 ranking (decorrelated queries)"
        timer.enable(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            ops.cosine_topk_prefilter(qd, gallery, gal_bf, gal_bound, a.k, idx_offset=lo, workspace=ws,
                                      max_workspace_bytes=ws_max)
        torch.cuda.synchronize()
        el_d = time.perf_counter() - t0
        f_ms, f_n = timer.collect(_lib.TIME_COSINE)
        sel_ms, _ = timer.collect(_lib.TIME_SELECT)
        timer.collect(_lib.TIME_GEMM), timer.collect(_lib.TIME_ELEM), timer.collect(_lib.TIME_COSINE_SEED)
        timer.enable(False)
        fl = 2.0 * q_total * (hi - lo) * a.dim
        ach = fl / (f_ms / 1e3 / max(1, f_n)) / 1e12 if f_n else 0.0
        decorrelated = {"queries": f"{q_total} seeded Gaussian unit vectors", "bit_identical_to_exhaustive": True,
                        "ranker_ms_per_search": round(el_d / a.steps * 1e3, 3),
                        "cosine_filter": {"bound": "mfma", "dtype": "bf16", "achieved": round(ach, 2),
                                          "peak": PEAK_TFLOPS["bf16"], "unit": "TFLOP/s",
                                          "frac": round(ach / PEAK_TFLOPS["bf16"], 4),
                                          "ms_per_search": round(f_ms / a.steps, 3)},
                        "select_and_rescore_ms_per_search": round(sel_ms / a.steps, 3),
                        "bf16_filter_survivors_per_query": {"mean": round(surv_d.mean().item(), 1),
                                                            "min": int(surv_d.min().item()),
                                                            "max": int(surv_d.max().item())}}

    # ---- roofline (algorithmic FLOPs / measured kernel time) ----
    s_rows = seed_rows(hi - lo, a.k)
    flop_filter = 2.0 * q_total * max(0, (hi - lo) - s_rows) * a.dim  # per filter launch (one per step)
    flop_seed = 2.0 * q_total * s_rows * a.dim
    attn_flops_img = 0
    if a.workload == "c4":
        conv_flops_img, attn_flops_img = W.vit_flops(out_dim=a.dim)
    elif a.workload == "c5":
        conv_flops_img = sum(sum(W.resnet_conv_flops(a.arch, int(224.0 * sc), int(224.0 * sc)).values())
                             + 2 * 2 * 2048 * 2048 for sc in scales)
        flop_filter *= 2  # two searches (before and after alpha-QE)
        flop_seed *= 2
    else:
        conv_flops_img = sum(W.resnet_conv_flops(a.arch, 224, 224).values()) + 2 * 2 * 2048 * 2048  # + whiten, PCA-w
    conv_bytes_step, conv_floor_ms, floor_parts = None, None, None
    if a.workload in ("c3", "c5"):
        # per-layer algorithmic bytes (weights.resnet_conv_bytes) and the layer-wise
        # roofline floor sum_l max(FLOP_l / peak, bytes_l / HBM peak) of the conv class
        pk = PEAK_TFLOPS[a.conv_math if a.conv_math in SPLIT_MATH else "fp32"] * 1e12
        conv_bytes_step, floor = 0.0, 0.0
        floor_parts = {"mfma": 0.0, "hbm": 0.0}  # the floor's time in MFMA-bound / HBM-bound layers
        for sc in (scales if a.workload == "c5" else (1.0,)):
            hh = int(224.0 * sc)
            fl_l = W.resnet_conv_flops(a.arch, hh, hh)
            by_l = W.resnet_conv_bytes(a.arch, hh, hh, a.batch, weight_bytes=WEIGHT_BYTES[a.conv_math],
                                       fused=a.conv_math == "h2")
            for name in fl_l:
                conv_bytes_step += by_l[name]
                t_f, t_b = fl_l[name] * a.batch / pk, by_l[name] / (PEAK_HBM_GBS * 1e9)
                floor += max(t_f, t_b)
                floor_parts["mfma" if t_f >= t_b else "hbm"] += max(t_f, t_b)
            lin_by = 2 * (2 * a.batch * 2048 * 4 + 2048 * 2048 * 4)  # whiten + PCA-w (exact-fp32 core)
            conv_bytes_step += lin_by
            floor += max(2 * 2 * 2048 * 2048 * a.batch / (PEAK_TFLOPS["fp32"] * 1e12), lin_by / (PEAK_HBM_GBS * 1e9))
        conv_floor_ms = floor * 1e3
    traffic = load_traffic()
    rank_dt = "bf16" if pre else a.dtype  # the dtype the gallery sweep runs in
    esz = {"fp32": 4, "bf16": 2, "fp8": 1}[rank_dt]
    rows_filter = max(0, (hi - lo) - s_rows)
    if pre:  # the prefilter sweeps every row (the seed rows again) in bf16
        rows_filter = hi - lo
        flop_filter = 2.0 * q_total * rows_filter * a.dim
    # (class, algorithmic FLOPs, algorithmic HBM bytes or None, dtype of its MFMA)
    searches = 2 if a.workload == "c5" else 1
    conv_dt = a.dtype if a.workload == "c4" else (a.conv_math if a.conv_math in SPLIT_MATH else "fp32")
    # attention (C4): bf16 MFMA when the ViT runs in bf16; per layer it reads
    # the QKV rows once and writes the head outputs
    attn_dt = "bf16" if (a.workload == "c4" and a.dtype != "fp32") else "fp32"
    # (the bf16 ViT's QKV linear writes bf16 rows, networks.VisionTransformer._forward_bf16)
    attn_bytes = (12.0 * a.batch * 197 * 768 * (3 + 1) * (2 if attn_dt == "bf16" else 4)
                  if a.workload == "c4" else None)
    entries = (("cosine_filter", flop_filter, searches * float(rows_filter) * a.dim * esz, rank_dt),
               ("conv_gemm", conv_flops_img * a.batch, conv_bytes_step, conv_dt),
               ("cosine_seed", flop_seed, searches * float(s_rows) * a.dim * esz, rank_dt),
               ("attention", attn_flops_img * a.batch, attn_bytes, attn_dt))
    def roofline_entries(cls):
        rk = {}
        for name, fl_step, by_step, dt in entries:
            ms, n = cls[name]
            if n == 0 or ms <= 0:
                continue
            sec = ms / 1e3 / a.steps
            peak = PEAK_TFLOPS[dt]
            t_mfma = fl_step / (peak * 1e12)
            t_hbm = by_step / (PEAK_HBM_GBS * 1e9) if by_step else 0.0
            if name == "conv_gemm" and floor_parts is not None:
                # a class of layers with their own bounds: the bound of the layers that
                # hold most of its roofline floor (not of the class's summed bytes vs FLOPs)
                hbm_bound = floor_parts["hbm"] > floor_parts["mfma"]
            else:
                hbm_bound = t_hbm > t_mfma
            if hbm_bound:
                ach = by_step / sec / 1e9
                e = {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(ach / PEAK_HBM_GBS, 4)}
            else:
                ach = fl_step / sec / 1e12
                e = {"bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(ach / peak, 4)}
            if dt in SPLIT_MATH:
                e["math"] = SPLIT_MATH[dt][1] + (" (every conv incl. the stem; the whiten and PCA-w linears, 0.2% of "
                                                 "the FLOPs, run on the exact-fp32 core)")
                e["mfma_flop_per_launch"] = SPLIT_MATH[dt][0] * fl_step / max(1.0, n / a.steps)
                # the class's fp32-equivalent rate (algorithmic FLOPs / time) whichever
                # bound is reported, against both split cores' ceilings
                e["fp32_equiv_tflops"] = round(fl_step / sec / 1e12, 2)
                e["frac_of_split_ceiling"] = round(fl_step / sec / 1e12 / PEAK_TFLOPS[dt], 4)
                if dt == "h2":  # the previous core's ceiling, for comparison across rounds
                    e["frac_of_bf16x3_ceiling"] = round(fl_step / sec / 1e12 / PEAK_TFLOPS["s3"], 4)
            e.update({"dtype": "fp32" if dt in SPLIT_MATH else dt, "ms_per_step": round(ms / a.steps, 3),
                      "launches_per_step": n / a.steps,
                      "algorithmic_flop_per_launch": fl_step / max(1.0, n / a.steps),
                      "algorithmic_bytes_per_launch": (by_step / max(1.0, n / a.steps)) if by_step else None,
                      "traffic": ((traffic or {}).get(name) or {}).get("hbm_bytes_per_launch")
                      if (traffic and traffic.get("workload") == a.workload and a.gallery == 1_600_000
                          and a.batch == traffic.get("batch", 320) and pre
                          and a.conv_math == traffic.get("conv_math", "s3")) else None})
            if name == "conv_gemm" and conv_floor_ms is not None:
                e["layer_roofline_floor_ms_per_step"] = round(conv_floor_ms, 3)
                e["frac_of_layer_floor"] = round(conv_floor_ms / (ms / a.steps), 4)
                e["layer_floor_split_ms"] = {k: round(v * 1e3, 3) for k, v in floor_parts.items()}
            rk[name] = e
        for name in ("select", "elementwise"):
            ms, n = cls[name]
            rk[name] = {"ms_per_step": round(ms / a.steps, 3), "launches_per_step": n / a.steps}
        return rk

    rk = roofline_entries(cls)
    if alt_sched is not None:
        rk_alt = roofline_entries(alt_cls)
        alt_sched["roofline_by_kernel"] = {k: rk_alt[k] for k in ("conv_gemm", "cosine_filter", "select",
                                                                   "elementwise") if k in rk_alt}
    dominant = max(("cosine_filter", "conv_gemm"), key=lambda c: cls[c][0])
    roof = dict(rk[dominant])
    roof["kernel"] = dominant

    res = {"metric": METRIC, "value": round(value, 2), "unit": "images/s", "n_gpus": world, "steps": a.steps,
           "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": a.dtype,
           "data": "synthetic: uint8 224x224x3 images RandomState(1234+rank); seeded "
                   + ("Gaussian" if a.gallery_kind == "gaussian" else "clustered (81,313 classes)")
                   + " L2-normalised gallery; seeded ResNet/whiten/PCA-w weights (no pretrained weights offline)",
           "config": {"workload": {"c3": f"C3: {a.arch}-GeM 2048-d + PCA-whiten",
                                   "c4": f"C4: ViT-B/16 CLS {a.dim}-d ({a.dtype} GEMMs + {a.dtype} cosine)",
                                   "c5": f"C5: {a.arch}-GeM+PCA-w at 3 scales, {a.dtype} cosine + alpha-QE "
                                         f"(n=2, alpha=3) re-rank"}[a.workload] +
                                  f", embed + {'exact' if a.dtype == 'fp32' else a.dtype} top-{a.k} against a {a.gallery}x{a.dim} gallery"
                                  + (" (ranker: bf16-bound prefilter + exact fp32 rescoring, bit-identical to the "
                                     "exhaustive fp32 ranker)" if pre else ""),
                      "global_batch": q_total,
                      "images_per_gpu_per_step": a.batch, "gallery_rows": a.gallery, "dim": a.dim, "k": a.k,
                      "parallelism": f"query-dp{world} + gallery-shard{world}",
                      "conv_math": a.conv_math if a.workload != "c4" else None,
                      "pipeline": sched["pipeline"],
                      "embed_streams": sched["streams"],
                      **({"tuning": a.tune} if a.tune else {}),
                      "ranker_workspace_bytes_per_rank": int(ws.numel()),
                      "ranker_workspace_worst_case_bytes": int(ws_full)},
           "roofline": roof, "roofline_by_kernel": rk}
    if exhaustive is not None:
        res["ranker"] = {"kind": "prefilter", "detail": "bf16-bound prefilter + exact fp32 rescoring; results "
                         "asserted bit-identical to the exhaustive fp32 ranker on a measured batch",
                         "gallery_kind": a.gallery_kind, "exhaustive_fp32": exhaustive,
                         "sweep_ms_per_step": rk.get("cosine_filter", {}).get("ms_per_step"),
                         "select_and_rescore_ms_per_step": rk.get("select", {}).get("ms_per_step"),
                         **(prefilter_stats or {}),
                         **({"decorrelated_queries": decorrelated} if decorrelated else {})}
    if alt_sched is not None:
        res["one_stream_schedule" if alt_sched["embed_streams"] == 1 else "overlapped_schedule"] = alt_sched
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.workload == "c3":
        t = time.time()
        res["cpu_baseline"] = cpu_baseline(a.arch, a.gallery, a.dim, a.k)
        log(f"cpu baseline {time.time() - t:.1f}s")
    if rank == 0:
        print(json.dumps(res, default=_json_scalar), flush=True)
    if DIST_ON:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
