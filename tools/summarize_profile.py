"""Summarise a tools/profile.sh run into profiles/ (committed evidence).

HBM bytes per MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE counts exactly half of a wide (16 B/lane) coalesced
streaming read, so read bytes = 2 * FETCH_SIZE * 1024 (all librr GEMM A/B
loads are 16 B/lane float4).  WRITE_SIZE is exact for 16-B streaming stores;
librr's GEMM epilogue stores 4 B/lane (conv) — uncalibrated, reported as is.
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

def short(name):
    m = re.search(r"(rr::(?:\(anonymous namespace\)::)?\w+(<[^>]*>)?)", name)
    return m.group(1) if m else name[:60]


def cls_of(name):
    """Kernel class as bench.py's timer classes: gemm_kernel<WM, WN, FM, FN,
    AMODE, EMODE, ...> by its epilogue (EMODE 2 = cosine filter sweep, 1 =
    seed scores, 0 = stored C: convs / linears); gemm_s3_kernel and the
    persistent gemm_s3p_kernel / gemm_s3q_kernel, the halo-staged gemm_h2_halo_kernel /
    stem_pool_halo_kernel = convs; sweep128 / sweep16 = cosine filter."""
    if ("gemm_s3_kernel" in name or "gemm_s3p_kernel" in name or "gemm_s3q_kernel" in name
            or "gemm_h2_halo_kernel" in name or "stem_pool_halo_kernel" in name or "seam_h2_kernel" in name):
        return "conv_gemm"
    if "sweep128_kernel" in name or "sweep16_kernel" in name:  # the hand-scheduled bf16 filter sweeps
        return "cosine_filter"
    if "gemm_lpp" in name:  # the persistent bf16 stored-C tiles (ViT linears)
        return "conv_gemm"
    m = re.search(r"gemm_8p_kernel<(\d)>", name)
    if m:  # the 8-phase bf16 sweep (filter / seed scores only)
        return {2: "cosine_filter", 1: "cosine_seed"}.get(int(m.group(1)), "other")
    m = re.search(r"gemm_kernel<([^>]*)>", name)
    if m:
        args = [int(x) for x in m.group(1).split(",")]
        return {2: "cosine_filter", 1: "cosine_seed"}.get(args[5], "conv_gemm")
    if re.search(r"select_|merge_kernel|prefilter_", name):
        return "select"
    if "attention_kernel" in name:
        return "attention"
    if "rr::" in name:
        return "elementwise"
    return "other"


def counters(path, names):
    per = defaultdict(lambda: defaultdict(float))
    n = defaultdict(set)
    if not os.path.exists(path):
        return per, n
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] in names:
            k = short(r["Kernel_Name"])
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[k].add(r["Dispatch_Id"])
    return per, n


def main(src, tag):
    dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    fetch, nf = counters(os.path.join(src, "fetch", "run_counter_collection.csv"), {"FETCH_SIZE"})
    write, nw = counters(os.path.join(src, "write", "run_counter_collection.csv"), {"WRITE_SIZE"})
    mf, nm = counters(os.path.join(src, "mfma", "run_counter_collection.csv"),
                      {"SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_BUSY_CU_CYCLES"})
    rows = []
    for s in stats:
        k = short(s["Name"])
        calls = int(s["Calls"])
        r = {"kernel": k, "class": cls_of(s["Name"]), "calls": calls, "avg_us": float(s["AverageNs"]) / 1e3,
             "total_ms": float(s["TotalDurationNs"]) / 1e6, "pct": float(s["Percentage"])}
        if k in fetch and nf[k]:
            r["read_bytes_per_launch"] = 2 * fetch[k]["FETCH_SIZE"] * 1024 / len(nf[k])
        if k in write and nw[k]:
            r["write_bytes_per_launch"] = write[k]["WRITE_SIZE"] * 1024 / len(nw[k])
        if k in mf and nm[k]:
            busy, act = mf[k]["SQ_VALU_MFMA_BUSY_CYCLES"], mf[k]["GRBM_GUI_ACTIVE"]
            r["mfma_busy_cycles_per_launch"] = busy / len(nm[k])
            # per-SIMD MFMA busy fraction: busy / (GRBM cycles x 256 CUs x 4 SIMDs)
            if act > 0:
                r["mfma_util"] = busy / (act / 8 * 256 * 4)
        rows.append(r)
    with open(os.path.join(dst, f"{tag}_kernel_summary.json"), "w") as f:
        json.dump(rows, f, indent=1)
    traffic = {}
    for c in ("cosine_filter", "cosine_seed", "conv_gemm"):
        rs = [r for r in rows if r["class"] == c and "read_bytes_per_launch" in r]
        if c.startswith("cosine") and rs:
            # one instantiation per step, in the ranker's dtype (DT template
            # arg: 1 = bf16 prefilter sweep, 0 = exhaustive fp32); the bench's
            # side calls (exhaustive comparison, sanity search) are excluded
            dt = os.environ.get("RR_PROFILE_RANK_DT", "1")
            # (the 8-phase kernel is bf16 only: gemm_8p_kernel<EM>)
            rs = [r for r in rs if (r["kernel"].split(",")[7].strip() if r["kernel"].count(",") >= 7 else "1") == dt] or rs
            rs = [max(rs, key=lambda r: r["total_ms"])]
        if rs:
            tot_calls = sum(r["calls"] for r in rs)
            rb = sum(r["read_bytes_per_launch"] * r["calls"] for r in rs) / tot_calls
            wb = sum(r.get("write_bytes_per_launch", 0) * r["calls"] for r in rs) / tot_calls
            traffic[c] = {"kernels": [r["kernel"] for r in rs], "hbm_read_bytes_per_launch": rb, "hbm_write_bytes_per_launch": wb,
                          "hbm_bytes_per_launch": rb + wb, "source": f"profiles/{tag}_kernel_summary.json"}
    traffic["workload"] = os.environ.get("RR_PROFILE_WORKLOAD", "c3")
    traffic["conv_math"] = os.environ.get("RR_PROFILE_CONV_MATH", "h2")  # bench.py's default --conv-math
    traffic["batch"] = int(os.environ.get("RR_PROFILE_BATCH", "1280"))  # bench.py's default --batch
    with open(os.path.join(dst, "traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1)
    # raw rocprofv3 stats, committed verbatim
    import shutil
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    for r in rows[:12]:
        print({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()})
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
