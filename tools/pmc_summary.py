"""Summarise rocprofv3 --pmc counter CSVs (tools/s3_pmc.sh layout): per
directory, the named kernel's counters averaged over its dispatches.
usage: python tools/pmc_summary.py <dir> [kernel-name substring, default gemm_s3]"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "gemm_s3"
for tag in sorted(os.listdir(root)):
    d = os.path.join(root, tag)
    if not os.path.isdir(d):
        continue
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kname not in r.get("Kernel_Name", ""):
                continue
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    c = {k: sum(v) / len(v) for k, v in acc.items()}
    if not c:
        print(tag, "no data")
        continue
    mf = c.get("SQ_INSTS_MFMA", 1)
    print(f"== {tag}")
    for k in sorted(c):
        extra = f"  ({c[k] / mf:.2f} per MFMA)" if k.startswith("SQ_INSTS") else ""
        print(f"  {k:28s} {c[k]:.4g}{extra}")
    if "SQ_WAVE_CYCLES" in c and "SQ_WAIT_INST_ANY" in c:
        print(f"  wait_inst_any / wave_cycles = {c['SQ_WAIT_INST_ANY'] / c['SQ_WAVE_CYCLES']:.3f}")
    if "SQ_WAIT_ANY" in c and "SQ_WAVE_CYCLES" in c:
        print(f"  wait_any / wave_cycles = {c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.3f}")
    if "GRBM_GUI_ACTIVE" in c and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
        print(f"  mfma busy = {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (c['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
