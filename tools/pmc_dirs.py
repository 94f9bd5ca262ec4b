"""Summarise a rocprofv3 run tree: kernel_stats (average duration) and every
counter_collection.csv under <dir> for kernels whose name contains SUBSTR
(averaged over dispatches), with FETCH_SIZE doubled per the gfx950
correction (MI355X_MICROARCH.md, HBM) and the MFMA-busy / wait fractions.
usage: python tools/pmc_dirs.py <dir> [SUBSTR]"""
import collections
import csv
import glob
import sys

root, sub = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "seam")
for f in glob.glob(root + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sub in r["Name"]:
            print(f"{r['Name'][:80]}: {r['Calls']} calls, avg {float(r['AverageNs']) / 1e3:.1f} us")
acc = collections.defaultdict(list)
for f in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
c = {k: sum(v) / len(v) for k, v in acc.items()}
for k in sorted(c):
    print(f"  {k:28s} {c[k]:.4g}")
if "FETCH_SIZE" in c:
    print(f"  read bytes (2 x FETCH_SIZE KiB) = {2 * c['FETCH_SIZE'] * 1024 / 1e9:.3f} GB")
if "WRITE_SIZE" in c:
    print(f"  write bytes = {c['WRITE_SIZE'] * 1024 / 1e9:.3f} GB")
if "GRBM_GUI_ACTIVE" in c and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
    print(f"  mfma busy = {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (c['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
    if k in c and "SQ_WAVE_CYCLES" in c:
        print(f"  {k} / wave cycles = {c[k] / c['SQ_WAVE_CYCLES']:.3f}")
