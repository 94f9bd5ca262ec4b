#!/bin/bash
# r04t: HBM bytes of the C3 filter sweep per launch under the default block
# order and the 2-panel-group XCD order (FETCH_SIZE / WRITE_SIZE passes)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r04t; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for ord in 0 2; do
  PF_KEY=sweep_order PF_CFGS="$ord" timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$ord -o run -- python3 $R/tools/prefilter_ab.py > $O/fetch_$ord.log 2>&1 || exit 1
  PF_KEY=sweep_order PF_CFGS="$ord" timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$ord -o run -- python3 $R/tools/prefilter_ab.py > $O/write_$ord.log 2>&1 || exit 1
done
cd $R
python - <<'PY'
import csv, glob
for ord in (0, 2):
    for kind, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        f = glob.glob(f"gpurun_out/r04t/{kind}_{ord}/**/run_counter_collection.csv", recursive=True) or glob.glob(f"gpurun_out/r04t/{kind}_{ord}/run_counter_collection.csv")
        rows = [r for r in csv.DictReader(open(f[0])) if "gemm_kernel<4, 2, 2, 5, 0, 2," in r.get("Kernel_Name", "")]
        per = {}
        for r in rows:
            per.setdefault(r["Dispatch_Id"], 0.0)
            per[r["Dispatch_Id"]] += float(r["Counter_Value"])
        v = sorted(per.values())
        mult = 2 * 1024 if kind == "fetch" else 1024
        print(ord, kind, len(v), "median GB per launch", round(v[len(v) // 2] * mult / 1e9, 3) if v else None)
PY
echo call-done
