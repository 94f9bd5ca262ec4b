#!/bin/bash
# r04x: rocprofv3 kernel trace of the C4 bench with the LayerNorm fold
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r04x; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --workload c4 --steps 4 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1
cd $R; ls $O/trace
python - <<'PY'
import csv
rows=list(csv.DictReader(open("gpurun_out/r04x/trace/run_kernel_stats.csv")))
rows.sort(key=lambda r:-float(r["TotalDurationNs"]))
for r in rows[:12]: print(r["Calls"], round(float(r["TotalDurationNs"])/1e6,2), round(float(r["AverageNs"])/1e3,1), r["Name"][:110])
PY
echo call-done
