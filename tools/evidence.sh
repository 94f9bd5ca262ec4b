#!/bin/bash
# Round-end evidence on one MI355X (gpurun): rocprofv3 kernel trace + PMC passes
# of the default C3 bench (tools/profile.sh), then the bench lines of the other
# workloads.  usage: bash tools/evidence.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ev}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 420 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.log || { echo "bench c3 failed"; exit 1; }
echo "c3 done"
bash tools/profile.sh > $O/profile.log 2>&1 || { echo "profile failed"; exit 1; }
for w in "c4" "c5" "c3 --gallery-kind clustered" "c2"; do
  n=$(echo $w | tr ' ' '_' | tr -d '-')
  timeout -k 10 420 python -u bench.py --workload $w > $O/bench_$n.json 2> $O/bench_$n.log || { echo "bench $w failed"; exit 1; }
  echo "$w done"
done
echo evidence-done
