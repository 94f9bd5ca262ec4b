#!/bin/bash
# The bench lines of the non-default workloads (C4, C5, C3 on the clustered
# gallery, C2), one timeout each.  usage: bash tools/evidence_lines.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-lines}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for w in "c4" "c5" "c3 --gallery-kind clustered" "c2"; do
  n=$(echo $w | tr ' ' '_' | tr -d '-')
  timeout -k 10 420 python -u bench.py --workload $w > $O/bench_$n.json 2> $O/bench_$n.log || { echo "bench $w failed"; tail -5 $O/bench_$n.log; exit 1; }
  echo "$w: $(tail -c 300 $O/bench_$n.json | head -c 0)$(python -c "import json;d=json.loads(open('$O/bench_$n.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
done
echo lines-done
