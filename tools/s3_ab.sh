#!/bin/bash
# GPU A/B of split-bf16 kernel variants: tests + per-layer timing under each
# env setting given as an argument (e.g. "RR_S3_PIPE=1").
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3ab
mkdir -p $O
cd $R
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python -u -m pytest tests/test_gpu_s3.py -x -q -s --timeout 120 --timeout-method thread > $O/tests_$i.log 2>&1 || { echo "tests failed for $e"; exit 1; }
  env $e timeout -k 10 200 python -u tools/s3_bench.py 320 10 > $O/bench_$i.log 2>&1 || exit 1
  echo "$i: $e $(tail -1 $O/bench_$i.log)"
done
