#!/bin/bash
# GPU A/B of RR_S3_VAR variants: s3 tests (unless the variant is an ablation,
# marked with a trailing '!'), then per-layer s3 timing, interleaved rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3var
mkdir -p $O
cd $R
ROUNDS=${ROUNDS:-2}
for v in "$@"; do
  case $v in *!) continue;; esac
  RR_S3_VAR=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_s3.py -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "tests failed for VAR=$v"; tail -20 $O/tests_$v.log; exit 1; }
  echo "tests ok VAR=$v"
done
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    vv=${v%!}
    S3_ONLY=1 RR_S3_VAR=$vv timeout -k 10 200 python -u tools/s3_bench.py 320 10 > $O/bench_${vv}_r$r.log 2>&1 || exit 1
    echo "r$r VAR=$vv $(tail -1 $O/bench_${vv}_r$r.log)"
  done
done
