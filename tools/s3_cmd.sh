#!/bin/bash
# GPU: split-bf16 core tests + per-layer timing per tile config (args: configs,
# "auto" = the picker) + the full GPU suite and the default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_s3.py -x -v -s --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for c in "$@"; do
  if [ "$c" = auto ]; then unset RR_S3_CFG; else export RR_S3_CFG=$c; fi
  timeout -k 10 200 python -u tools/s3_bench.py 320 10 > $O/bench_cfg$c.log 2>&1 || exit 1
done
unset RR_S3_CFG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_all.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
echo done
