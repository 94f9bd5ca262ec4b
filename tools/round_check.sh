#!/bin/bash
# One GPU call: parity tests, smoke, default bench (with CPU baseline), C4/C5
# bench lines, rocprofv3 evidence (kernel trace + stats, then one PMC pass per
# counter group).  Every GPU step has its own time limit; steps chained by &&.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/rc
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err && \
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err && \
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err && \
timeout -k 10 900 bash tools/profile.sh > $O/profile.log 2>&1 && \
echo all-done
