#!/bin/bash
# usage: bash tools/gpu_check.sh <tag> [pytest paths...]: the given GPU tests, then the C3 bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-chk}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -v -s --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
echo tests-ok
timeout -k 10 400 python -u bench.py > $O/c3.json 2> $O/c3.log || { echo "bench failed"; tail -20 $O/c3.log; exit 1; }
cat $O/c3.json | head -c 600; echo
echo all-done
