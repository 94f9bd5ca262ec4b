#!/bin/bash
# Quick GPU check: selected test files (default: the whole -m gpu suite), then smoke.
# usage: bash tools/rc_quick.sh <tag> [pytest paths...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-quick}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
T=${@:-tests}
timeout -k 10 900 python -u -m pytest $T -m gpu -x -v -s --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo all-done
