#!/bin/bash
# r04z1: round-end evidence 1 -- the whole -m gpu suite + smoke, the default
# C3 line, rocprofv3 kernel trace + PMC passes of the default C3 bench
set -o pipefail
O=gpurun_out/r04z; mkdir -p $O
bash tools/rc_quick.sh r04z || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 400 python -u bench.py > $O/c3.json 2> $O/c3.log || exit 1
cat $O/c3.json
rm -rf gpurun_out/prof
bash tools/profile.sh > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
ls gpurun_out/prof
echo call-done
