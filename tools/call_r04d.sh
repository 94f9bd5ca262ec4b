#!/bin/bash
# r04d: the whole -m gpu suite + smoke, then the default C3 bench line
set -o pipefail
O=gpurun_out/r04d; mkdir -p $O
bash tools/rc_quick.sh r04d && \
timeout -k 10 400 python -u bench.py > $O/c3.json 2> $O/c3.log && tail -3 $O/gpu_tests.log && cat $O/c3.json && echo call-done
