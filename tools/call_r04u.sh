#!/bin/bash
# r04u: the final tree's whole -m gpu suite + smoke
set -o pipefail
bash tools/rc_quick.sh r04u || { grep -E "FAILED|Error" gpurun_out/r04u/gpu_tests.log | head; exit 1; }
tail -1 gpurun_out/r04u/gpu_tests.log
echo call-done
