#!/bin/bash
# r04s: conv_il on the dense (no-residual) layers only, on the bench's own embed
set -o pipefail
O=gpurun_out/r04s; mkdir -p $O
timeout -k 10 120 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 100 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
E2E_EMBED="conv_il=0 conv_il=2 conv_il=1" timeout -k 10 600 python -u tools/e2e_ab.py 1280 6 > $O/e2e_conv_il.txt 2>&1
grep -v amdgpu.ids $O/e2e_conv_il.txt; tail -1 $O/tests.log
echo call-done
