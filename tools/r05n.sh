#!/bin/bash
# the persistent bf16 tile (lp_cfg 6): bit-identity, then the C4 embed A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_gpu_vit.py::test_linear_bf16_persistent_tile_bit_identical" > gpurun_out/r05q_tests.log 2>&1 || { tail -30 gpurun_out/r05q_tests.log; exit 1; }
tail -2 gpurun_out/r05q_tests.log
E2E_WORKLOAD=c4 E2E_EMBED="lp_cfg=0 lp_cfg=6" timeout -k 10 400 python -u tools/e2e_ab.py 1280 4 > gpurun_out/r05q_e2e_c4.txt 2>&1 || { tail -5 gpurun_out/r05q_e2e_c4.txt; exit 1; }
cat gpurun_out/r05q_e2e_c4.txt
