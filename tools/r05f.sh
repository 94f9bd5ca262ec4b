#!/bin/bash
# round 5: the centered LayerNorm fold, seam and config-15 tests, then config
# 15 (persistent 256x256) per layer and on the bench's embed
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -s"
timeout -k 10 700 $T \
  "tests/test_gpu_h2.py::test_h2_persistent_256_tile_bit_identical" "tests/test_gpu_h2.py::test_h2_persistent_tile_bit_identical" \
  > gpurun_out/r05f_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r05f_tests.log; exit 1; }
tail -3 gpurun_out/r05f_tests.log
timeout -k 10 300 python -u tools/h2_cfg_sweep.py 1280 0,15 > gpurun_out/r05f_cfg15_sweep.txt 2>&1 || exit 1
cat gpurun_out/r05f_cfg15_sweep.txt
E2E_EMBED="s3_cfg=0 s3_cfg=15 s3_cfg_res=15" timeout -k 10 300 python -u tools/e2e_ab.py 1280 4 > gpurun_out/r05f_cfg15_e2e.txt 2>&1 || exit 1
cat gpurun_out/r05f_cfg15_e2e.txt
