#!/bin/bash
# config 15 vs 16 (sc1 stores / nt residual loads): bit-identity, per layer, embed
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -s \
  "tests/test_gpu_h2.py::test_h2_persistent_256_tile_bit_identical" > gpurun_out/r05i_tests.log 2>&1 || { tail -30 gpurun_out/r05i_tests.log; exit 1; }
tail -2 gpurun_out/r05i_tests.log
timeout -k 10 300 python -u tools/h2_cfg_sweep.py 1280 0,16 > gpurun_out/r05i_sweep.txt 2>&1 || exit 1
grep -E "1024|2048|weighted" gpurun_out/r05i_sweep.txt
E2E_EMBED="s3_cfg=0 s3_cfg=16" timeout -k 10 300 python -u tools/e2e_ab.py 1280 4 > gpurun_out/r05i_e2e.txt 2>&1 || exit 1
cat gpurun_out/r05i_e2e.txt
