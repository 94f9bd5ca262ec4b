#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  "tests/test_gpu_h2.py::test_h2_halo_persistent_bit_identical" > gpurun_out/r05w_tests.log 2>&1 || { tail -30 gpurun_out/r05w_tests.log; exit 1; }
tail -1 gpurun_out/r05w_tests.log
timeout -k 10 300 python -u tools/h2_cfg_sweep.py 1280 0,16 > gpurun_out/r05w_sweep.txt 2>&1 || exit 1
grep -E "k3 s1|weighted" gpurun_out/r05w_sweep.txt
E2E_EMBED="s3_cfg=0 s3_cfg=16" timeout -k 10 300 python -u tools/e2e_ab.py 1280 4 > gpurun_out/r05w_e2e.txt 2>&1 || exit 1
cat gpurun_out/r05w_e2e.txt
