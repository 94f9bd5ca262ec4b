#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  "tests/test_gpu_vit.py::test_linear_bf16_persistent_tile_bit_identical" > gpurun_out/r05u_tests.log 2>&1 || { tail -30 gpurun_out/r05u_tests.log; exit 1; }
tail -1 gpurun_out/r05u_tests.log
timeout -k 10 300 python -u tools/vit_lin_ab.py 1280 3,0,6 > gpurun_out/r05u_vitlin.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r05u_vitlin.txt
