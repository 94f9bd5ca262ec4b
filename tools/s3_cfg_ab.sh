#!/bin/bash
# Forced split-bf16 tile configs per R101 layer + stem at 1280 images, interleaved:
#   CFGS="0 7" ROWS="<grep pattern>" bash tools/s3_cfg_ab.sh
set -o pipefail
mkdir -p gpurun_out/s3cfg
for r in 1 2; do
  for c in ${CFGS:-0 7}; do
    S3_ONLY=1 S3_CFG=$c timeout -k 10 200 python -u tools/s3_bench.py 1280 8 > gpurun_out/s3cfg/cfg${c}_$r.txt 2>&1 || exit 1
    S3_CFG=$c timeout -k 10 100 python -u tools/stem_ab.py 1280 >> gpurun_out/s3cfg/cfg${c}_$r.txt 2>&1 || exit 1
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_tile_configs.py -k "s3" > gpurun_out/s3cfg/tests.log 2>&1; tail -1 gpurun_out/s3cfg/tests.log
grep -h -E -e "${ROWS:-64->   64|256->   64|stem s3}" gpurun_out/s3cfg/cfg*_[12].txt
