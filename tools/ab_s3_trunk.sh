#!/bin/bash
# A/B of librr builds on the R101 trunk layers (tools/s3_bench.py, 1280 images),
# interleaved on one device: bash tools/ab_s3_trunk.sh <tag> <lib>... (paths
# relative to the repo; "main" = the in-tree librr.so)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for r in 1 2; do
  for L in "$@"; do
    n=$(basename $L .so)
    if [ "$L" = main ]; then
      S3_ONLY=1 timeout -k 10 200 python -u tools/s3_bench.py 1280 8 > gpurun_out/$TAG/${n}_$r.txt 2>&1 || exit 1
      timeout -k 10 100 python -u tools/stem_ab.py 1280 >> gpurun_out/$TAG/${n}_$r.txt 2>&1 || exit 1
    else
      S3_ONLY=1 RR_LIB_PATH=$L timeout -k 10 200 python -u tools/s3_bench.py 1280 8 > gpurun_out/$TAG/${n}_$r.txt 2>&1 || exit 1
      RR_LIB_PATH=$L timeout -k 10 100 python -u tools/stem_ab.py 1280 >> gpurun_out/$TAG/${n}_$r.txt 2>&1 || exit 1
    fi
  done
done
grep -E "TOTAL|s3" gpurun_out/$TAG/*.txt | grep -v "^.*:h "
