#!/bin/bash
# First-round stagger sweep of the split-bf16 trunk convs (tools/s3_bench.py at
# 1280 images), interleaved: bash tools/stagger_ab.sh <tag> <values...>
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for r in 1 2; do
  for v in "$@"; do
    S3_ONLY=1 S3_STAGGER=$v timeout -k 10 200 python -u tools/s3_bench.py 1280 8 > gpurun_out/$TAG/st${v}_$r.txt 2>&1 || exit 1
  done
done
grep TOTAL gpurun_out/$TAG/*.txt
