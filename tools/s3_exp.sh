#!/bin/bash
# Epilogue vs main-loop cost of the K=256 expansion layers (s3 core).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3exp
mkdir -p $O
cd $R
for cfg in 3 1 6; do
for shape in "320 14 14 256 1024 1 1 0 0" "320 14 14 256 1024 1 1 0 1" "320 14 14 512 1024 1 1 0 0" "320 14 14 512 1024 1 1 0 1" "320 14 14 128 1024 1 1 0 1" "320 14 14 1024 1024 1 1 0 1"; do
  echo "cfg $cfg $shape $(RR_S3_CFG=$cfg timeout -k 10 60 python tools/s3_one.py $shape 1 20 2>/dev/null | tail -1)" >> $O/exp.log || exit 1
done
done
echo done
