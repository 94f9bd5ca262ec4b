#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3lin
mkdir -p $O
cd $R
for e in "RR_S3_CFG=0"; do
  env $e timeout -k 10 120 python -u tools/s3_lin.py 20 >> $O/lin.log 2>&1 || exit 1
done
echo done
