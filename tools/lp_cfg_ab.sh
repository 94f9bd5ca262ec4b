#!/bin/bash
# Forced bf16-core configs on the ViT-B/16 linears at 1280 images, interleaved:
#   CFGS="auto 6" bash tools/lp_cfg_ab.sh <tag>
set -o pipefail
TAG=${1:-lpcfg}
mkdir -p gpurun_out/$TAG
for r in 1 2; do
  for c in ${CFGS:-auto 6}; do
    LP_B=1280 LP_SWEEPS=0 LP_CFG=$c timeout -k 10 200 python -u tools/lp_bench.py > gpurun_out/$TAG/cfg${c}_$r.txt 2>&1 || exit 1
  done
done
grep -h linear gpurun_out/$TAG/*.txt
