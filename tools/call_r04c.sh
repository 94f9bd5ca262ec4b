#!/bin/bash
# r04c: fetch-ceiling with the 16x16x32 sweep variant; lp_cfg A/B of the C3 prefilter sweep
set -o pipefail
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 120 ./tools/fetch_ceiling 5 > $O/fetch_ceiling.txt 2>&1 || exit 1
PF_CFGS="0 3 5" timeout -k 10 300 python -u tools/prefilter_ab.py > $O/lpcfg_ab.txt 2>&1 || exit 1
PF_QKIND=corr PF_CFGS="0 3 5" timeout -k 10 300 python -u tools/prefilter_ab.py > $O/lpcfg_ab_corr.txt 2>&1 || exit 1
echo call-done
