#!/bin/bash
# r04c: fetch-ceiling with the 16x16x32 sweep variant; the production sweep on
# 16x16x32 (sweep_mf16) and lp_cfg A/B of the C3 prefilter sweep; their tests
set -o pipefail
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 120 ./tools/fetch_ceiling 5 > $O/fetch_ceiling.txt 2>&1 || exit 1
PF_KEY=sweep_mf16 PF_CFGS="0 1" timeout -k 10 300 python -u tools/prefilter_ab.py > $O/mf16_ab.txt 2>&1 || exit 1
PF_QKIND=corr PF_KEY=sweep_mf16 PF_CFGS="0 1" timeout -k 10 300 python -u tools/prefilter_ab.py > $O/mf16_ab_corr.txt 2>&1 || exit 1
PF_CFGS="0 3 5" timeout -k 10 300 python -u tools/prefilter_ab.py > $O/lpcfg_ab.txt 2>&1 || exit 1
PF_QKIND=corr PF_CFGS="0 3 5" timeout -k 10 300 python -u tools/prefilter_ab.py > $O/lpcfg_ab_corr.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_rank.py tests/test_gpu_trunk.py -m gpu -x -v -s --timeout 240 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
echo call-done
