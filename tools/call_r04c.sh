#!/bin/bash
# r04c: fetch-ceiling with the 16x16x32 sweep variant; the production sweep on
# 16x16x32 (sweep_mf16) and lp_cfg A/B of the C3 prefilter sweep; the halo
# 3x3 on 16x16x32 (s3_cfg 14) vs 13; their tests
set -o pipefail
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 120 ./tools/fetch_ceiling 5 > $O/fetch_ceiling.txt 2>&1 || exit 1
PF_KEY=sweep_mf16 PF_CFGS="0 1" timeout -k 10 300 python -u tools/prefilter_ab.py > $O/mf16_ab.txt 2>&1 || exit 1
PF_QKIND=corr PF_KEY=sweep_mf16 PF_CFGS="0 1" timeout -k 10 300 python -u tools/prefilter_ab.py > $O/mf16_ab_corr.txt 2>&1 || exit 1
PF_QKIND=corr PF_CFGS="0 3 5" timeout -k 10 300 python -u tools/prefilter_ab.py > $O/lpcfg_ab_corr.txt 2>&1 || exit 1
timeout -k 10 400 python -u tools/h2_cfg_sweep.py 1280 0,13,14 > $O/h2_cfg_halo_mf16.txt 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_rank.py tests/test_gpu_trunk.py tests/test_gpu_h2.py tests/test_gpu_ops.py -m gpu -x -v -s --timeout 240 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
echo call-done
