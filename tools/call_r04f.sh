#!/bin/bash
# r04f: the production sweep with the DMA issue spread among the MFMAs
# (sweep_il) on both MFMA shapes, random and near-parallel queries; its tests
set -o pipefail
O=gpurun_out/r04f; mkdir -p $O
PF_KEY=sweep_il PF_CFGS="0 1" timeout -k 10 300 python -u tools/prefilter_ab.py > $O/il_ab.txt 2>&1 && \
PF_QKIND=corr PF_KEY=sweep_il PF_CFGS="0 1" timeout -k 10 300 python -u tools/prefilter_ab.py > $O/il_ab_corr.txt 2>&1 && \
PF_QKIND=corr PF_EXTRA="sweep_mf16=1" PF_KEY=sweep_il PF_CFGS="0 1" timeout -k 10 300 python -u tools/prefilter_ab.py > $O/il_mf16_ab_corr.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_rank.py tests/test_gpu_ops.py -m gpu -x -v -s --timeout 240 --timeout-method thread -k "sweep or tuning" > $O/tests.log 2>&1
tail -3 $O/*.txt; tail -2 $O/tests.log
echo call-done
