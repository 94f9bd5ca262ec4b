#!/bin/bash
# r04g: the f16x2 256x256 conv tile with its loads spread among the MFMAs
# (conv_il) per R101 layer at 1280 images; the sweep defaults' tests
set -o pipefail
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 400 python -u tools/h2_cfg_sweep.py 1280 0,0i > $O/h2_cfg_il.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_rank.py tests/test_gpu_ops.py -m gpu -x -v -s --timeout 240 --timeout-method thread > $O/tests.log 2>&1
tail -22 $O/h2_cfg_il.txt; tail -2 $O/tests.log
echo call-done
