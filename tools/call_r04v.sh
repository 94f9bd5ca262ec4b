#!/bin/bash
set -o pipefail
O=gpurun_out/r04v; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_vit.py -m gpu -x -v -s --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" $O/tests.log | tail -8; tail -1 $O/tests.log
echo call-done rc=$rc
