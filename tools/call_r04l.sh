#!/bin/bash
# r04l: the split cores' round stagger and the residual layers' tile config on
# the bench's own embed; clock / power / temperature through the embed and the ranker
set -o pipefail
O=gpurun_out/r04l; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
timeout -k 10 280 python -u tools/power_probe.py 12 8 > $O/power_probe.txt 2>&1 && \
E2E_EMBED="s3_stagger=-1 s3_stagger=0 s3_stagger=16 s3_stagger=4" timeout -k 10 600 python -u tools/e2e_ab.py 1280 5 > $O/e2e_stagger.txt 2>&1 && \
E2E_EMBED="s3_cfg_res=0 s3_cfg_res=8 s3_cfg_res=12" timeout -k 10 600 python -u tools/e2e_ab.py 1280 5 > $O/e2e_cfg_res.txt 2>&1
grep -v amdgpu.ids $O/e2e_*.txt; tail -1 $O/tests.log; grep -c SAMPLE $O/power_probe.txt; grep PHASE $O/power_probe.txt
echo call-done
