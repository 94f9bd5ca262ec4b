#!/bin/bash
# r04k: the halo 3x3 MFMA form on the bench's own C3 embed; the ViT linears'
# DMA spread (lp_il) on the C4 embed; their bit-identity tests
set -o pipefail
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_vit.py tests/test_gpu_ops.py -m gpu -x -v -s --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
E2E_EMBED="halo_mf=0 halo_mf=-1 halo_mf=1" timeout -k 10 600 python -u tools/e2e_ab.py 1280 5 > $O/e2e_halo.txt 2>&1 && \
E2E_WORKLOAD=c4 E2E_EMBED="lp_il=0 lp_il=1" timeout -k 10 400 python -u tools/e2e_ab.py 1280 5 > $O/e2e_c4_il.txt 2>&1
grep -v amdgpu.ids $O/e2e_*.txt; tail -1 $O/tests.log
echo call-done
