#!/bin/bash
# r04w: the C3 prefilter sweep's tile configs on the bench's own descriptors
set -o pipefail
O=gpurun_out/r04w; mkdir -p $O
E2E_RANK="lp_cfg=0 lp_cfg=3,sweep_il=1 lp_cfg=3,sweep_il=0 lp_cfg=5 lp_cfg=0,sweep_order=2" \
  timeout -k 10 600 python -u tools/e2e_ab.py 1280 4 > $O/e2e_sweep_cfg.txt 2>&1
grep -v amdgpu.ids $O/e2e_sweep_cfg.txt
echo call-done
