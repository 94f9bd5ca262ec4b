#!/bin/bash
# r04k: the halo 3x3 MFMA form on the bench's own embed; the defaults' sweep again
set -o pipefail
O=gpurun_out/r04k; mkdir -p $O
E2E_EMBED="halo_mf=0 halo_mf=-1 halo_mf=1" E2E_RANK="sweep_il=0 sweep_il=-1" \
  timeout -k 10 600 python -u tools/e2e_ab.py 1280 6 > $O/e2e_ab.txt 2>&1
grep -v amdgpu.ids $O/e2e_ab.txt
echo call-done
