#!/bin/bash
# r04j: conv_il / sweep_il / sweep_mf16 on the bench's own embed and ranker
set -o pipefail
O=gpurun_out/r04j; mkdir -p $O
E2E_EMBED="conv_il=0 conv_il=1" E2E_RANK="sweep_il=0,sweep_mf16=0 sweep_il=1,sweep_mf16=0 sweep_il=0,sweep_mf16=1 sweep_il=1,sweep_mf16=1" \
  timeout -k 10 600 python -u tools/e2e_ab.py 1280 4 > $O/e2e_ab.txt 2>&1
cat $O/e2e_ab.txt | grep -v amdgpu.ids
echo call-done
