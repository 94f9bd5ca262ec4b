#!/bin/bash
# r04i: the C3 line with the round-4 issue-spread / 16x16x32 sweep defaults vs
# all three off (same box, back to back, twice)
set -o pipefail
O=gpurun_out/r04i; mkdir -p $O
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/c3_new_$r.json 2> $O/c3_new_$r.log || exit 1
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --tune sweep_il=0,sweep_mf16=0,conv_il=0 > $O/c3_old_$r.json 2> $O/c3_old_$r.log || exit 1
done
for f in $O/c3_*.json; do python -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);r=d['roofline_by_kernel'];print('$f',d['value'],d['ms_per_step'],r['conv_gemm']['ms_per_step'],r['cosine_filter']['ms_per_step'])"; done
echo call-done
