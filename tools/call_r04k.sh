#!/bin/bash
# r04k: the halo 3x3 MFMA form on the bench's own C3 embed; the ViT linears'
# DMA spread (lp_il) on the C4 embed; the fp8 sweeps' spread on the C5 line;
# their bit-identity tests
set -o pipefail
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_vit.py tests/test_gpu_ops.py tests/test_gpu_rank.py -m gpu -x -v -s --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
E2E_EMBED="halo_mf=0 halo_mf=-1 halo_mf=1" timeout -k 10 600 python -u tools/e2e_ab.py 1280 5 > $O/e2e_halo.txt 2>&1 && \
E2E_WORKLOAD=c4 E2E_EMBED="lp_il=0 lp_il=1" timeout -k 10 400 python -u tools/e2e_ab.py 1280 5 > $O/e2e_c4_il.txt 2>&1 && \
timeout -k 10 400 python -u bench.py --workload c5 --no-cpu-baseline --steps 6 > $O/c5_base.json 2> $O/c5_base.log && \
timeout -k 10 400 python -u bench.py --workload c5 --no-cpu-baseline --steps 6 --tune sweep_il=1 > $O/c5_il.json 2> $O/c5_il.log
grep -v amdgpu.ids $O/e2e_*.txt; tail -1 $O/tests.log
for f in $O/c5_*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);r=d['roofline_by_kernel'];print('$f',d['value'],d['ms_per_step'],r['cosine_filter'])"; done
echo call-done
