# A/B: 256x320 bf16 sweep tile, 2-stage (default) vs 4-stage LDS-DMA ring (q320r)
set -o pipefail
O=gpurun_out/q320r
mkdir -p $O
RR_GEMM_LPCFG=q320r timeout -k 10 300 python -u -m pytest tests/test_gpu_rank.py tests/test_gpu_fullsize.py -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for c in default q320r default q320r; do
  if [ "$c" = default ]; then unset RR_GEMM_LPCFG; else export RR_GEMM_LPCFG=$c; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 >> $O/c3_$c.json 2>> $O/c3_$c.err || exit 2
done
echo all-done
