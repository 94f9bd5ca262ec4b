# C4 with the short-K sweep pick; C5 fp8 sweep default vs forced 256x256
mkdir -p gpurun_out/swp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lowp.py tests/test_gpu_rank.py -x -q --timeout 120 --timeout-method thread > gpurun_out/swp/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline --steps 5 > gpurun_out/swp/c4_new.json 2> gpurun_out/swp/c4_new.err || exit 1
for c in default big; do
  if [ "$c" = default ]; then unset RR_GEMM_LPCFG; else export RR_GEMM_LPCFG=$c; fi
  timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --steps 5 > gpurun_out/swp/c5_$c.json 2> gpurun_out/swp/c5_$c.err || exit 1
done
