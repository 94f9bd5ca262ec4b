mkdir -p gpurun_out/fp8
for c in big q320 big4; do
  RR_GEMM_LPCFG=$c timeout -k 10 200 python tools/lp_bench.py >> gpurun_out/fp8/lp_bench2.log 2>&1 || exit 2
done
timeout -k 10 400 python bench.py --workload c5 --no-cpu-baseline > gpurun_out/fp8/c5.json 2> gpurun_out/fp8/c5.err || exit 3
