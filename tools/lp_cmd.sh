mkdir -p gpurun_out
for c in 22 big q320; do
  RR_GEMM_LPCFG=$c timeout -k 10 200 python tools/lp_bench.py >> gpurun_out/lp_bench3.log 2>&1 || exit 1
done
RR_GEMM_LPCFG=big timeout -k 10 300 python -m pytest tests/test_gpu_lowp.py tests/test_gpu_vit.py tests/test_gpu_rank.py -x -q > gpurun_out/lp_tests3.log 2>&1 || exit 2
