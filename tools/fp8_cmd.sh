# fp8 cosine on the block-scaled MFMA: low-precision tests, then the sweep per config
mkdir -p gpurun_out/fp8
timeout -k 10 300 python -u -m pytest tests/test_gpu_lowp.py -x -v --timeout 120 --timeout-method thread > gpurun_out/fp8/tests.log 2>&1 || exit 1
for c in auto 22 41; do
  RR_GEMM_LPCFG=$c timeout -k 10 200 python tools/lp_bench.py >> gpurun_out/fp8/lp_bench.log 2>&1 || exit 2
done
