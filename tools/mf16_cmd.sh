# bf16 MFMA shape A/B: 32x32x16 (default) vs 16x16x32 (RR_BF16_MF16=1): tests under MF16, then lp_bench per arm
mkdir -p gpurun_out/mf16
RR_BF16_MF16=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_lowp.py tests/test_gpu_vit.py tests/test_gpu_rank.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mf16/tests.log 2>&1 || exit 1
for c in 22 big auto; do
  RR_GEMM_LPCFG=$c RR_BF16_MF16=0 timeout -k 10 200 python tools/lp_bench.py 2>&1 | sed 's/"cfg"/"mf16": 0, "cfg"/' >> gpurun_out/mf16/lp.log || exit 2
  RR_GEMM_LPCFG=$c RR_BF16_MF16=1 timeout -k 10 200 python tools/lp_bench.py 2>&1 | sed 's/"cfg"/"mf16": 1, "cfg"/' >> gpurun_out/mf16/lp.log || exit 3
done
