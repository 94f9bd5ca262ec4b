# 8-phase 256x256 bf16 GEMM (RR_GEMM_8P=1): low-precision / ViT / rank tests, then A/B timing
mkdir -p gpurun_out/p8
RR_GEMM_8P=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_lowp.py tests/test_gpu_vit.py -x -q --timeout 120 --timeout-method thread > gpurun_out/p8/tests.log 2>&1 || exit 1
for m in 0 1; do
  RR_GEMM_LPCFG=big RR_GEMM_8P=$m timeout -k 10 200 python tools/lp_bench.py 2>&1 | sed "s/\"cfg\"/\"p8\": $m, \"cfg\"/" >> gpurun_out/p8/lp.log || exit 2
done
RR_GEMM_8P=1 timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline --steps 5 > gpurun_out/p8/c4.json 2> gpurun_out/p8/c4.err || exit 3
