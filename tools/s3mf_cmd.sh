# s3 core MFMA shape A/B: 32x32x16 vs 16x16x32 (RR_S3_MF16=1), tests under MF16 then per-layer timing
mkdir -p gpurun_out/s3mf
RR_S3_MF16=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_s3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s3mf/tests_auto.log 2>&1 || exit 1
RR_S3_MF16=1 RR_S3_CFG=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_s3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s3mf/tests_cfg4.log 2>&1 || exit 1
for c in auto 3 4; do
  for m in 0 1; do
    if [ "$c" = auto ]; then unset RR_S3_CFG; else export RR_S3_CFG=$c; fi
    S3_ONLY=1 RR_S3_MF16=$m timeout -k 10 200 python -u tools/s3_bench.py 320 10 > gpurun_out/s3mf/b_${c}_$m.log 2>&1 || exit 2
  done
done
