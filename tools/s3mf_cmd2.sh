mkdir -p gpurun_out/s3mf
for c in 2 5; do
  for m in 0 1; do
    RR_S3_CFG=$c S3_ONLY=1 RR_S3_MF16=$m timeout -k 10 200 python -u tools/s3_bench.py 320 10 > gpurun_out/s3mf/b_${c}_$m.log 2>&1 || exit 2
  done
done
