mkdir -p gpurun_out
for shape in "320 14 14 256 256 3 1 1 0" "320 14 14 256 1024 1 1 0 1" "320 14 14 1024 256 1 1 0 0" "320 28 28 128 512 1 1 0 1" "320 7 7 512 2048 1 1 0 1" "320 56 56 64 256 1 1 0 1" "320 56 56 256 128 1 1 0 0" "320 28 28 512 256 1 1 0 0" "320 28 28 512 1024 1 2 0 0" "320 14 14 1024 2048 1 2 0 0" "320 14 14 1024 512 1 1 0 0" "320 7 7 2048 512 1 1 0 0" "320 56 56 256 512 1 2 0 0" "320 56 56 64 256 1 1 0 0" "320 56 56 256 64 1 1 0 0"; do
  for cfg in 22 88; do
    echo "$cfg $shape $(RR_GEMM_CFG=$cfg timeout -k 10 60 python tools/conv_one.py $shape 2>/dev/null | tail -1)" >> gpurun_out/conv_88b.log || exit 1
  done
  echo "auto $shape $(timeout -k 10 60 python tools/conv_one.py $shape 2>/dev/null | tail -1)" >> gpurun_out/conv_88b.log || exit 1
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1
RR_GEMM_NO88=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3_no88.log 2>&1
