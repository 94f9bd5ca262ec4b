# cosine sweep tile at 1280 queries: default pick vs forced 256x256 (big, 16x16x32) in the C3 / C4 benches
mkdir -p gpurun_out/swp
for c in default big; do
  if [ "$c" = default ]; then unset RR_GEMM_LPCFG; else export RR_GEMM_LPCFG=$c; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 > gpurun_out/swp/c3_$c.json 2> gpurun_out/swp/c3_$c.err || exit 1
  timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline --steps 5 > gpurun_out/swp/c4_$c.json 2> gpurun_out/swp/c4_$c.err || exit 1
done
