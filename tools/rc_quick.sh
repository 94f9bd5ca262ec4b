set -o pipefail
O=gpurun_out/r1f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err && \
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err && \
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err && \
echo all-done
