set -o pipefail
O=gpurun_out/r03x; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1; echo "tests rc=$?"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo smoke-ok && \
timeout -k 10 300 python -u bench.py > $O/c3.json 2> $O/c3.log && echo bench-ok && \
timeout -k 10 300 python -u tools/resid_ab.py 1280 "0:-1,0:0,0:16,0:24,8:-1,8:16" > $O/resid_ab.txt 2>&1 && echo resid-ok && \
timeout -k 10 300 python -u bench.py --workload c4 > $O/c4.json 2> $O/c4.log && echo c4-ok && \
timeout -k 10 300 python -u bench.py --workload c5 > $O/c5.json 2> $O/c5.log && echo c5-ok
