# full-size (1.6 M x 2048) ranker property tests, then the whole GPU suite
set -o pipefail
O=gpurun_out/fs
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 240 --timeout-method thread > $O/fullsize.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
echo all-done
