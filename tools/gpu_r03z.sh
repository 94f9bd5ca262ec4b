set -o pipefail
O=gpurun_out/r03z; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_h2.py -m gpu -x -v -s --timeout 120 --timeout-method thread -k "residual_pipelined" > $O/rp_tests.log 2>&1 && echo rp-tests-ok && \
timeout -k 10 300 python -u tools/resid_ab.py 1280 "0:-1,8:-1,14:0" > $O/resid_ab.txt 2>&1 && echo resid-ok
