set -o pipefail
O=gpurun_out/fslp
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize_lowp.py -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 && echo all-done
