set -o pipefail
O=gpurun_out/r03w; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_h2.py -m gpu -x -v -s --timeout 120 --timeout-method thread -k "halo or tile_configs" > $O/halo_tests.log 2>&1 && echo halo-tests-ok && \
timeout -k 10 400 python -u tools/h2_cfg_sweep.py 1280 0,13 > $O/h2_sweep.txt 2>&1 && echo sweep-ok && \
timeout -k 10 300 python -u bench.py > $O/c3.json 2> $O/c3.log && echo bench-ok && \
bash tools/profile.sh > $O/profile.log 2>&1 && echo profile-ok
