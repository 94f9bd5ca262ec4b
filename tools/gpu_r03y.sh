set -o pipefail
O=gpurun_out/r03y; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_h2.py -m gpu -x -v -s --timeout 120 --timeout-method thread -k "stem" > $O/stem_tests.log 2>&1 && echo stem-tests-ok && \
timeout -k 10 200 python -u tools/stem_ab.py 1280 > $O/stem_ab.txt 2>&1 && echo stem-ab-ok && \
timeout -k 10 300 python -u bench.py > $O/c3.json 2> $O/c3.log && echo c3-ok && \
timeout -k 10 500 python -u bench.py --workload c2 > $O/c2.json 2> $O/c2.log && echo c2-ok && \
timeout -k 10 300 python -u bench.py --workload c3 --gallery-kind clustered > $O/c3_clustered.json 2> $O/c3_clustered.log && echo clustered-ok
