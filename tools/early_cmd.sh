# A/B: filter epilogue with / without the per-lane max early-out (ab/base.so vs ab/early.so)
set -o pipefail
O=gpurun_out/early
mkdir -p $O
RR_LIB_PATH=$PWD/ab/early.so timeout -k 10 400 python -u -m pytest tests/test_gpu_rank.py tests/test_gpu_fullsize.py tests/test_gpu_lowp.py -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || exit 1
bash tools/ab.sh 2 python -u bench.py --no-cpu-baseline --steps 5 > $O/c3.log 2> $O/c3.err || exit 2
bash tools/ab.sh 2 python -u bench.py --workload c4 --no-cpu-baseline --steps 5 > $O/c4.log 2> $O/c4.err || exit 3
echo all-done
