# seam kernel: its tests, the embed A/B (fuse_seams off/on), trunk/e2e/h2 tests, the C3 bench line
set -o pipefail
O=gpurun_out/${1:-r05c}; mkdir -p $O
ok() { r=$1; [ $r -eq 0 ] && return 0; [ $r -eq 1 ] && return 0; echo "fatal rc $r"; exit $r; }  # 1 = test failures: go on
timeout -k 10 300 python -u -m pytest tests/test_gpu_seam.py -v -s --timeout 120 --timeout-method thread > $O/seam_tests.log 2>&1; ok $?
tail -3 $O/seam_tests.log
E2E_EMBED="fuse_seams=0 fuse_seams=1" timeout -k 10 300 python -u tools/e2e_ab.py 1280 4 > $O/e2e_seam.txt 2>&1 || { echo e2e-failed; tail -20 $O/e2e_seam.txt; exit 1; }
tail -3 $O/e2e_seam.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_trunk.py tests/test_gpu_e2e.py -v -s --timeout 240 --timeout-method thread > $O/trunk_tests.log 2>&1; ok $?
tail -3 $O/trunk_tests.log
timeout -k 10 400 python -u bench.py > $O/c3.json 2> $O/c3.log || { echo bench-failed; tail -20 $O/c3.log; exit 1; }
head -c 300 $O/c3.json; echo
echo all-done
