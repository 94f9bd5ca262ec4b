# seam v2: its tests, the probe (wall + trace + counters), the embed A/B
set -o pipefail
R=$(pwd); O=$R/gpurun_out/${1:-r05e}; mkdir -p $O
ok() { r=$1; [ $r -eq 0 ] && return 0; [ $r -eq 1 ] && return 0; echo "fatal rc $r"; exit $r; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_seam.py -v -s --timeout 120 --timeout-method thread > $O/seam_tests.log 2>&1; ok $?
grep -E "seam |h1 vs|rescaled|passed|failed" $O/seam_tests.log | tail -12
SEAM_UNFUSED=1 timeout -k 10 120 python -u tools/seam_probe.py > $O/probe.txt 2>&1 || { echo probe-failed; tail $O/probe.txt; exit 1; }
cat $O/probe.txt
E2E_EMBED="fuse_seams=0 fuse_seams=1" timeout -k 10 300 python -u tools/e2e_ab.py 1280 4 > $O/e2e_seam.txt 2>&1 || { echo e2e-failed; tail -20 $O/e2e_seam.txt; exit 1; }
tail -2 $O/e2e_seam.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/tools/seam_probe.py > $O/fetch.log 2>&1 || { echo fetch-failed; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS --output-format csv -d $O/sq -o run -- python3 $R/tools/seam_probe.py > $O/sq.log 2>&1 || { echo sq-failed; exit 1; }
echo all-done
