# seam probe: wall times, rocprofv3 kernel trace, PMC passes on the fused kernel
set -o pipefail
R=$(pwd); O=$R/gpurun_out/${1:-r05d}; mkdir -p $O
SEAM_UNFUSED=1 timeout -k 10 120 python -u tools/seam_probe.py > $O/probe.txt 2>&1 || { echo probe-failed; tail $O/probe.txt; exit 1; }
cat $O/probe.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/seam_probe.py > $O/trace.log 2>&1 || { echo trace-failed; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/tools/seam_probe.py > $O/fetch.log 2>&1 || { echo fetch-failed; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/tools/seam_probe.py > $O/write.log 2>&1 || { echo write-failed; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS --output-format csv -d $O/sq -o run -- python3 $R/tools/seam_probe.py > $O/sq.log 2>&1 || { echo sq-failed; exit 1; }
echo all-done
