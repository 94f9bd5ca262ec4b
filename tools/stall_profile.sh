#!/bin/bash
# SQ stall counters for the cosine kernel (microbench), one counter group per pass.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/stall
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
M="python3 $R/tools/microbench.py --q 256 --n 400000"
export PYTHONPATH=$R
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/p1 -o run -- $M > $OUT/p1.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_F32 --output-format csv -d $OUT/p2 -o run -- $M > $OUT/p2.log 2>&1 || true
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/p3 -o run -- $M > $OUT/p3.log 2>&1 || true
echo done
