#!/bin/bash
# SQ counters for single conv shapes (one counter group per rocprofv3 pass)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/cstall
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
for shape in "320 14 14 256 256 3 1 1 0" "320 14 14 256 1024 1 1 0 1" "320 14 14 1024 256 1 1 0 0"; do
  tag=$(echo $shape | tr ' ' '_')
  timeout -k 10 120 python3 $R/tools/conv_one.py $shape > $OUT/time_$tag.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/p1_$tag -o run -- python3 $R/tools/conv_one.py $shape > $OUT/p1_$tag.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2_$tag -o run -- python3 $R/tools/conv_one.py $shape > $OUT/p2_$tag.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_F32 --output-format csv -d $OUT/p3_$tag -o run -- python3 $R/tools/conv_one.py $shape > $OUT/p3_$tag.log 2>&1
done
echo done
