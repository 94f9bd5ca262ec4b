#!/bin/bash
# SQ counters for single split-bf16 conv shapes, one counter group per pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/s3c
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
for shape in "320 14 14 256 256 3 1 1 0" "320 14 14 256 1024 1 1 0 1"; do
  tag=$(echo $shape | tr ' ' '_')
  timeout -k 10 120 python3 $R/tools/s3_one.py $shape > $OUT/time_$tag.log 2>&1 || exit 1
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA" \
             "SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD" ; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/p${i}_$tag -o run -- python3 $R/tools/s3_one.py $shape 320 > $OUT/p${i}_$tag.log 2>&1 || echo "pass $i failed" >> $OUT/fail.log
  done
done
echo done
