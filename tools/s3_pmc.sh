#!/bin/bash
# SQ counters of the split conv kernels (RR_CORE=h2 default, or s3) on the
# three R101 layer3 shapes (B=1280): one rocprofv3 --pmc pass per counter
# group (no trace domains).  usage (GPU box): bash tools/s3_pmc.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/${1:-gpurun_out/s3pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P3="SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for shape in "1280 14 14 256 1024 1 1 0 1" "1280 14 14 1024 256 1 1 0 0" "1280 14 14 256 256 3 1 1 0"; do
  tag=$(echo $shape | tr ' ' _)
  i=1
  for P in "$P1" "$P2" "$P3"; do
    mkdir -p $OUT/$tag
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/$tag/p$i -o run -- python3 $R/tools/s3_one.py $shape 5 > $OUT/$tag/p$i.log 2>&1
    i=$((i+1))
  done
done
echo pmc-done
