#!/bin/bash
# SQ counters + kernel trace of the bf16 GEMM core on the ViT-B/16 linears at
# 1280 images (M = 252160): one rocprofv3 pass per counter group.
# usage (GPU box): bash tools/lp_pmc.sh <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/${1:-gpurun_out/lppmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"
for shape in "252160 768 2304 0 1 0" "252160 768 3072 2 1 0" "252160 3072 768 0 0 1"; do
  tag=$(echo $shape | tr ' ' _)
  mkdir -p $OUT/$tag
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag/kt -o run -- python3 $R/tools/lp_one.py $shape 5 > $OUT/$tag/kt.log 2>&1
  i=1
  for P in "$P1" "$P2"; do
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/$tag/p$i -o run -- python3 $R/tools/lp_one.py $shape 5 > $OUT/$tag/p$i.log 2>&1
    i=$((i+1))
  done
done
echo pmc-done
