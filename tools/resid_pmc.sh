#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, no trace domains) on the
# residual expansion 256->1024 @14x14 (config 12), the 1024->256 reduction and
# the 3x3 256@14 halo tile at B=1280, plus the pure HBM read/write mix probe.
# Counter names are checked against `rocprofv3 -L` first; unknown ones drop.
# usage (GPU box): bash tools/resid_pmc.sh <outdir>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/${1:-gpurun_out/resid_pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
have() { grep -qw "$1" $OUT/counters_list.txt; }
pick() { local o=""; for c in "$@"; do if have $c || have ${c%_sum}; then o="$o $c"; fi; done; echo $o; }
P1=$(pick SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE)
P2=$(pick TA_TA_BUSY_sum TA_BUSY_avr TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE)
P3=$(pick TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE)
P4=$(pick TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum GRBM_GUI_ACTIVE)
echo "P1=$P1" > $OUT/passes.txt; echo "P2=$P2" >> $OUT/passes.txt; echo "P3=$P3" >> $OUT/passes.txt; echo "P4=$P4" >> $OUT/passes.txt
for shape in "1280 14 14 256 1024 1 1 0 1" "1280 14 14 1024 256 1 1 0 0" "1280 14 14 256 256 3 1 1 0"; do
  tag=$(echo $shape | tr ' ' _)
  i=1
  for P in "$P1" "$P2" "$P3" "$P4"; do
    mkdir -p $OUT/$tag
    [ -n "$P" ] && timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/$tag/p$i -o run -- python3 $R/tools/h2_one.py conv $shape 5 > $OUT/$tag/p$i.log 2>&1 || echo "pass $tag p$i rc=$?" >> $OUT/passes.txt
    i=$((i+1))
  done
done
echo pmc-done
