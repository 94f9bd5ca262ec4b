#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, no trace domains) on the
# C3 trunk's N = 64 halo 3x3 (layer1, 64@56) and the halo stem + max-pool at
# B = 1280 (tools/h2_one.py), plus the 3x3 256@14 halo for comparison.
# Counter names are checked against `rocprofv3 -L` first; unknown ones drop.
# usage (GPU box): bash tools/halo_pmc.sh <outdir>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/${1:-gpurun_out/halo_pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
have() { grep -qw "$1" $OUT/counters_list.txt; }
pick() { local o=""; for c in "$@"; do if have $c || have ${c%_sum}; then o="$o $c"; fi; done; echo $o; }
P1=$(pick SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE)
P2=$(pick SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE)
P3=$(pick SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT GRBM_GUI_ACTIVE)
echo "P1=$P1" > $OUT/passes.txt; echo "P2=$P2" >> $OUT/passes.txt; echo "P3=$P3" >> $OUT/passes.txt
for shape in "stem 1280" "conv 1280 56 56 64 64 3 1 1 0" "conv 1280 14 14 256 256 3 1 1 0"; do
  tag=$(echo $shape | tr ' ' _)
  mkdir -p $OUT/$tag
  timeout -k 10 120 python3 $R/tools/h2_one.py $shape 10 > $OUT/$tag/time.log 2>&1 || { echo "time $tag rc=$?" >> $OUT/passes.txt; exit 1; }
  i=1
  for P in "$P1" "$P2" "$P3"; do
    if [ -n "$P" ]; then
      timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/$tag/p$i -o run -- python3 $R/tools/h2_one.py $shape 3 > $OUT/$tag/p$i.log 2>&1 || { echo "pass $tag p$i rc=$?" >> $OUT/passes.txt; exit 1; }
    fi
    i=$((i+1))
  done
done
echo pmc-done
