#!/bin/bash
# A/B two librr builds in alternating processes on one box (a change a tuning
# key cannot switch): usage: bash tools/lib_ab.sh <tag> <libA> <libB> [rounds]
# -> per-layer sweep (h2_cfg_sweep, the picks) and the bench's embed per lib.
set -o pipefail
TAG=$1; A=$2; B=$3; N=${4:-3}
O=gpurun_out/$TAG
mkdir -p $O
for i in $(seq 1 $N); do
  for L in $A $B; do
    n=$(basename $L .so)
    RR_LIB_PATH=$L timeout -k 10 200 python -u tools/h2_cfg_sweep.py 1280 0 > $O/sweep_${n}_$i.txt 2>&1 || { echo "sweep $L failed"; tail -5 $O/sweep_${n}_$i.txt; exit 1; }
    E2E_EMBED="s3_cfg=0" RR_LIB_PATH=$L timeout -k 10 200 python -u tools/e2e_ab.py 1280 3 > $O/e2e_${n}_$i.txt 2>&1 || { echo "e2e $L failed"; tail -5 $O/e2e_${n}_$i.txt; exit 1; }
    echo "$n round $i: $(grep weighted $O/sweep_${n}_$i.txt) | $(grep embed $O/e2e_${n}_$i.txt)"
  done
done
