#!/bin/bash
# Stem + max-pool launch A/B between two librr builds (alternating processes,
# one box): usage: bash tools/stem_ab.sh <libA> <libB> [rounds]
set -o pipefail
A=$1; B=$2; N=${3:-3}
for i in $(seq 1 $N); do
  for L in $A $B; do
    echo -n "$(basename $L .so) round $i: "
    RR_LIB_PATH=$L timeout -k 10 120 python3 tools/h2_one.py stem 1280 20 2>/dev/null || exit 1
  done
done
