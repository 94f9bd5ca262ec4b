#!/bin/bash
# Same-device A/B of librr builds: ab.sh <rounds> <cmd...>; runs cmd once per
# ab/*.so per round, interleaved, output tagged by variant.
R=$1; shift
for r in $(seq 1 $R); do
  for so in ab/*.so; do
    echo "== $(basename $so) round $r"
    RR_LIB_PATH=$PWD/$so timeout -k 10 200 "$@" || exit 1
  done
done
