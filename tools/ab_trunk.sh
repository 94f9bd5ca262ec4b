#!/bin/bash
# Interleaved A/B of the R101 trunk convs + stem at 1280 images on one device
# (tools/s3_bench.py, tools/stem_ab.py), two rounds:
#   bash tools/ab_trunk.sh <tag> lib <path.so|main>...   librr builds (RR_LIB_PATH)
#   bash tools/ab_trunk.sh <tag> cfg <0..7>...           forced split-bf16 tile config
#   bash tools/ab_trunk.sh <tag> stagger <-1..200>...    forced round stagger
set -o pipefail
TAG=$1; KIND=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
for r in 1 2; do
  for v in "$@"; do
    case $KIND in
      lib) n=$(basename $v .so); if [ "$v" = main ]; then env=""; else env="RR_LIB_PATH=$v"; fi ;;
      cfg) n=cfg$v; env="S3_CFG=$v" ;;
      stagger) n=st$v; env="S3_STAGGER=$v" ;;
      *) echo "unknown kind $KIND"; exit 2 ;;
    esac
    env $env S3_ONLY=1 timeout -k 10 200 python -u tools/s3_bench.py 1280 8 > $O/${n}_$r.txt 2>&1 || exit 1
    env $env timeout -k 10 100 python -u tools/stem_ab.py 1280 >> $O/${n}_$r.txt 2>&1 || exit 1
  done
done
grep -H -E "TOTAL|stem s3" $O/*.txt
