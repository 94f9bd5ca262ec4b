#!/bin/bash
# Same-binary A/B over an environment knob: ab_env.sh VAR "v1 v2 ..." rounds cmd...
VAR=$1; VALS=$2; R=$3; shift 3
for r in $(seq 1 $R); do
  for v in $VALS; do
    echo "== $VAR=$v round $r"
    env $VAR=$v timeout -k 10 200 "$@" || exit 1
  done
done
