#!/bin/bash
# Diagnostic librr with the f16x2 kernels' s_memtime phase timers compiled in
# (-DRR_S3_PHASES=1, gemm_s3.hip) -> ab/librr_phases.so; tools/phase_run.py
# loads it through RR_LIB_PATH.  Built here (CPU), not on the GPU box.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
B=/tmp/rr_phase_build
mkdir -p $B $R/ab
cd $R/research_image_retrieval_amd/csrc
objs=""
for f in *.hip; do
  o=$B/${f%.hip}.o
  extra=""
  [ "$f" = gemm_s3.hip ] && extra="-DRR_S3_PHASES=1"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $extra -c $f -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o $R/ab/librr_phases.so
echo built $R/ab/librr_phases.so
