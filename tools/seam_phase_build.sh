#!/bin/bash
# Diagnostic librr with the seam kernel's s_memtime phase timers
# (-DRR_SEAM_PHASES=1, gemm_seam.hip) -> ab/librr_seam_phases.so, for
# tools/seam_probe.py with SEAM_PHASES=1 (RR_LIB_PATH=ab/librr_seam_phases.so).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
B=/tmp/rr_seam_phase_build
mkdir -p $B $R/ab
cd $R/research_image_retrieval_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -DRR_SEAM_PHASES=1 -c gemm_seam.hip -o $B/gemm_seam.o
objs=$B/gemm_seam.o
for f in *.o; do [ "$f" = gemm_seam.o ] || objs="$objs $f"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o $R/ab/librr_seam_phases.so
echo built $R/ab/librr_seam_phases.so
