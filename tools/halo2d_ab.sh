#!/bin/bash
# A/B of the 2-D block halo tiles on C2's wide stride-1 3x3 layers (1024 x 768
# gallery images: 64@256x192, 128@128x96, 256@64x48 at batch B, default 64;
# and a batch-1 query crop's, 600 x 800), halo_2d 0 (the implicit-GEMM tiles)
# vs the default, alternating processes on one box.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
B=${B:-64}
for rep in 1 2; do
  for shape in "$B 256 192 64 64" "$B 128 96 128 128" "$B 64 48 256 256" "1 150 200 64 64" "1 75 100 128 128" "1 38 50 256 256"; do
    for t in 0 -1 1; do
      echo -n "halo_2d=$t conv $shape: "
      H2_TUNE=halo_2d=$t timeout -k 10 120 python3 $R/tools/h2_one.py conv $shape 3 1 1 0 20 2>/dev/null
    done
  done
done
