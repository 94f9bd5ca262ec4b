#!/bin/bash
# r04z2: round-end evidence 2 -- the C4, C5, clustered-gallery C3 and C2 lines
set -o pipefail
bash tools/evidence_lines.sh r04z2
