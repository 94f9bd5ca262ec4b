#!/bin/bash
# r04e: DMA issue spread across the MFMAs (fetch_ceiling IL variants)
set -o pipefail
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 180 ./tools/fetch_ceiling 5 il > $O/fetch_ceiling_il.txt 2>&1 && tail -9 $O/fetch_ceiling_il.txt && echo call-done
