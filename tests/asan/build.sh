#!/bin/bash
# Sanitizer builds, host code only: the GPU pool runs no GPU
# AddressSanitizer, so -fsanitize goes on the host side of every hipcc line
# (-Xarch_host) and device code is built unchanged.
#   bash tests/asan/build.sh : oracle_check (gcc ASan+UBSan over oracle/cosine_topk.c),
#                              librr_asan.so (librr with ASan host code) and abi_check
# `abi_check` runs the no-GPU checks, `abi_check gpu` adds the device ones (GPU box).
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
OUT=$HERE/out
mkdir -p "$OUT"
SRC=$(sed -n 's/^SRCS := //p' "$ROOT/research_image_retrieval_amd/csrc/Makefile")  # the product library's sources
SAN="-Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
gcc -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -ffp-contract=off -std=c11 \
    "$ROOT/oracle/cosine_topk.c" "$HERE/oracle_check.c" -lm -o "$OUT/oracle_check"
pids=()
for f in $SRC; do
  $HIPCC --offload-arch=gfx950 -O2 -g -std=c++17 -fPIC $SAN -c "$ROOT/research_image_retrieval_amd/csrc/$f" \
      -o "$OUT/${f%.hip}.o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
$HIPCC --offload-arch=gfx950 -shared -fPIC $SAN "$OUT"/*.o -o "$OUT/librr_asan.so"
$HIPCC --offload-arch=gfx950 -O1 -g -std=c++17 $SAN "$HERE/abi_check.cpp" \
    -L"$OUT" -lrr_asan -Wl,-rpath,'$ORIGIN' -o "$OUT/abi_check"
rm -f "$OUT"/*.o
echo "asan build ok"
