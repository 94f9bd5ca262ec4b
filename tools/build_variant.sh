#!/bin/bash
# Build the working tree's librr with extra compiler flags into ab/<name>.so
# (A/B experiments: RR_LIB_PATH=ab/<name>.so).  usage: build_variant.sh name -DFLAG ...
set -e
ROOT=$(git -C "$(dirname "$0")" rev-parse --show-toplevel)
NAME=$1; shift
T=$(mktemp -d)
mkdir -p $T/research_image_retrieval_amd/csrc $T/include
cp $ROOT/research_image_retrieval_amd/csrc/*.hip $ROOT/research_image_retrieval_amd/csrc/*.hpp $ROOT/research_image_retrieval_amd/csrc/Makefile $T/research_image_retrieval_amd/csrc/
cp $ROOT/include/*.h $T/include/
make -s -C $T/research_image_retrieval_amd/csrc -j8 CXXFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $*" 2>&1 | grep -v hip-link || true
mkdir -p $ROOT/ab
cp $T/research_image_retrieval_amd/librr.so $ROOT/ab/$NAME.so
rm -rf $T
echo "built ab/$NAME.so"
