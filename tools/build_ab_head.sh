#!/bin/bash
# Build librr from the committed HEAD into ab/head.so and the working tree into ab/new.so.
set -e
ROOT=$(git rev-parse --show-toplevel)
T=$(mktemp -d)
git -C $ROOT archive HEAD research_image_retrieval_amd/csrc include | tar -x -C $T
make -s -C $T/research_image_retrieval_amd/csrc -j8
mkdir -p $ROOT/ab
cp $T/research_image_retrieval_amd/librr.so $ROOT/ab/head.so
make -s -C $ROOT/research_image_retrieval_amd/csrc -j8
cp $ROOT/research_image_retrieval_amd/librr.so $ROOT/ab/new.so
rm -rf $T
