#!/bin/bash
# Dev A/B: build the library with ${HEAD_SRC:-tools/dev/qlin_gemv_head.hip} (e.g. `git show HEAD:...`
# written there before the push) in place of csrc/qlin_gemv.hip as
# tools/dev/libqlin_head.so (on the GPU box: a pushed second library makes the tree twice as big)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
D=llama3-quantization_amd/csrc_head
rm -rf $D && mkdir -p $D
cp llama3-quantization_amd/csrc/*.hip llama3-quantization_amd/csrc/*.h llama3-quantization_amd/csrc/Makefile $D/
cp "${HEAD_SRC:-tools/dev/qlin_gemv_head.hip}" $D/qlin_gemv.hip
make -s -C $D -j16 OUT=$PWD/tools/dev/libqlin_head.so
rm -rf $D
