#!/bin/bash
# Experiment build of libocffm.so with extra compiler flags (run from the repo root):
#   bash tools/build_variant.sh <tag> "<flags>" [patch]  ->  one-class-ffm_amd/exp/libocffm_<tag>.so
# Select it at run time with OCFFM_LIB=one-class-ffm_amd/exp/libocffm_<tag>.so.
# patch (optional): a diff of csrc/ applied to a copy of the sources first.
set -e -o pipefail
tag=$1
flags=$2
patch_file=${3:-}
cd one-class-ffm_amd
make -s build/sgd.o build/host_data.o build/devbuild.o
mkdir -p exp build_$tag
src=csrc
if [ -n "$patch_file" ]; then
  rm -rf csrc_$tag && cp -r csrc csrc_$tag  # (same depth: the sources include ../../include)
  (cd csrc_$tag && patch -p3 < "$patch_file")
  src=csrc_$tag
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I../include $flags \
  -c -o build_$tag/solver.o $src/solver.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o exp/libocffm_$tag.so build_$tag/solver.o build/sgd.o \
  build/devbuild.o build/host_data.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
