#!/bin/bash
# Experiment build of libocffm.so with extra compiler flags (run from the repo root):
#   bash tools/build_variant.sh <tag> "<flags>"   ->  one-class-ffm_amd/exp/libocffm_<tag>.so
# Select it at run time with OCFFM_LIB=one-class-ffm_amd/exp/libocffm_<tag>.so.
set -e -o pipefail
tag=$1
flags=$2
cd one-class-ffm_amd
make -s build/sgd.o build/host_data.o
mkdir -p exp build_$tag
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I../include $flags \
  -c -o build_$tag/solver.o csrc/solver.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o exp/libocffm_$tag.so build_$tag/solver.o build/sgd.o \
  build/host_data.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
