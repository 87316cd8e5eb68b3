#!/bin/bash
# Build an experiment variant of liblvgpu.so with extra kernel defines:
#   tools/build_variant.sh NAME -DLVK_FOO=1 ...  ->  leveldb-rs_amd/lib/variants/liblvgpu_NAME.so
# SRC=hash (or another csrc/*.hip stem) rebuilds that source instead of
# crc32c_batch.hip.  Select the variant at run time with LVGPU_EXPERIMENT=1
# LVGPU_LIB=<path> (the binding ignores LVGPU_LIB otherwise).  Variants never
# ship: lib/variants is in .gpurunignore, so build them on the GPU box inside
# the call that runs them.
set -e
name=$1; shift
src=${SRC:-crc32c_batch}
cd "$(dirname "$0")/../leveldb-rs_amd"
make -s -j8 >/dev/null
mkdir -p build/variants lib/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -munsafe-fp-atomics -O3 -std=c++17 -fPIC -Wall -DLVK_EXPERIMENT_BUILD=1 "$@" \
  -c csrc/$src.hip -o build/variants/${src}_$name.o
objs=$(ls build/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib/variants/liblvgpu_$name.so build/variants/${src}_$name.o $objs
echo lib/variants/liblvgpu_$name.so
