#!/bin/bash
# Build an experiment variant of liblvgpu.so with extra kernel defines:
#   tools/build_variant.sh NAME -DLVK_FOO=1 ...  ->  leveldb-rs_amd/lib/variants/liblvgpu_NAME.so
# Every HIP translation unit of the product (Makefile HIP_SRCS) is rebuilt
# with -DLVK_EXPERIMENT_BUILD=1 and the given defines (lvk/knobs.h refuses
# LVK_* switches in any other build).  Select the variant at run time with
# LVGPU_EXPERIMENT=1 LVGPU_LIB=<path> (the binding ignores LVGPU_LIB
# otherwise).  Variants never ship: lib/variants is in .gpurunignore, so
# build them on the GPU box inside the call that runs them.
set -e
name=$1; shift
cd "$(dirname "$0")/../leveldb-rs_amd"
make -s -j8 >/dev/null
srcs=$(make -s -f - print-hip <<'MK'
include Makefile
print-hip:
	@echo $(HIP_SRCS)
MK
)
mkdir -p build/variants/$name lib/variants
for src in $srcs; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -munsafe-fp-atomics -O3 -std=c++17 -fPIC -Wall -DLVK_EXPERIMENT_BUILD=1 "$@" \
    -c csrc/$src.hip -o build/variants/$name/$src.o &
done
wait
hostobjs="build/crc32c_scalar.o build/crc32c_multi.o build/wal_host.o build/sst_format.o"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib/variants/liblvgpu_$name.so build/variants/$name/*.o $hostobjs
echo lib/variants/liblvgpu_$name.so
