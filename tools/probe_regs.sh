#!/bin/bash
# Register/spill report of per-G sorted_stream probe kernels (development aid).
set -e
src=/root/repo/leveldb-rs_amd/csrc/crc32c_batch.hip
python3 - "$src" <<'PY'
import sys
s=open(sys.argv[1]).read()
probe='''
template <int G>
__global__ __launch_bounds__(kThreads) void sorted_probe_kernel(Params P, const uint4 *__restrict__ image) {
    stage_tables(image);
    const uint32_t lane = threadIdx.x & 63u;
    const Lut L = make_lut(lane);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    sorted_stream<G>(P, blockIdx.x * kWaves + wave, gridDim.x * kWaves, lane, L);
}
template __global__ void sorted_probe_kernel<1>(Params, const uint4 *);
template __global__ void sorted_probe_kernel<4>(Params, const uint4 *);
template __global__ void sorted_probe_kernel<16>(Params, const uint4 *);
'''
s=s.replace("__device__ __forceinline__ uint64_t splitmix64", probe + "\n__device__ __forceinline__ uint64_t splitmix64",1)
d='/root/repo/leveldb-rs_amd/csrc/'
s=s.replace('#include "../../include','#include "/root/repo/include').replace('#include "crc32c_gf2.h"','#include "'+d+'crc32c_gf2.h"').replace('#include "lv_internal.h"','#include "'+d+'lv_internal.h"')
open('/tmp/probe.hip','w').write(s)
PY
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o /tmp/probe.s /tmp/probe.hip -Rpass-analysis=kernel-resource-usage 2>&1 \
 | grep -E "Function Name|VGPRs:|VGPRs Spill" | grep -A2 "probe_kernel\|classes" | grep -v "^--" | sed 's/.*remark: *//; s/ \[-Rpass.*//'
