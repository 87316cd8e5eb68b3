// Standalone HBM read-bandwidth probe (not product code): how fast can gfx950
// stream 1 GiB with dwordx4 loads in the access shapes the CRC kernel uses?
//   mode 0: grid-stride, each lane 16 B per iteration, fully coalesced 1 KiB/wave
//   mode 1: G-lane groups reading 16*G-byte rows of 4 KiB blocks (the CRC kernel's shape)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 g_u32x4;

__global__ __launch_bounds__(1024) void probe_stream(const u32x4* __restrict__ p, uint64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    u32x4 v = ((g_u32x4*)p)[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int G, int U>
__global__ __launch_bounds__(1024) void probe_groups(const u32x4* __restrict__ p, uint64_t nblocks, uint32_t blk16, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t gid = ((uint64_t)blockIdx.x * 16 + wave) * (64 / G) + lane / G;
  const uint64_t gstride = (uint64_t)gridDim.x * 16 * (64 / G);
  uint32_t acc = 0;
  for (uint64_t b = gid; b < nblocks; b += gstride) {
    const g_u32x4* q = (g_u32x4*)p + b * blk16 + (lane % G);
    for (uint32_t r = 0; r < blk16 / G; r += U) {
      u32x4 v[U];
#pragma unroll
      for (int j = 0; j < U; ++j) v[j] = q[(r + j) * G];
#pragma unroll
      for (int j = 0; j < U; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const uint64_t bytes = 1ull << 30;
  u32x4* d; uint32_t* o;
  hipMalloc(&d, bytes); hipMalloc(&o, 4);
  hipMemset(d, 1, bytes);
  int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  auto run = [&](const char* name, auto launch) {
    std::vector<float> ts;
    for (int it = 0; it < 23; ++it) {
      hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b); if (it >= 3) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    printf("%-40s median %.4f ms  %.0f GB/s  (min %.4f ms %.0f GB/s)\n", name, ts[ts.size()/2], bytes / (ts[ts.size()/2] * 1e-3) / 1e9, ts[0], bytes / (ts[0]*1e-3)/1e9);
  };
  for (int wgs : {cus, 2 * cus, 4 * cus, 8 * cus}) {
    char nm[64]; snprintf(nm, 64, "stream wg=%d x1024", wgs);
    run(nm, [&] { hipLaunchKernelGGL(probe_stream, dim3(wgs), dim3(1024), 0, 0, d, bytes / 16, o); });
  }
  const uint64_t nb = bytes / 4096;
  run("groups G=16 U=4 4KiB wg=cus", [&] { hipLaunchKernelGGL((probe_groups<16,4>), dim3(cus), dim3(1024), 0, 0, d, nb, 256u, o); });
  run("groups G=16 U=8 4KiB wg=cus", [&] { hipLaunchKernelGGL((probe_groups<16,8>), dim3(cus), dim3(1024), 0, 0, d, nb, 256u, o); });
  run("groups G=64 U=4 4KiB wg=cus", [&] { hipLaunchKernelGGL((probe_groups<64,4>), dim3(cus), dim3(1024), 0, 0, d, nb, 256u, o); });
  run("groups G=4 U=4 4KiB wg=cus", [&] { hipLaunchKernelGGL((probe_groups<4,4>), dim3(cus), dim3(1024), 0, 0, d, nb, 256u, o); });
  run("groups G=1 U=4 4KiB wg=cus", [&] { hipLaunchKernelGGL((probe_groups<1,4>), dim3(cus), dim3(1024), 0, 0, d, nb, 256u, o); });
  run("groups G=16 U=4 4KiB wg=2cus", [&] { hipLaunchKernelGGL((probe_groups<16,4>), dim3(2*cus), dim3(1024), 0, 0, d, nb, 256u, o); });
  return 0;
}
