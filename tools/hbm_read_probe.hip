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

template <bool NT>
__global__ __launch_bounds__(1024) void probe_stream_u(const u32x4* __restrict__ p, uint64_t n16, uint32_t* out) {
  // 4 independent 16-B loads per lane per iteration, 64 KiB per workgroup-iteration
  uint32_t acc = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 4;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x * 4 + threadIdx.x; i < n16; i += stride) {
    u32x4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      g_u32x4* q = (g_u32x4*)p + i + j * blockDim.x;
      v[j] = NT ? __builtin_nontemporal_load(q) : *q;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int G, int U, bool NT = false>
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
      for (int j = 0; j < U; ++j) v[j] = NT ? __builtin_nontemporal_load(q + (r + j) * G) : q[(r + j) * G];
#pragma unroll
      for (int j = 0; j < U; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// G lanes per 4 KiB block, each lane owning 32 contiguous bytes of a 32*G-byte
// row (two 16-B loads at +0 and +16), U rows per batch, nt
template <int G, int U>
__global__ __launch_bounds__(1024) void probe_pairs(const u32x4* __restrict__ p, uint64_t nblocks, uint32_t blk16, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t gid = ((uint64_t)blockIdx.x * 16 + wave) * (64 / G) + lane / G;
  const uint64_t gstride = (uint64_t)gridDim.x * 16 * (64 / G);
  uint32_t acc = 0;
  for (uint64_t b = gid; b < nblocks; b += gstride) {
    const g_u32x4* q = (g_u32x4*)p + b * blk16 + 2 * (lane % G);
    for (uint32_t r = 0; r < blk16 / (2 * G); r += U) {
      u32x4 v[U][2];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        v[j][0] = __builtin_nontemporal_load(q + (r + j) * 2 * G);
        v[j][1] = __builtin_nontemporal_load(q + (r + j) * 2 * G + 1);
      }
#pragma unroll
      for (int j = 0; j < U; ++j) acc ^= v[j][0].x ^ v[j][0].y ^ v[j][0].z ^ v[j][0].w ^ v[j][1].x ^ v[j][1].w;
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
    for (int it = 0; it < 100; ++it) {
      hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b); if (it >= 60) ts.push_back(ms);
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
  for (int wgs : {cus, 2 * cus, 4 * cus}) {
    char nm[64]; snprintf(nm, 64, "stream4 nt wg=%d x1024", wgs);
    run(nm, [&] { hipLaunchKernelGGL(probe_stream_u<true>, dim3(wgs), dim3(1024), 0, 0, d, bytes / 16, o); });
    snprintf(nm, 64, "stream4 rt wg=%d x1024", wgs);
    run(nm, [&] { hipLaunchKernelGGL(probe_stream_u<false>, dim3(wgs), dim3(1024), 0, 0, d, bytes / 16, o); });
  }
  run("groups nt G=16 U=4 4KiB wg=cus", [&] { hipLaunchKernelGGL((probe_groups<16,4,true>), dim3(cus), dim3(1024), 0, 0, d, nb, 256u, o); });
  run("groups nt G=16 U=8 4KiB wg=cus", [&] { hipLaunchKernelGGL((probe_groups<16,8,true>), dim3(cus), dim3(1024), 0, 0, d, nb, 256u, o); });
  run("groups nt G=64 U=4 4KiB wg=cus", [&] { hipLaunchKernelGGL((probe_groups<64,4,true>), dim3(cus), dim3(1024), 0, 0, d, nb, 256u, o); });
  run("groups nt G=16 U=4 4KiB wg=2cus", [&] { hipLaunchKernelGGL((probe_groups<16,4,true>), dim3(2*cus), dim3(1024), 0, 0, d, nb, 256u, o); });
  // rows not 128-B aligned (the offsets API's end-aligned rows of byte-packed buffers)
  for (int sh : {16, 48, 64, 112}) {
    char nm[64]; snprintf(nm, 64, "groups nt G=16 U=4 4KiB +%dB", sh);
    run(nm, [&] { hipLaunchKernelGGL((probe_groups<16,4,true>), dim3(cus), dim3(1024), 0, 0, d + sh / 16, nb - 1, 256u, o); });
  }
  run("groups nt G=8 U=4 4KiB wg=cus", [&] { hipLaunchKernelGGL((probe_groups<8,4,true>), dim3(cus), dim3(1024), 0, 0, d, nb, 256u, o); });
  run("groups nt G=4 U=4 4KiB wg=cus", [&] { hipLaunchKernelGGL((probe_groups<4,4,true>), dim3(cus), dim3(1024), 0, 0, d, nb, 256u, o); });
  run("pairs nt G=16 U=2 4KiB wg=cus", [&] { hipLaunchKernelGGL((probe_pairs<16,2>), dim3(cus), dim3(1024), 0, 0, d, nb, 256u, o); });
  run("pairs nt G=16 U=4 4KiB wg=cus", [&] { hipLaunchKernelGGL((probe_pairs<16,4>), dim3(cus), dim3(1024), 0, 0, d, nb, 256u, o); });
  run("pairs nt G=8 U=4 4KiB wg=cus", [&] { hipLaunchKernelGGL((probe_pairs<8,4>), dim3(cus), dim3(1024), 0, 0, d, nb, 256u, o); });
  run("pairs nt G=32 U=2 4KiB wg=cus", [&] { hipLaunchKernelGGL((probe_pairs<32,2>), dim3(cus), dim3(1024), 0, 0, d, nb, 256u, o); });
  return 0;
}
