// Standalone probe (not product code): throughput of the Latin-square LDS
// lookup step (v_perm address + ds_read_b32 + xor) with no global memory.
// Reports lookups/clk/CU (using s_memtime cycles) and equivalent CRC GB/s at
// 1.25 lookups per byte.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

__shared__ __attribute__((aligned(16))) uint32_t lds[16384];

template <int CH, int ITERS>
__global__ void probe(uint32_t* out, uint64_t* cyc) {
  for (int i = threadIdx.x; i < 16384; i += blockDim.x) lds[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, g = lane & 31, c = g & 7, q = g >> 3;
  uint32_t lv = 0, sel[4];
  for (uint32_t i = 0; i < 4; ++i) { uint32_t k = (q + i) & 3; lv |= ((4*c+k)*4) << (8*i); sel[i] = 0x0C0C0000u | ((7-k) << 8) | i; }
  uint32_t s[CH];
  for (int j = 0; j < CH; ++j) s[j] = threadIdx.x * 7919u + j * 104729u + blockIdx.x;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; ++it) {
    uint32_t a[CH][4], t[CH][4];
#pragma unroll
    for (int j = 0; j < CH; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) a[j][k] = __builtin_amdgcn_perm(s[j], lv, sel[k]);
#pragma unroll
    for (int j = 0; j < CH; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) t[j][k] = lds[a[j][k] / 4];
#pragma unroll
    for (int j = 0; j < CH; ++j) s[j] = (t[j][0] ^ t[j][1]) ^ (t[j][2] ^ t[j][3]) ^ (uint32_t)it;
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t acc = 0;
  for (int j = 0; j < CH; ++j) acc ^= s[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CH>
void run(int threads, uint32_t* o, uint64_t* cy, int cus) {
  constexpr int ITERS = 2048;
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  std::vector<float> ts;
  for (int rep = 0; rep < 7; ++rep) {
    hipEventRecord(a);
    hipLaunchKernelGGL((probe<CH, ITERS>), dim3(cus), dim3(threads), 0, 0, o, cy);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  std::vector<uint64_t> h(cus);
  hipMemcpy(h.data(), cy, cus * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  double lookups = (double)cus * threads * ITERS * CH * 4;
  double per_cu_clk = (double)threads * ITERS * CH * 4 / (double)h[cus/2];
  printf("chains=%d waves/CU=%2d  %.3f ms  %.2f Tlookup/s  %.2f lookups/clk/CU(memtime)  => CRC %.0f GB/s at 1.25 lk/B\n",
         CH, threads / 64, ts[3], lookups / (ts[3] * 1e-3) / 1e12, per_cu_clk, lookups / 1.25 / (ts[3] * 1e-3) / 1e9);
}

int main() {
  int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* o; uint64_t* cy;
  hipMalloc(&o, cus * 1024 * 4); hipMalloc(&cy, cus * 8);
  for (int th : {256, 512, 1024}) { run<1>(th, o, cy, cus); run<2>(th, o, cy, cus); run<4>(th, o, cy, cus); run<8>(th, o, cy, cus); }
  return 0;
}
