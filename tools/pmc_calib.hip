// PMC calibration (tools only): a kernel whose VALU / SALU instruction counts
// are known from its source, to read what SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU
// and SQ_BUSY_CYCLES count on this part (per wave instruction? sampled?)
// before pricing the hash kernel's VALU issue with them.
//   hipcc --offload-arch=gfx950 -O3 -o tools/pmc_calib tools/pmc_calib.hip
//   rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU ... -- tools/pmc_calib
// Each wave runs kIters iterations of 16 dependent v_add_u32 (inline asm)
// and the loop's scalar counter / compare / branch; it prints the expected
// totals for comparison.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 4096;

__global__ void __launch_bounds__(256) valu_calib(uint32_t *out, uint32_t seed) {
    uint32_t x = seed + threadIdx.x, y = blockIdx.x | 1u;
    for (int i = 0; i < kIters; ++i) {
        asm volatile(
            "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n"
            "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n"
            "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n"
            "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n"
            : "+v"(x)
            : "v"(y));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

int main() {
    const int blocks = 2048, threads = 256;
    uint32_t *d = nullptr;
    if (hipMalloc(&d, sizeof(uint32_t) * blocks * threads) != hipSuccess) return 1;
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(valu_calib, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a, 0);
    hipLaunchKernelGGL(valu_calib, dim3(blocks), dim3(threads), 0, 0, d, 2u);
    hipEventRecord(b, 0);
    if (hipEventSynchronize(b) != hipSuccess) return 1;
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double waves = double(blocks) * threads / 64;
    printf("{\"waves\": %.0f, \"valu_per_wave\": %d, \"valu_total\": %.0f, \"ms\": %.4f, "
           "\"valu_issue_frac_at_4cyc_2.4GHz_1024simd\": %.4f}\n",
           waves, 16 * kIters, waves * 16 * kIters, ms, waves * 16 * kIters * 4 / (1024 * 2.4e9 * ms * 1e-3));
    hipFree(d);
    return 0;
}
