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

// the same with the hash chain's 32-bit multiply (v_mul_lo_u32)
__global__ void __launch_bounds__(256) mul_calib(uint32_t *out, uint32_t seed) {
    uint32_t x = seed + threadIdx.x, y = blockIdx.x | 1u;
    for (int i = 0; i < kIters; ++i) {
        asm volatile(
            "v_mul_lo_u32 %0, %0, %1\n v_mul_lo_u32 %0, %0, %1\n v_mul_lo_u32 %0, %0, %1\n v_mul_lo_u32 %0, %0, %1\n"
            "v_mul_lo_u32 %0, %0, %1\n v_mul_lo_u32 %0, %0, %1\n v_mul_lo_u32 %0, %0, %1\n v_mul_lo_u32 %0, %0, %1\n"
            "v_mul_lo_u32 %0, %0, %1\n v_mul_lo_u32 %0, %0, %1\n v_mul_lo_u32 %0, %0, %1\n v_mul_lo_u32 %0, %0, %1\n"
            "v_mul_lo_u32 %0, %0, %1\n v_mul_lo_u32 %0, %0, %1\n v_mul_lo_u32 %0, %0, %1\n v_mul_lo_u32 %0, %0, %1\n"
            : "+v"(x)
            : "v"(y));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <typename K>
static float time_kernel(K kern, uint32_t *d, int blocks, int threads) {
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, 2u);
    (void)hipEventRecord(b, 0);
    if (hipEventSynchronize(b) != hipSuccess) return -1.0f;
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    const int blocks = 2048, threads = 256;
    uint32_t *d = nullptr;
    if (hipMalloc(&d, sizeof(uint32_t) * blocks * threads) != hipSuccess) return 1;
    const double waves = double(blocks) * threads / 64, instr = waves * 16 * kIters;
    const float ms_add = time_kernel(valu_calib, d, blocks, threads), ms_mul = time_kernel(mul_calib, d, blocks, threads);
    // SIMD cycles per wave-level instruction at 2.4 GHz on 1,024 SIMDs (8 waves per SIMD, dependent chains)
    printf("{\"waves\": %.0f, \"instr_per_kernel\": %.0f, \"ms_v_add_u32\": %.4f, \"ms_v_mul_lo_u32\": %.4f, "
           "\"cycles_per_instr_add_at_2.4GHz\": %.3f, \"cycles_per_instr_mul_at_2.4GHz\": %.3f}\n",
           waves, instr, ms_add, ms_mul, ms_add * 1e-3 * 2.4e9 * 1024 / instr, ms_mul * 1e-3 * 2.4e9 * 1024 / instr);
    hipFree(d);
    return 0;
}
