// Launch-overhead probe: HIP-event time per launch of back-to-back kernels on
// one stream that do no work -- (a) an empty 256 x 1024-thread grid, (b) the
// same with the class kernel's 160 KiB of static LDS, (c) a grid that reads a
// device flag and exits (the shape of an early-exiting persistent kernel),
// (d) (c) with 1024 workgroups of 256 threads (the sort passes' shape).
// Tells what a kernel that early-exits on a device-side decision costs.
// Round 6 (2nd): (e) the empty grid with 0-160 KiB of dynamic LDS, and (f) a
// streaming read of 256 MiB per launch (nt dwordx4, 256 x 1024 threads) with
// 0 / 64 / 160 KiB of LDS allocated: does the per-launch gap between
// back-to-back kernels grow with the LDS a workgroup holds?
// build: hipcc --offload-arch=gfx950 -O3 tools/launch_probe.hip -o tools/launch_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(1024) void k_empty() {}
__global__ __launch_bounds__(1024) void k_lds(uint32_t *out) {
    __shared__ uint32_t big[40960];  // 160 KiB
    if (threadIdx.x == 1 && out == nullptr) big[threadIdx.x] = 1;
    __syncthreads();
    if (out && threadIdx.x == 0 && big[5] == 12345u) out[0] = 1;
}
__global__ __launch_bounds__(1024) void k_flag(const uint32_t *flag, uint32_t *out) {
    if (*flag == 0) return;
    out[blockIdx.x * blockDim.x + threadIdx.x] = 1;
}
__global__ __launch_bounds__(256) void k_flag256(const uint32_t *flag, uint32_t *out) {
    if (*flag == 0) return;
    out[blockIdx.x * blockDim.x + threadIdx.x] = 1;
}

__global__ __launch_bounds__(1024) void k_dyn(uint32_t *out) {
    extern __shared__ uint32_t dyn[];
    if (threadIdx.x == 1 && out == nullptr) dyn[threadIdx.x] = 1;
    __syncthreads();
    if (out && threadIdx.x == 0 && dyn[5] == 12345u) out[0] = 1;
}
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(1024) void k_stream(const u32x4 *__restrict__ src, uint64_t n16, uint32_t *out) {
    extern __shared__ uint32_t dyn[];
    uint32_t x = 0;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n16; i += 4 * stride) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = __builtin_nontemporal_load(&src[i + k * stride < n16 ? i + k * stride : i]);
#pragma unroll
        for (int k = 0; k < 4; ++k) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    if (x == 0x12345678u) {
        dyn[threadIdx.x] = x;
        out[0] = dyn[(threadIdx.x + 1) & 1023];
    }
}

template <class F>
static float per_launch(hipStream_t s, int n, F f) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 50; ++i) f();
    (void)hipEventRecord(a, s);
    for (int i = 0; i < n; ++i) f();
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1000.f / n;
}

int main() {
    hipStream_t s;
    (void)hipStreamCreate(&s);
    uint32_t *flag, *out;
    (void)hipMalloc(&flag, 4);
    (void)hipMalloc(&out, 1 << 22);
    (void)hipMemset(flag, 0, 4);
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount, n = 2000;
    printf("{\"cus\": %d, \"us_per_launch\": {", cus);
    printf("\"empty_%dx1024\": %.3f, ", cus, per_launch(s, n, [&] { hipLaunchKernelGGL(k_empty, dim3(cus), dim3(1024), 0, s); }));
    printf("\"lds160k_%dx1024\": %.3f, ", cus, per_launch(s, n, [&] { hipLaunchKernelGGL(k_lds, dim3(cus), dim3(1024), 0, s, out); }));
    printf("\"flag_exit_%dx1024\": %.3f, ", cus, per_launch(s, n, [&] { hipLaunchKernelGGL(k_flag, dim3(cus), dim3(1024), 0, s, flag, out); }));
    printf("\"flag_exit_1024x256\": %.3f, ", per_launch(s, n, [&] { hipLaunchKernelGGL(k_flag256, dim3(1024), dim3(256), 0, s, flag, out); }));
    printf("\"flag_exit_16x1024\": %.3f", per_launch(s, n, [&] { hipLaunchKernelGGL(k_flag, dim3(16), dim3(1024), 0, s, flag, out); }));
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_dyn), hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_stream), hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    for (int kib : {0, 16, 32, 64, 80, 96, 128, 160}) {
        const size_t b = static_cast<size_t>(kib) << 10;
        printf(", \"dyn%dk_%dx1024\": %.3f", kib, cus,
               per_launch(s, n, [&] { hipLaunchKernelGGL(k_dyn, dim3(cus), dim3(1024), b, s, out); }));
    }
    printf("}, \"stream_256MiB_us_per_launch\": {");
    const uint64_t bytes = 256ull << 20;
    u32x4 *src = nullptr;
    (void)hipMalloc(&src, bytes);
    (void)hipMemset(src, 1, bytes);
    bool first = true;
    for (int rep = 0; rep < 2; ++rep)
        for (int kib : {0, 64, 160}) {
            const size_t b = static_cast<size_t>(kib) << 10;
            printf("%s\"lds%dk_r%d\": %.3f", first ? "" : ", ", kib, rep,
                   per_launch(s, 400, [&] { hipLaunchKernelGGL(k_stream, dim3(cus), dim3(1024), b, s, src, bytes / 16, out); }));
            first = false;
        }
    printf("}}\n");
    (void)hipFree(src);
    return 0;
}
