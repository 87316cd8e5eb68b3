// Launch-overhead probe: HIP-event time per launch of back-to-back kernels on
// one stream that do no work -- (a) an empty 256 x 1024-thread grid, (b) the
// same with the class kernel's 160 KiB of static LDS, (c) a grid that reads a
// device flag and exits (the shape of an early-exiting persistent kernel),
// (d) (c) with 1024 workgroups of 256 threads (the sort passes' shape).
// Tells what a kernel that early-exits on a device-side decision costs.
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
    printf("}}\n");
    return 0;
}
