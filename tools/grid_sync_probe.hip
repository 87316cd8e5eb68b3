// Cost of one grid-wide barrier in a persistent 1,024-thread grid (one
// workgroup per CU), against the kernel boundary it would replace: per
// launch, (a) a kernel that only writes one word per workgroup, (b) the same
// kernel followed by a second empty launch (the boundary), (c) one
// cooperative launch with a cooperative-groups grid.sync() between the two
// halves.  Events around 400 back-to-back launches after 100 of warmup.
//   hipcc --offload-arch=gfx950 -O3 -o tools/grid_sync_probe tools/grid_sync_probe.hip
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>

#include <cstdio>

namespace cg = cooperative_groups;

__global__ __launch_bounds__(1024) void half(unsigned *out) {
    __shared__ unsigned s[16384];  // ~64 KiB of LDS, as the join
    s[threadIdx.x] = blockIdx.x;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = s[threadIdx.x ^ 1] + 1;
}

__global__ __launch_bounds__(1024) void both(unsigned *out) {
    __shared__ unsigned s[16384];
    s[threadIdx.x] = blockIdx.x;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = s[threadIdx.x ^ 1] + 1;
    cg::this_grid().sync();
    if (threadIdx.x == 0) out[gridDim.x + blockIdx.x] = out[(blockIdx.x + 1) % gridDim.x] + 1;
}

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e = (x);                                                \
        if (e != hipSuccess) {                                             \
            printf("%s: %s\n", #x, hipGetErrorString(e));                  \
            return 1;                                                      \
        }                                                                  \
    } while (0)

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int g = p.multiProcessorCount;
    unsigned *out;
    CK(hipMalloc(&out, 2 * g * sizeof(unsigned)));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](int mode, int n) -> float {
        for (int i = 0; i < n; ++i) {
            if (mode == 0) {
                hipLaunchKernelGGL(half, dim3(g), dim3(1024), 0, 0, out);
            } else if (mode == 1) {
                hipLaunchKernelGGL(half, dim3(g), dim3(1024), 0, 0, out);
                hipLaunchKernelGGL(half, dim3(g), dim3(1024), 0, 0, out + g);
            } else {
                void *args[] = {&out};
                if (hipLaunchCooperativeKernel(reinterpret_cast<void *>(both), dim3(g), dim3(1024), args, 0, 0) !=
                    hipSuccess)
                    return -1.f;
            }
        }
        return 0.f;
    };
    const char *names[] = {"one launch", "two launches (boundary)", "cooperative + grid.sync"};
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 3; ++mode) {
            if (run(mode, 100) < 0) {
                printf("cooperative launch failed\n");
                return 1;
            }
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a, 0));
            run(mode, 400);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("%-28s %.2f us per call (%d workgroups)\n", names[mode], ms * 1e3f / 400, g);
        }
    unsigned h[4];
    CK(hipMemcpy(h, out + g, sizeof(h), hipMemcpyDeviceToHost));
    printf("check %u %u\n", h[0], h[1]);
    return 0;
}
