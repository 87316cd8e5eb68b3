// SSTable block trailers on MI355X: seal (builder side)
// and verify (ReadOptions::verify_checksums, options.rs:84) of many blocks
// at once.  Each block's CRC unit is contents||type, contiguous in the file,
// so the checksums are one lv_crc32c_batch_device call over (offset, size+1)
// units; the kernels here only turn handles into units and compare/store the
// 4-byte trailers.  Trailer layout: see include/lvgpu/table.h.
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/lvgpu/crc32c.h"
#include "../../include/lvgpu/table.h"
#include "lv_internal.h"

namespace lvs {

constexpr uint32_t kMaskDelta = 0xa282ead8u;  // crc32c.rs:22

__device__ __forceinline__ uint32_t mask(uint32_t c) { return ((c >> 15) | (c << 17)) + kMaskDelta; }
__device__ __forceinline__ uint32_t unmask(uint32_t m) {
    const uint32_t r = m - kMaskDelta;
    return (r >> 17) | (r << 15);
}

__device__ __forceinline__ bool in_range(uint64_t o, uint64_t sz, uint64_t file_bytes) {
    return sz < 0xffffffffull && o <= file_bytes && sz <= file_bytes - o &&
           file_bytes - o - sz >= LV_SST_TRAILER_SIZE;
}

// Handles -> CRC units (offset, size+1); SEAL also writes the type byte.
template <bool SEAL>
__global__ void __launch_bounds__(256) units_kernel(uint8_t *file, uint64_t file_bytes,
                                                    const uint64_t *__restrict__ handles,
                                                    const uint8_t *__restrict__ types, uint32_t n,
                                                    uint64_t *__restrict__ uoff, uint32_t *__restrict__ ulen) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t o = handles[2ull * i], sz = handles[2ull * i + 1];
    const bool ok = in_range(o, sz, file_bytes);
    uoff[i] = ok ? o : 0;
    ulen[i] = ok ? static_cast<uint32_t>(sz + 1) : 0u;
    if (SEAL && ok) file[o + sz] = types ? types[i] : static_cast<uint8_t>(LV_SST_NO_COMPRESSION);
}

__global__ void __launch_bounds__(256) seal_kernel(uint8_t *file, const uint64_t *__restrict__ uoff,
                                                   const uint32_t *__restrict__ ulen,
                                                   const uint32_t *__restrict__ crc, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || ulen[i] == 0) return;
    const uint32_t m = mask(crc[i]);
    uint8_t *p = file + uoff[i] + ulen[i];  // offset + size + 1
    p[0] = m & 0xff;
    p[1] = (m >> 8) & 0xff;
    p[2] = (m >> 16) & 0xff;
    p[3] = m >> 24;
}

__global__ void __launch_bounds__(256) verify_kernel(const uint8_t *file, const uint64_t *__restrict__ uoff,
                                                     const uint32_t *__restrict__ ulen,
                                                     const uint32_t *__restrict__ crc, uint32_t n,
                                                     uint32_t *__restrict__ status, uint32_t *__restrict__ crc_out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (ulen[i] == 0) {
        status[i] = LV_SST_BLOCK_OUT_OF_RANGE;
        if (crc_out) crc_out[i] = 0;
        return;
    }
    const uint8_t *p = file + uoff[i] + ulen[i];
    const uint32_t stored = p[0] | (p[1] << 8) | (p[2] << 16) | (static_cast<uint32_t>(p[3]) << 24);
    status[i] = unmask(stored) == crc[i] ? LV_SST_BLOCK_OK : LV_SST_BLOCK_CHECKSUM_MISMATCH;
    if (crc_out) crc_out[i] = crc[i];
}

// Unit arrays for n blocks, stream-ordered allocation.
struct Units {
    uint64_t *off = nullptr;
    uint32_t *len = nullptr, *crc = nullptr;
    void *raw = nullptr;
};

int alloc_units(size_t n, hipStream_t s, Units *u) {
    hipError_t e = hipMallocAsync(&u->raw, n * 16, s);
    if (e != hipSuccess)
        return lvgpu_internal::set_error(static_cast<int>(e), (std::string("hipMallocAsync: ") + hipGetErrorString(e)).c_str());
    u->off = static_cast<uint64_t *>(u->raw);
    u->len = reinterpret_cast<uint32_t *>(u->off + n);
    u->crc = u->len + n;
    return LV_OK;
}

int free_units(Units *u, hipStream_t s, int rc) {
    if (u->raw) {
        hipError_t e = hipFreeAsync(u->raw, s);
        if (e != hipSuccess && rc == LV_OK)
            rc = lvgpu_internal::set_error(static_cast<int>(e), "hipFreeAsync failed");
    }
    return rc;
}

int check_args(const void *file, const uint64_t *handles, size_t n) {
    if (!file || !handles) return lvgpu_internal::set_error(LV_ERR_INVALID, "null device pointer");
    if (n > 0xffffffffull) return lvgpu_internal::set_error(LV_ERR_INVALID, "more than 2^32-1 blocks per call");
    return LV_OK;
}

}  // namespace lvs

extern "C" {

int lv_sst_seal_blocks_device(uint8_t *d_file, uint64_t file_bytes, const uint64_t *d_handles,
                              const uint8_t *d_types, size_t n, void *stream) {
    lvgpu_internal::clear_error();
    if (n == 0) return LV_OK;
    if (int rc = lvs::check_args(d_file, d_handles, n)) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    lvs::Units u;
    if (int rc = lvs::alloc_units(n, s, &u)) return rc;
    const uint32_t grid = static_cast<uint32_t>((n + 255) / 256), nn = static_cast<uint32_t>(n);
    hipLaunchKernelGGL(lvs::units_kernel<true>, dim3(grid), dim3(256), 0, s, d_file, file_bytes, d_handles, d_types,
                       nn, u.off, u.len);
    int rc = lvgpu_internal::launch_status();
    if (rc == LV_OK) rc = lv_crc32c_batch_device(d_file, u.off, u.len, nullptr, u.crc, n, 0, s);
    if (rc == LV_OK) {
        hipLaunchKernelGGL(lvs::seal_kernel, dim3(grid), dim3(256), 0, s, d_file, u.off, u.len, u.crc, nn);
        rc = lvgpu_internal::launch_status();
    }
    return lvs::free_units(&u, s, rc);
}

int lv_sst_verify_blocks_device(const uint8_t *d_file, uint64_t file_bytes, const uint64_t *d_handles, size_t n,
                                uint32_t *d_status, uint32_t *d_crc, void *stream) {
    lvgpu_internal::clear_error();
    if (n == 0) return LV_OK;
    if (int rc = lvs::check_args(d_file, d_handles, n)) return rc;
    if (!d_status) return lvgpu_internal::set_error(LV_ERR_INVALID, "null status pointer");
    hipStream_t s = static_cast<hipStream_t>(stream);
    lvs::Units u;
    if (int rc = lvs::alloc_units(n, s, &u)) return rc;
    const uint32_t grid = static_cast<uint32_t>((n + 255) / 256), nn = static_cast<uint32_t>(n);
    hipLaunchKernelGGL(lvs::units_kernel<false>, dim3(grid), dim3(256), 0, s, const_cast<uint8_t *>(d_file),
                       file_bytes, d_handles, nullptr, nn, u.off, u.len);
    int rc = lvgpu_internal::launch_status();
    if (rc == LV_OK) rc = lv_crc32c_batch_device(d_file, u.off, u.len, nullptr, u.crc, n, 0, s);
    if (rc == LV_OK) {
        hipLaunchKernelGGL(lvs::verify_kernel, dim3(grid), dim3(256), 0, s, d_file, u.off, u.len, u.crc, nn, d_status,
                           d_crc);
        rc = lvgpu_internal::launch_status();
    }
    return lvs::free_units(&u, s, rc);
}

int lv_sst_verify_blocks_host(const uint8_t *file, uint64_t file_bytes, const uint64_t *handles, size_t n,
                              uint32_t *status, int device) {
    lvgpu_internal::clear_error();
    if (n == 0) return LV_OK;
    if ((!file && file_bytes) || !handles || !status)
        return lvgpu_internal::set_error(LV_ERR_INVALID, "null host pointer");
    hipStream_t s = nullptr;
    uint8_t *d_file = nullptr;
    uint64_t *d_h = nullptr;
    uint32_t *d_st = nullptr;
    int rc = LV_OK;
    auto hip = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && rc == LV_OK)
            rc = lvgpu_internal::set_error(static_cast<int>(e), (std::string(what) + ": " + hipGetErrorString(e)).c_str());
        return rc == LV_OK;
    };
    lvgpu_internal::DeviceGuard dg;  // the caller's current device comes back on return
    if (int e = dg.set(device)) return e;
    if (hip(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "stream") &&
        hip(hipMalloc(&d_file, file_bytes + 16), "hipMalloc") && hip(hipMalloc(&d_h, n * 16), "hipMalloc") &&
        hip(hipMalloc(&d_st, n * 4), "hipMalloc") &&
        hip(hipMemcpyAsync(d_file, file, file_bytes, hipMemcpyHostToDevice, s), "H2D") &&
        hip(hipMemcpyAsync(d_h, handles, n * 16, hipMemcpyHostToDevice, s), "H2D")) {
        rc = lv_sst_verify_blocks_device(d_file, file_bytes, d_h, n, d_st, nullptr, s);
        if (rc == LV_OK) hip(hipMemcpyAsync(status, d_st, n * 4, hipMemcpyDeviceToHost, s), "D2H");
        if (rc == LV_OK) hip(hipStreamSynchronize(s), "sync");
    }
    if (s) (void)hipStreamSynchronize(s);
    for (void *p : {static_cast<void *>(d_file), static_cast<void *>(d_h), static_cast<void *>(d_st)})
        if (p) (void)hipFree(p);
    if (s) (void)hipStreamDestroy(s);
    return rc;
}

}  // extern "C"
