// SSTable block trailers on MI355X: seal (builder side)
// and verify (ReadOptions::verify_checksums, options.rs:84) of many blocks
// at once.  Each block's CRC unit is contents||type, contiguous in the file;
// the kernel (one launch: handles -> CRC -> trailer epilogue) lives with the
// other CRC kernels in crc32c_batch.hip.  Trailer layout: see
// include/lvgpu/table.h.
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/lvgpu/crc32c.h"
#include "../../include/lvgpu/table.h"
#include "lv_internal.h"

namespace lvs {

int check_args(const void *file, const uint64_t *handles, size_t n) {
    if (!file || !handles) return lvgpu_internal::set_error(LV_ERR_INVALID, "null device pointer");
    if (n > 0xffffffffull) return lvgpu_internal::set_error(LV_ERR_INVALID, "more than 2^32-1 blocks per call");
    if (reinterpret_cast<uintptr_t>(handles) % 8) return lvgpu_internal::set_error(LV_ERR_INVALID, "handles must be 8-byte aligned");
    return LV_OK;
}

}  // namespace lvs

extern "C" {

// Both device entry points are ONE kernel launch (lvk::sst_blocks_kernel,
// crc32c_batch.hip): the handles are read in file order, the CRC walk is the
// offsets API's G = 16 aligned-row walk, and the trailer compare / write is
// its epilogue.
int lv_sst_seal_blocks_device(uint8_t *d_file, uint64_t file_bytes, const uint64_t *d_handles,
                              const uint8_t *d_types, size_t n, void *stream) {
    lvgpu_internal::clear_error();
    if (n == 0) return LV_OK;
    if (int rc = lvs::check_args(d_file, d_handles, n)) return rc;
    return lvgpu_internal::launch_sst_blocks(true, d_file, file_bytes, d_handles, d_types, n, nullptr, nullptr, stream);
}

int lv_sst_verify_blocks_device(const uint8_t *d_file, uint64_t file_bytes, const uint64_t *d_handles, size_t n,
                                uint32_t *d_status, uint32_t *d_crc, void *stream) {
    lvgpu_internal::clear_error();
    if (n == 0) return LV_OK;
    if (int rc = lvs::check_args(d_file, d_handles, n)) return rc;
    if (!d_status) return lvgpu_internal::set_error(LV_ERR_INVALID, "null status pointer");
    return lvgpu_internal::launch_sst_blocks(false, d_file, file_bytes, d_handles, nullptr, n, d_status, d_crc, stream);
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
