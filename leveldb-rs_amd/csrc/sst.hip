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

// The file goes to the device through the device's host path (cached arena;
// pinned input: one DMA, pageable: pipelined pinned staging), the handles and
// the status words through its cached scratch buffer, as lv_wal_scan_host
// does: after the first call of a given size nothing is allocated on the
// device.
int lv_sst_verify_blocks_host(const uint8_t *file, uint64_t file_bytes, const uint64_t *handles, size_t n,
                              uint32_t *status, int device) {
    lvgpu_internal::clear_error();
    if (n == 0) return LV_OK;
    if ((!file && file_bytes) || !handles || !status)
        return lvgpu_internal::set_error(LV_ERR_INVALID, "null host pointer");
    if (n > 0xffffffffull) return lvgpu_internal::set_error(LV_ERR_INVALID, "more than 2^32-1 blocks per call");
    lvgpu_internal::HostPath hp;
    if (int rc = lvgpu_internal::host_upload(device, file, file_bytes, 16, &hp)) return rc;
    hipStream_t s = static_cast<hipStream_t>(hp.stream);
    const size_t hbytes = n * 16, sbytes = (n * 4 + 15) & ~static_cast<size_t>(15);
    uint8_t *scr = nullptr;
    if (int rc = lvgpu_internal::host_scratch(&hp, 0, hbytes + sbytes, &scr)) return rc;
    uint64_t *d_h = reinterpret_cast<uint64_t *>(scr);
    uint32_t *d_st = reinterpret_cast<uint32_t *>(scr + hbytes);
    auto hip = [&](hipError_t e, const char *what) {
        if (e == hipSuccess) return LV_OK;
        (void)hipStreamSynchronize(s);
        return lvgpu_internal::set_error(static_cast<int>(e), (std::string(what) + ": " + hipGetErrorString(e)).c_str());
    };
    if (int rc = hip(hipMemcpyAsync(d_h, handles, hbytes, hipMemcpyHostToDevice, s), "H2D")) return rc;
    lvgpu_internal::count_h2d(hbytes);
    if (int rc = lv_sst_verify_blocks_device(hp.d_arena, file_bytes, d_h, n, d_st, nullptr, s)) {
        (void)hipStreamSynchronize(s);
        return rc;
    }
    if (int rc = hip(hipMemcpyAsync(status, d_st, n * 4, hipMemcpyDeviceToHost, s), "D2H")) return rc;
    lvgpu_internal::count_d2h(n * 4);
    return hip(hipStreamSynchronize(s), "sync");
}

}  // extern "C"
