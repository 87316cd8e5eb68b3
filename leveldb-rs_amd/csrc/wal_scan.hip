// Host-memory WAL scan (the reader side of SURVEY 8f row 1): upload, then
// the device scan lv_wal_scan_device (crc32c_batch.hip: each 32 KiB block's
// header chain is walked inside the length sort's passes, as
// Reader::read_physical_record frames it, log_reader.rs:271-331, and every
// [type || payload] unit is checksummed), then the arrays come back.
// Headers past a checksum mismatch in the same block are also emitted: the
// host reader never consults them (it drops the rest of the block,
// log_reader.rs:337-342).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "../../include/lvgpu/crc32c.h"
#include "../../include/lvgpu/wal.h"
#include "lv_internal.h"

namespace {

constexpr size_t align16(size_t x) { return (x + 15) & ~static_cast<size_t>(15); }

int hip_err(hipError_t e, const char *what) {
    if (e == hipSuccess) return LV_OK;
    return lvgpu_internal::set_error(static_cast<int>(e), (std::string(what) + ": " + hipGetErrorString(e)).c_str());
}

}  // namespace

// The log goes to the device through the device's host path (cached arena;
// pinned input: one DMA, pageable: pipelined pinned staging); the scan is
// lv_wal_scan_device (framing fused into the length sort, four launches)
// into the device's cached scratch buffer, so a scan allocates nothing on the
// device after the first call.  The capacity starts at a guess (one record per
// 256 log bytes, at least 8 per block); a log with more records is scanned
// again at its exact count.
extern "C" lv_wal_scan *lv_wal_scan_host(const uint8_t *log, size_t bytes, int device) {
    if (!log && bytes) {
        lvgpu_internal::set_error(LV_ERR_INVALID, "null log");
        return nullptr;
    }
    lv_wal_scan *scan = new lv_wal_scan();
    const uint64_t nblocks = (bytes + LV_WAL_BLOCK_SIZE - 1) / LV_WAL_BLOCK_SIZE;
    if (nblocks == 0) return scan;
    lvgpu_internal::HostPath hp;
    if (lvgpu_internal::host_upload(device, log, bytes, 16, &hp)) {
        delete scan;
        return nullptr;
    }
    hipStream_t s = static_cast<hipStream_t>(hp.stream);
    uint64_t cap = std::max<uint64_t>(bytes / 256, nblocks * 8), count = 0;
    for (int attempt = 0; attempt < 2; ++attempt) {
        const size_t wsb = align16(lv_wal_scan_workspace_bytes(bytes, cap));
        const size_t need = wsb + align16(cap * 8) + 2 * align16(cap * 4) + 16;
        uint8_t *scr = nullptr;
        if (lvgpu_internal::host_scratch(&hp, 0, need, &scr)) break;
        uint64_t *d_hdr = reinterpret_cast<uint64_t *>(scr + wsb);
        uint32_t *d_crc = reinterpret_cast<uint32_t *>(scr + wsb + align16(cap * 8));
        uint32_t *d_info = reinterpret_cast<uint32_t *>(scr + wsb + align16(cap * 8) + align16(cap * 4));
        uint64_t *d_count = reinterpret_cast<uint64_t *>(scr + need - 16);
        if (lv_wal_scan_device(hp.d_arena, bytes, d_hdr, d_crc, d_info, cap, d_count, scr, wsb, s)) break;
        if (hip_err(hipMemcpyAsync(&count, d_count, 8, hipMemcpyDeviceToHost, s), "D2H") ||
            hip_err(hipStreamSynchronize(s), "sync"))
            break;
        if (count > cap) {  // more records than the guess: once more at the exact count
            cap = count;
            continue;
        }
        lvgpu_internal::count_d2h(8 + count * 16);
        scan->off.resize(count);
        scan->crc.resize(count);
        scan->info.resize(count);
        if (count &&
            (hip_err(hipMemcpyAsync(scan->off.data(), d_hdr, count * 8, hipMemcpyDeviceToHost, s), "D2H") ||
             hip_err(hipMemcpyAsync(scan->crc.data(), d_crc, count * 4, hipMemcpyDeviceToHost, s), "D2H") ||
             hip_err(hipMemcpyAsync(scan->info.data(), d_info, count * 4, hipMemcpyDeviceToHost, s), "D2H") ||
             hip_err(hipStreamSynchronize(s), "sync")))
            break;
        return scan;
    }
    (void)hipStreamSynchronize(s);
    if (!*lv_last_error()) lvgpu_internal::set_error(LV_ERR_INVALID, "WAL scan failed");
    delete scan;
    return nullptr;
}
