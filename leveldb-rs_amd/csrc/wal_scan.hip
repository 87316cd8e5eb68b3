// GPU framing of a write-ahead log (the reader side of SURVEY 8f row 1).
//
// Every 32 KiB block is independent: records never straddle blocks
// (log_writer.rs:67-80 pads a block tail < HEADER_SIZE with zeros and starts
// a new block).  One thread walks one block's header chain exactly as
// Reader::read_physical_record does (log_reader.rs:271-331): stop when fewer
// than HEADER_SIZE bytes remain, at a length that overruns the block ("bad
// record length") or at a ZERO/0 header (the reader clears the buffer).  Two
// passes (count, then emit after an exclusive scan of the per-block counts)
// produce the records in log order; the CRC of every [type || payload] unit
// is then one lv_crc32c_batch_device call.  Headers past a checksum mismatch
// in the same block are also emitted: the host reader never consults them
// (it drops the rest of the block, log_reader.rs:337-342).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstring>
#include <initializer_list>
#include <string>

#include "../../include/lvgpu/crc32c.h"
#include "../../include/lvgpu/wal.h"
#include "lv_internal.h"

namespace lvw {

constexpr uint32_t kBlock = LV_WAL_BLOCK_SIZE;
constexpr uint32_t kHeader = LV_WAL_HEADER_SIZE;

// 8 bytes of the log starting at byte pos (log 8-B aligned, 16 B of padding
// after its end): two aligned loads and a funnel shift.
__device__ __forceinline__ uint64_t load8(const uint8_t *log, uint64_t pos) {
    const uint64_t *p = reinterpret_cast<const uint64_t *>(log + (pos & ~7ull));
    const uint32_t sh = static_cast<uint32_t>(pos & 7u) * 8u;
    const uint64_t lo = p[0];
    return sh ? (lo >> sh) | (p[1] << (64u - sh)) : lo;
}

template <bool EMIT>
__global__ void frame_blocks(const uint8_t *__restrict__ log, uint64_t size, uint64_t nblocks,
                             uint32_t *__restrict__ counts, const uint32_t *__restrict__ first,
                             uint64_t *__restrict__ hdr_off, uint64_t *__restrict__ unit_off,
                             uint32_t *__restrict__ unit_len, uint32_t *__restrict__ info) {
    const uint64_t b = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (b >= nblocks) return;
    const uint64_t start = b * kBlock;
    const uint32_t blen = static_cast<uint32_t>(size - start < kBlock ? size - start : kBlock);
    uint32_t pos = 0, k = 0;
    const uint32_t o = EMIT ? first[b] : 0u;
    while (blen - pos >= kHeader) {
        const uint64_t h = load8(log, start + pos);     // crc(4) | length(2) | type(1)
        const uint32_t len = static_cast<uint32_t>(h >> 32) & 0xffffu;
        const uint32_t t = static_cast<uint32_t>(h >> 48) & 0xffu;
        uint32_t status = LV_WAL_REC_OK;
        if (kHeader + len > blen - pos)
            status = LV_WAL_REC_BAD_LENGTH;             // log_reader.rs:312-324
        else if (t == 0 && len == 0)
            status = LV_WAL_REC_ZERO;                   // log_reader.rs:326-331
        if (EMIT) {
            hdr_off[o + k] = start + pos;
            unit_off[o + k] = start + pos + 6;          // [type || payload], log_reader.rs:336
            unit_len[o + k] = status == LV_WAL_REC_OK ? len + 1 : 0u;
            info[o + k] = t | (status << 8) | (len << 16);
        }
        ++k;
        if (status != LV_WAL_REC_OK) break;
        pos += kHeader + len;
    }
    if (!EMIT) counts[b] = k;
}

}  // namespace lvw

namespace {

#define WAL_HIP(call)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess) {                                                            \
            lvgpu_internal::set_error(static_cast<int>(e_),                                \
                                      (std::string(#call) + ": " + hipGetErrorString(e_)).c_str()); \
            goto fail;                                                                     \
        }                                                                                  \
    } while (0)

constexpr size_t align16(size_t x) { return (x + 15) & ~static_cast<size_t>(15); }

}  // namespace

// The log goes to the device through the device's host path (cached arena;
// pinned input: one DMA, pageable: pipelined pinned staging) and every device
// array comes from its cached scratch buffers, so a scan allocates nothing on
// the device after the first call.
extern "C" lv_wal_scan *lv_wal_scan_host(const uint8_t *log, size_t bytes, int device) {
    lv_wal_scan *scan = new lv_wal_scan();
    lvgpu_internal::HostPath hp;
    hipStream_t s = nullptr;
    uint8_t *d_log = nullptr, *scr0 = nullptr, *scr1 = nullptr, *d_tmp = nullptr;
    uint32_t *d_counts = nullptr, *d_first = nullptr, *d_len = nullptr, *d_info = nullptr, *d_crc = nullptr;
    uint64_t *d_hdr = nullptr, *d_unit = nullptr;
    size_t tmp_bytes = 0;
    uint32_t last_first = 0, last_count = 0, total = 0;
    const uint64_t nblocks = (bytes + lvw::kBlock - 1) / lvw::kBlock;
    if (!log && bytes) {
        lvgpu_internal::set_error(LV_ERR_INVALID, "null log");
        delete scan;
        return nullptr;
    }
    if (nblocks == 0) return scan;
    if (nblocks > 0xffffffffull / 4681) {
        lvgpu_internal::set_error(LV_ERR_INVALID, "log too large for one scan");
        delete scan;
        return nullptr;
    }
    if (lvgpu_internal::host_upload(device, log, bytes, 16, &hp)) goto fail;  // 16 zero bytes: load8's 2nd word
    s = static_cast<hipStream_t>(hp.stream);
    d_log = hp.d_arena;
    WAL_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, d_counts, d_first, nblocks, s));
    if (lvgpu_internal::host_scratch(&hp, 0, align16(nblocks * 4) * 2 + tmp_bytes, &scr0)) goto fail;
    d_counts = reinterpret_cast<uint32_t *>(scr0);
    d_first = reinterpret_cast<uint32_t *>(scr0 + align16(nblocks * 4));
    d_tmp = scr0 + 2 * align16(nblocks * 4);
    {
        const uint32_t grid = static_cast<uint32_t>((nblocks + 255) / 256);
        hipLaunchKernelGGL(lvw::frame_blocks<false>, dim3(grid), dim3(256), 0, s, d_log, bytes, nblocks, d_counts,
                           nullptr, nullptr, nullptr, nullptr, nullptr);
        WAL_HIP(hipGetLastError());
        WAL_HIP(hipcub::DeviceScan::ExclusiveSum(d_tmp, tmp_bytes, d_counts, d_first, nblocks, s));
        WAL_HIP(hipMemcpyAsync(&last_first, d_first + nblocks - 1, 4, hipMemcpyDeviceToHost, s));
        WAL_HIP(hipMemcpyAsync(&last_count, d_counts + nblocks - 1, 4, hipMemcpyDeviceToHost, s));
        WAL_HIP(hipStreamSynchronize(s));
        total = last_first + last_count;
        if (total) {
            const size_t t8 = align16(total * 8ull), t4 = align16(total * 4ull);
            if (lvgpu_internal::host_scratch(&hp, 1, 2 * t8 + 3 * t4, &scr1)) goto fail;
            d_hdr = reinterpret_cast<uint64_t *>(scr1);
            d_unit = reinterpret_cast<uint64_t *>(scr1 + t8);
            d_len = reinterpret_cast<uint32_t *>(scr1 + 2 * t8);
            d_info = reinterpret_cast<uint32_t *>(scr1 + 2 * t8 + t4);
            d_crc = reinterpret_cast<uint32_t *>(scr1 + 2 * t8 + 2 * t4);
            hipLaunchKernelGGL(lvw::frame_blocks<true>, dim3(grid), dim3(256), 0, s, d_log, bytes, nblocks, nullptr,
                               d_first, d_hdr, d_unit, d_len, d_info);
            WAL_HIP(hipGetLastError());
            if (int rc = lv_crc32c_batch_device(d_log, d_unit, d_len, nullptr, d_crc, total, 0, s)) {
                (void)rc;  // error text already set
                goto fail;
            }
            scan->off.resize(total);
            scan->crc.resize(total);
            scan->info.resize(total);
            WAL_HIP(hipMemcpyAsync(scan->off.data(), d_hdr, total * 8ull, hipMemcpyDeviceToHost, s));
            WAL_HIP(hipMemcpyAsync(scan->crc.data(), d_crc, total * 4ull, hipMemcpyDeviceToHost, s));
            WAL_HIP(hipMemcpyAsync(scan->info.data(), d_info, total * 4ull, hipMemcpyDeviceToHost, s));
            WAL_HIP(hipStreamSynchronize(s));
        }
    }
    return scan;
fail:
    if (s) (void)hipStreamSynchronize(s);
    delete scan;
    return nullptr;
}
