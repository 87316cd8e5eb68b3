// Multi-GPU host batch (SURVEY 8b `lv_crc32c_batch_multi`, 8e): buffers are
// independent, so the batch is split into contiguous buffer ranges balanced
// by payload bytes (prefix sum of lengths), one range per device and one host
// thread per device; each device receives only its range's buffers and
// metadata and writes back its slice of out[].  No collective, no peer
// traffic.
//
// What "its range's buffers" costs on the bus depends on where they lie.
// Byte-packed buffers in index order (a log, a table file) occupy one span
// about the size of their payload, which ships as is.  Buffers listed in any
// other order (shuffled offsets, a gather over a large arena) can spread a
// range over the whole arena: shipping the span [min off, max end) would send
// every device ~the whole arena.  When the span exceeds kPackRatio x the
// range's payload (plus kPackSlack), the range's buffers are packed into a
// contiguous host copy first, in index order, so the device receives its
// payload and nothing else.  The pack goes straight into page-locked memory,
// which the host upload DMAs as is: one host copy of the payload, the copy
// the pageable upload's staging pass would have made (round 3 packed into
// pageable memory, which the upload then staged again: two copies).  It is
// done in chunks of kPackChunk bytes so the copy never holds a range's whole
// payload; a chunk's pack is not overlapped with the previous chunk's upload.
// The page-locked pack buffer is cached per device for the process's life
// (round 5, ADVICE r04: pinning up to kPackChunk per call cost a
// hipHostMalloc and an implicitly synchronising hipHostFree every time).
#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lvgpu/crc32c.h"
#include "lv_internal.h"

namespace {

// Buffer-range boundaries b[0..k]: range r holds ~ total*r/k payload bytes.
std::vector<size_t> byte_balanced(const uint32_t *len, size_t n, int k) {
    std::vector<uint64_t> pre(n + 1, 0);
    for (size_t i = 0; i < n; ++i) pre[i + 1] = pre[i] + len[i];
    std::vector<size_t> b(k + 1, n);
    b[0] = 0;
    for (int r = 1; r < k; ++r) {
        const uint64_t target = pre[n] / k * r + (pre[n] % k) * r / k;
        b[r] = static_cast<size_t>(std::lower_bound(pre.begin(), pre.end(), target) - pre.begin());
        b[r] = std::max(b[r], b[r - 1]);
    }
    return b;
}

struct Shard {
    int rc = LV_OK;
    std::string err;
};

constexpr double kPackRatio = 1.5;
constexpr uint64_t kPackSlack = 1ull << 20;
constexpr uint64_t kPackChunk = 256ull << 20;

// Page-locked pack buffer of one device, grown on demand and kept (never
// freed: a static destructor would run after the HIP runtime's teardown).
struct Pinned {
    std::mutex m;  // one packed range at a time per device
    uint8_t *p = nullptr;
    size_t cap = 0;
    int reserve(size_t bytes, int device) {
        if (cap >= bytes) return LV_OK;
        lvgpu_internal::pinned_free(p);
        p = nullptr;
        cap = 0;
        if (int rc = lvgpu_internal::pinned_alloc(bytes, &p)) return rc;
        lvgpu_internal::count_alloc(device);
        cap = bytes;
        return LV_OK;
    }
};

// Ships a scattered range in sub-ranges of at most kPackChunk payload bytes
// (a lone longer buffer is its own sub-range and ships from the arena as
// is), each packed into one reused page-locked buffer: host memory stays
// bounded by the chunk however large the range's payload is.
Pinned &pack_buffer(int device) {
    static Pinned *bufs = new Pinned[64];  // lv_crc32c_batch_multi_devices checks 0 <= device < 64
    return bufs[device];
}

int packed_ranges(const uint8_t *arena, const uint64_t *off, const uint32_t *len, const uint32_t *seed,
                  uint32_t *out, size_t cnt, uint32_t flags, int device) {
    Pinned &packed = pack_buffer(device);
    std::lock_guard<std::mutex> lk(packed.m);
    std::vector<uint64_t> poff;
    for (size_t lo = 0; lo < cnt;) {
        if (len[lo] >= kPackChunk) {
            const uint64_t zero = 0;
            const int rc = lv_crc32c_batch_host(arena + off[lo], len[lo], &zero, len + lo, seed ? seed + lo : nullptr,
                                                out + lo, 1, flags, device);
            if (rc) return rc;
            ++lo;
            continue;
        }
        size_t hi = lo;
        uint64_t bytes = 0;
        while (hi < cnt && len[hi] < kPackChunk && bytes + len[hi] <= kPackChunk) bytes += len[hi++];
        if (int rc = packed.reserve(bytes ? bytes : 1, device)) return rc;  // non-null even for all-empty buffers
        poff.resize(hi - lo);
        uint64_t pos = 0;
        for (size_t k = lo; k < hi; ++k) {
            std::memcpy(packed.p + pos, arena + off[k], len[k]);
            poff[k - lo] = pos;
            pos += len[k];
        }
        const int rc = lv_crc32c_batch_host(packed.p, bytes, poff.data(), len + lo, seed ? seed + lo : nullptr,
                                            out + lo, hi - lo, flags, device);
        if (rc) return rc;
        lo = hi;
    }
    return LV_OK;
}

}  // namespace

extern "C" {

int lv_crc32c_batch_multi_devices(const uint8_t *h_arena, size_t arena_bytes, const uint64_t *h_off,
                                  const uint32_t *h_len, const uint32_t *h_seed, uint32_t *h_out, size_t n,
                                  uint32_t flags, const int *devices, int ndev) {
    lvgpu_internal::clear_error();
    if (n == 0) return LV_OK;
    if (!h_arena || !h_off || !h_len || !h_out) return lvgpu_internal::set_error(LV_ERR_INVALID, "null host pointer");
    if (!devices || ndev <= 0) return lvgpu_internal::set_error(LV_ERR_INVALID, "no devices");
    for (int r = 0; r < ndev; ++r)
        if (devices[r] < 0 || devices[r] >= 64) return lvgpu_internal::set_error(LV_ERR_INVALID, "device out of range");
    for (size_t i = 0; i < n; ++i)
        if (h_off[i] > arena_bytes || h_len[i] > arena_bytes - h_off[i])
            return lvgpu_internal::set_error(LV_ERR_INVALID, "buffer outside arena");
    const std::vector<size_t> b = byte_balanced(h_len, n, ndev);
    std::vector<Shard> res(ndev);
    std::vector<std::thread> th;
    for (int r = 0; r < ndev; ++r) {
        if (b[r] == b[r + 1]) continue;
        th.emplace_back([&, r] {
            const size_t lo = b[r], cnt = b[r + 1] - b[r];
            uint64_t first = UINT64_MAX, last = 0, payload = 0;
            for (size_t i = lo; i < lo + cnt; ++i) {
                first = std::min(first, h_off[i]);
                last = std::max(last, h_off[i] + h_len[i]);
                payload += h_len[i];
            }
            const uint32_t *seed = h_seed ? h_seed + lo : nullptr;
            if (static_cast<double>(last - first) <= kPackRatio * static_cast<double>(payload) + kPackSlack) {
                std::vector<uint64_t> off(h_off + lo, h_off + lo + cnt);
                for (auto &o : off) o -= first;  // this device's span starts at `first`
                res[r].rc = lv_crc32c_batch_host(h_arena + first, last - first, off.data(), h_len + lo, seed,
                                                 h_out + lo, cnt, flags, devices[r]);
            } else {
                res[r].rc = packed_ranges(h_arena, h_off + lo, h_len + lo, seed, h_out + lo, cnt, flags, devices[r]);
            }
            if (res[r].rc) res[r].err = lv_last_error();
        });
    }
    for (auto &t : th) t.join();
    for (int r = 0; r < ndev; ++r)
        if (res[r].rc)
            return lvgpu_internal::set_error(res[r].rc, ("device " + std::to_string(devices[r]) + ": " + res[r].err).c_str());
    return LV_OK;
}

int lv_crc32c_batch_multi(const uint8_t *h_arena, size_t arena_bytes, const uint64_t *h_off, const uint32_t *h_len,
                          const uint32_t *h_seed, uint32_t *h_out, size_t n, uint32_t flags, int ngpu) {
    if (ngpu <= 0 || ngpu > 64) return lvgpu_internal::set_error(LV_ERR_INVALID, "ngpu must be in 1..64");
    std::vector<int> dev(ngpu);
    for (int i = 0; i < ngpu; ++i) dev[i] = i;
    return lv_crc32c_batch_multi_devices(h_arena, arena_bytes, h_off, h_len, h_seed, h_out, n, flags, dev.data(),
                                         ngpu);
}

}  // extern "C"
