// Per-device context of the product library and its host-memory paths:
// error plumbing, the LDS table images and GF(2) tables built once per device,
// the library-owned sort workspaces, piece matrices, the host-path staging
// (cached device arena, pinned staging slots) behind lv_crc32c_batch_host,
// lv_wal_scan_host and lv_sst_verify_blocks_host, the debug queries, and the
// synthetic payload generator.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <thread>

#include "../../include/lvgpu/crc32c.h"
#include "crc32c_gf2.h"
#include "lvh.h"

namespace lvk {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void fill_words_kernel(uint64_t *dst, uint64_t word0, uint64_t nwords, uint64_t seed) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nwords; i += gridDim.x * 256ull)
        dst[i] = splitmix64(seed ^ (word0 + i));
}

__global__ void fill_bytes_kernel(uint8_t *dst, uint64_t begin, uint64_t nbytes, uint64_t seed) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nbytes; i += gridDim.x * 256ull) {
        const uint64_t k = begin + i;
        dst[i] = static_cast<uint8_t>(splitmix64(seed ^ (k >> 3)) >> (8 * (k & 7)));
    }
}

}  // namespace lvk

namespace lvh {

thread_local std::string g_err;
thread_local const char *g_kernel = "";

int set_err(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

const std::vector<uint32_t> &host_image(int gi) {
    static std::vector<uint32_t> images[kImages];
    static std::once_flag once;
    std::call_once(once, [] {
        uint32_t T[4][256], C[6][4][256];
        lvgpu::slice_tables(T);
        for (int k = 0; k < 6; ++k) lvgpu::shift_tables(16ull << k, C[k]);
        for (int i = 0; i < 4; ++i) {
            const uint64_t G = static_cast<uint64_t>(kGs[i]);
            uint32_t W4[4][256], W1[4][256], W2[4][256];
            lvgpu::shift_tables(16ull * G * lvk::U, W4);
            lvgpu::shift_tables(16ull * G, W1);
            lvgpu::shift_tables(32ull * G, W2);
            std::vector<uint32_t> &im = images[i];
            im.assign(lvk::kImageWords, 0u);
            uint32_t *ra = &im[lvk::kRegionA / 4], *rb = &im[lvk::kRegionB / 4];
            for (int e = 0; e < 256; ++e)
                for (int c = 0; c < 8; ++c)
                    for (int k = 0; k < 4; ++k) {
                        // slot k is indexed by state byte 3-k (make_lut), so shift
                        // tables store their byte-(3-k) table there
                        ra[e * 64 + 4 * c + k] = T[k][e];
                        ra[e * 64 + 32 + 4 * c + k] = W4[3 - k][e];
                        rb[e * 64 + 4 * c + k] = W1[3 - k][e];
                        rb[e * 64 + 32 + 4 * c + k] = W2[3 - k][e];
                    }
            uint32_t *rc = &im[lvk::kComb / 4];
            for (int k = 0; k < 6; ++k)
                for (int j = 0; j < 4; ++j)
                    for (int e = 0; e < 256; ++e) rc[(k * 4 + j) * 256 + e] = C[k][j][e];
        }
        uint32_t WT[4][256];
        lvgpu::shift_tables(256ull * lvk::kSstRows, WT);
        images[kTableImage] = images[2];
        uint32_t *ra = &images[kTableImage][lvk::kRegionA / 4];
        for (int e = 0; e < 256; ++e)
            for (int c = 0; c < 8; ++c)
                for (int k = 0; k < 4; ++k) ra[e * 64 + 32 + 4 * c + k] = WT[3 - k][e];
    });
    return images[gi];
}

DevCounters g_count[64];

DevCounters &counters() {
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) d = 0;
    return g_count[d];
}

int grow_dev(uint8_t **p, size_t *cap, size_t need) {
    if (*cap >= need) return 0;
    if (*p) LV_HIP(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    LV_HIP(hipMalloc(p, need));
    counters().allocs++;
    *cap = need;
    return 0;
}

int grow_pinned(uint8_t **p, size_t *cap, size_t need) {
    if (*cap >= need) return 0;
    if (*p) LV_HIP(hipHostFree(*p));
    *p = nullptr;
    *cap = 0;
    LV_HIP(hipHostMalloc(p, need, hipHostMallocDefault));
    counters().allocs++;
    *cap = need;
    return 0;
}

// True if p is page-locked host memory (hipHostMalloc / hipHostRegister).
bool is_pinned(const void *p) {
    hipPointerAttribute_t a;
    const hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // pageable memory reports an error; clear it
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// memcpy split over up to 8 host threads (pageable -> pinned staging).
void par_memcpy(uint8_t *dst, const uint8_t *src, size_t bytes, unsigned threads) {
    unsigned nt = std::thread::hardware_concurrency();
    nt = nt == 0 ? 1 : (nt > threads ? threads : nt);
    if (bytes < (4u << 20) || nt == 1) {
        std::memcpy(dst, src, bytes);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (bytes + nt - 1) / nt;
    for (unsigned t = 0; t < nt; ++t) {
        const size_t lo = t * per;
        if (lo >= bytes) break;
        const size_t len = bytes - lo < per ? bytes - lo : per;
        th.emplace_back([=] { std::memcpy(dst + lo, src + lo, len); });
    }
    for (auto &x : th) x.join();
}

DevCtx g_dev[64];

int current_ctx(DevCtx **out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return set_err(LV_ERR_NO_DEVICE, std::string("hipGetDevice: ") + hipGetErrorString(e));
    if (dev < 0 || dev >= 64) return set_err(LV_ERR_NO_DEVICE, "device index out of range");
    DevCtx &c = g_dev[dev];
    std::lock_guard<std::mutex> lk(c.m);
    if (!c.ready) {
        hipDeviceProp_t prop;
        LV_HIP(hipGetDeviceProperties(&prop, dev));
        c.cus = prop.multiProcessorCount;
        for (int i = 0; i < kImages; ++i) {
            const auto &im = host_image(i);
            LV_HIP(hipMalloc(&c.image[i], im.size() * 4));
            counters().allocs++;
            LV_HIP(hipMemcpy(c.image[i], im.data(), im.size() * 4, hipMemcpyHostToDevice));
        }
        {
            std::vector<uint32_t> bt(lvk::kBaseMats * 1024);
            for (uint32_t i = 0; i < lvk::kBaseMats; ++i) {
                uint32_t S[4][256];
                lvgpu::shift_tables(1ull << i, S);
                for (int j = 0; j < 4; ++j)
                    for (int e = 0; e < 256; ++e) bt[i * 1024 + j * 256 + e] = S[j][e];
            }
            LV_HIP(hipMalloc(&c.base_tabs, bt.size() * 4));
            counters().allocs++;
            LV_HIP(hipMemcpy(c.base_tabs, bt.data(), bt.size() * 4, hipMemcpyHostToDevice));
        }
        c.ready = true;
    }
    *out = &c;
    return 0;
}

int pick_gi(uint64_t len) {
    if (len <= 128) return 0;    // G = 1
    if (len <= 1024) return 1;   // G = 4
    if (len <= 16384) return 2;  // G = 16
    return 3;                    // G = 64
}

int forced_gi(uint32_t flags) {
    const uint32_t f = (flags & LV_CRC_GROUP_MASK) >> 8;
    return f ? static_cast<int>(f) - 1 : -1;
}

// The library-owned workspace of (device, stream), grown on demand (the sort
// needs no initialised state).  Returns with the workspace's lock held in
// `lk`; the caller keeps it until its last launch has been enqueued.
static StreamWs *find_ws(DevCtx &c, hipStream_t s, bool create) {
    std::lock_guard<std::mutex> mk(c.ws_m);
    if (!create) {
        auto it = c.ws.find(s);
        return it == c.ws.end() ? nullptr : it->second.get();
    }
    auto &slot = c.ws[s];
    if (!slot) slot.reset(new StreamWs);
    return slot.get();
}

int stream_ws_bytes(DevCtx &c, hipStream_t s, size_t need, uint8_t **out, std::unique_lock<std::mutex> *lk) {
    StreamWs *w = find_ws(c, s, true);
    *lk = std::unique_lock<std::mutex>(w->m);
    if (w->cap < need) {
        if (w->p) LV_HIP(hipFree(w->p));
        w->p = nullptr;
        w->cap = 0;
        LV_HIP(hipMalloc(&w->p, need));
        counters().allocs++;
        w->cap = need;
    }
    *out = w->p;
    return 0;
}

int stream_ws(DevCtx &c, hipStream_t s, uint64_t n, uint8_t **out, std::unique_lock<std::mutex> *lk) {
    return stream_ws_bytes(c, s, sort_ws_bytes(n), out, lk);
}

// The stream's hint-violation word (zeroed on the stream before first use).
int stream_err(DevCtx &c, hipStream_t s, uint32_t **out) {
    StreamWs *w = find_ws(c, s, true);
    std::lock_guard<std::mutex> lk(w->em);
    if (!w->err) {
        LV_HIP(hipHostMalloc(reinterpret_cast<void **>(&w->herr), 4, hipHostMallocDefault));
        LV_HIP(hipMalloc(&w->err, 4));
        counters().allocs += 2;
        LV_HIP(hipMemsetAsync(w->err, 0, 4, s));
    }
    *out = w->err;
    return 0;
}

// lv_crc32c_batch_check: read and clear the stream's violation word.
int check_hints(hipStream_t s, uint32_t *violations) {
    if (violations) *violations = 0;
    DevCtx *c = nullptr;
    if (int rc = current_ctx(&c)) return rc;
    StreamWs *w = find_ws(*c, s, false);
    if (!w) return LV_OK;  // no hinted call on this stream yet
    std::lock_guard<std::mutex> lk(w->em);
    if (!w->err) return LV_OK;
    LV_HIP(hipMemcpyAsync(w->herr, w->err, 4, hipMemcpyDeviceToHost, s));
    LV_HIP(hipStreamSynchronize(s));
    const uint32_t v = *w->herr;
    if (!v) return LV_OK;
    LV_HIP(hipMemsetAsync(w->err, 0, 4, s));  // ordered before the stream's next calls
    if (violations) *violations = v;
    std::string msg = "batch hint violated on the device:";
    if (v & LV_HINT_ERR_MISALIGNED) msg += " an offset is not 16-byte aligned (LV_HINT_ALIGNED16);";
    if (v & LV_HINT_ERR_NOT_UNIFORM) msg += " a length differs from max_len (LV_HINT_UNIFORM);";
    if (v & LV_HINT_ERR_LONGER) msg += " a length exceeds max_len;";
    if (v & LV_HINT_ERR_TOTAL) msg += " the lengths do not sum to total_bytes;";
    msg += " the CRCs of the call(s) are undefined";
    return set_err(LV_ERR_HINT, msg);
}

// Shift_{j plen} (j < 64) and Shift_{64 plen} as 65 GF(2) matrices of 32
// column images on the device (combine_pieces_kernel, and the fused join of
// crc32c_blocks_kernel<16, ..., FUSE>); built once per plen.
int piece_mats(DevCtx &c, uint64_t plen, const uint32_t **out) {
    std::lock_guard<std::mutex> lk(c.mats_m);
    uint32_t *&d = c.piece_mats[plen];
    if (!d) {
        std::vector<uint32_t> h(65 * 32);
        const lvgpu::Gf2Mat step = lvgpu::shift_matrix(plen);
        lvgpu::Gf2Mat m = lvgpu::shift_matrix(0);
        for (uint32_t j = 0; j <= 64; ++j) {
            for (int b = 0; b < 32; ++b) h[j * 32 + b] = m.col[b];
            m = m.then(step);
        }
        uint32_t *p = nullptr;
        LV_HIP(hipMalloc(&p, h.size() * 4));
        counters().allocs++;
        LV_HIP(hipMemcpy(p, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        d = p;
    }
    *out = d;
    return 0;
}

// Byte tables of Shift_{2^v plen}, v < kPow2Tabs (4 x 256 words each), on the
// device (combine_pieces_wg_kernel); built once per plen.
int piece_tabs(DevCtx &c, uint64_t plen, const uint32_t **out) {
    std::lock_guard<std::mutex> lk(c.mats_m);
    uint32_t *&d = c.piece_tabs[plen];
    if (!d) {
        std::vector<uint32_t> h(lvk::kPow2Tabs * 1024);
        for (uint32_t v = 0; v < lvk::kPow2Tabs; ++v) {
            uint32_t S[4][256];
            lvgpu::shift_tables(plen << v, S);
            for (int j = 0; j < 4; ++j)
                for (int e = 0; e < 256; ++e) h[v * 1024 + j * 256 + e] = S[j][e];
        }
        uint32_t *p = nullptr;
        LV_HIP(hipMalloc(&p, h.size() * 4));
        counters().allocs++;
        LV_HIP(hipMemcpy(p, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        d = p;
    }
    *out = d;
    return 0;
}

int check_launch() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return set_err(static_cast<int>(e), std::string("kernel launch: ") + hipGetErrorString(e));
    return 0;
}

}  // namespace lvh

using namespace lvh;

namespace lvgpu_internal {
int set_error(int code, const char *msg) { return set_err(code, msg); }
void clear_error() { g_err.clear(); }
int launch_status() { return check_launch(); }
}  // namespace lvgpu_internal


extern "C" {

const char *lv_last_error(void) { return g_err.c_str(); }

const char *lv_version(void) { return "lvgpu 0.2.0 gfx950"; }

const char *lv_crc32c_last_kernel(void) { return g_kernel; }

int lv_device_counters(int device, uint64_t *out, size_t n) {
    if (device < 0 || device >= 64 || (!out && n)) return set_err(LV_ERR_INVALID, "device index or null pointer");
    const uint64_t v[3] = {g_count[device].h2d.load(), g_count[device].d2h.load(), g_count[device].allocs.load()};
    for (size_t i = 0; i < n && i < 3; ++i) out[i] = v[i];
    return LV_OK;
}

void *lv_host_alloc(size_t bytes) {
    g_err.clear();
    void *p = nullptr;
    const hipError_t e = hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault);
    if (e != hipSuccess) {
        set_err(static_cast<int>(e), std::string("hipHostMalloc: ") + hipGetErrorString(e));
        return nullptr;
    }
    return p;
}

int lv_host_free(void *p) {
    g_err.clear();
    if (!p) return LV_OK;
    LV_HIP(hipHostFree(p));
    return LV_OK;
}

int lv_crc32c_batch_check(void *stream, uint32_t *violations) {
    g_err.clear();
    return check_hints(static_cast<hipStream_t>(stream), violations);
}

int lv_device_init(void) {
    DevCtx *c = nullptr;
    return current_ctx(&c);
}

}  // extern "C"

// Caller holds c.host_m.  Copies h[0, bytes) to c.d_arena and zeroes `pad`
// bytes after it, on c.stream.
static int upload_locked(DevCtx &c, const uint8_t *h, size_t bytes, size_t pad) {
    if (!c.stream) LV_HIP(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    for (auto &ev : c.ev)
        if (!ev) LV_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    hipStream_t s = c.stream;
    if (int rc = grow_dev(&c.d_arena, &c.d_arena_cap, bytes + (pad > 16 ? pad : 16))) return rc;
    if (pad) LV_HIP(hipMemsetAsync(c.d_arena + bytes, 0, pad, s));
    if (bytes == 0) return LV_OK;
    // DMA straight from pinned/registered memory; otherwise a two-slot
    // pipeline (parallel memcpy into one pinned slot while the other slot's
    // H2D runs)
    counters().h2d += bytes;
    if (is_pinned(h)) {
        LV_HIP(hipMemcpyAsync(c.d_arena, h, bytes, hipMemcpyHostToDevice, s));
        return LV_OK;
    }
    for (int k = 0; k < 2; ++k)
        if (int rc = grow_pinned(&c.h_stage[k], &c.h_stage_cap[k], kStageBytes)) return rc;
    size_t k = 0;
    for (size_t pos = 0; pos < bytes; pos += kStageBytes, ++k) {
        const size_t len = bytes - pos < kStageBytes ? bytes - pos : kStageBytes;
        const int slot = static_cast<int>(k & 1);
        // the slot's previous H2D (this call's, or an earlier call's that
        // returned early on an error without synchronizing) must be done;
        // an event never recorded completes at once
        LV_HIP(hipEventSynchronize(c.ev[slot]));
        par_memcpy(c.h_stage[slot], h + pos, len);
        LV_HIP(hipMemcpyAsync(c.d_arena + pos, c.h_stage[slot], len, hipMemcpyHostToDevice, s));
        LV_HIP(hipEventRecord(c.ev[slot], s));
    }
    return LV_OK;
}

namespace lvgpu_internal {
int DeviceGuard::set(int device) {
    if (prev < 0) {
        int d = 0;
        LV_HIP(hipGetDevice(&d));
        prev = d;
    }
    LV_HIP(hipSetDevice(device));
    return LV_OK;
}

DeviceGuard::~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
}

int host_upload(int device, const uint8_t *h, size_t bytes, size_t pad, HostPath *hp) {
    if (int rc = hp->dg.set(device)) return rc;
    DevCtx *c = nullptr;
    if (int rc = current_ctx(&c)) return rc;
    hp->lk = std::unique_lock<std::mutex>(c->host_m);
    if (int rc = upload_locked(*c, h, bytes, pad)) return rc;
    hp->stream = c->stream;
    hp->d_arena = c->d_arena;
    return LV_OK;
}

int pinned_alloc(size_t bytes, uint8_t **p) {
    *p = nullptr;
    LV_HIP(hipHostMalloc(reinterpret_cast<void **>(p), bytes ? bytes : 1, hipHostMallocDefault));
    return LV_OK;
}

void pinned_free(uint8_t *p) {
    if (p) (void)hipHostFree(p);
}

void count_h2d(uint64_t bytes) { counters().h2d += bytes; }
void count_d2h(uint64_t bytes) { counters().d2h += bytes; }
void count_alloc(int device) {
    if (device >= 0 && device < 64) g_count[device].allocs++;
}

int host_scratch(HostPath *hp, int slot, size_t bytes, uint8_t **d) {
    (void)hp;  // the lock it holds is the device's host_m
    DevCtx *c = nullptr;
    if (int rc = current_ctx(&c)) return rc;
    if (slot < 0 || slot > 1) return set_err(LV_ERR_INVALID, "scratch slot");
    if (int rc = grow_dev(&c->d_scr[slot], &c->d_scr_cap[slot], bytes ? bytes : 16)) return rc;
    *d = c->d_scr[slot];
    return LV_OK;
}
}  // namespace lvgpu_internal

extern "C" {

// Host batch with long buffers: one 16-lane group owns a buffer on the GPU,
// so a buffer longer than kSplitBytes is cut into kChunkBytes pieces that run
// as independent units (piece 0 with the buffer's seed, the others from a
// zero register: extend(~0, D) = ~R(0, D)), and the host joins them by
// linearity, R(s, A||B) = Shift_|B|(R(s, A)) ^ R(0, B), with GF(2) shift
// matrices (crc32c_gf2.h).  The join is 32-bit arithmetic per piece; every
// byte is still checksummed on the GPU.
constexpr uint64_t kSplitBytes = 1ull << 20;
constexpr uint64_t kChunkBytes = 256ull << 10;

static int batch_host_split(const uint8_t *h_arena, size_t arena_bytes, const uint64_t *h_off,
                            const uint32_t *h_len, const uint32_t *h_seed, uint32_t *h_out, size_t n,
                            uint32_t flags, int device) {
    std::vector<uint64_t> off;
    std::vector<uint32_t> len, seed, out;
    std::vector<size_t> first(n + 1);  // pieces of buffer i: [first[i], first[i+1])
    for (size_t i = 0; i < n; ++i) {
        first[i] = off.size();
        const uint32_t s = h_seed ? h_seed[i] : 0u;
        if (h_len[i] <= kSplitBytes) {
            off.push_back(h_off[i]);
            len.push_back(h_len[i]);
            seed.push_back(s);
            continue;
        }
        for (uint64_t p = 0; p < h_len[i]; p += kChunkBytes) {
            off.push_back(h_off[i] + p);
            len.push_back(static_cast<uint32_t>(std::min<uint64_t>(kChunkBytes, h_len[i] - p)));
            seed.push_back(p == 0 ? s : 0xffffffffu);
        }
    }
    first[n] = off.size();
    out.resize(off.size());
    if (int rc = lv_crc32c_batch_host(h_arena, arena_bytes, off.data(), len.data(), seed.data(), out.data(),
                                      off.size(), flags & ~LV_CRC_MASK, device))
        return rc;
    const lvgpu::Gf2Mat shift_chunk = lvgpu::shift_matrix(kChunkBytes);
    for (size_t i = 0; i < n; ++i) {
        uint32_t crc = out[first[i]];
        if (first[i + 1] - first[i] > 1) {
            uint32_t r = ~crc;  // R(~seed, piece 0)
            for (size_t k = first[i] + 1; k < first[i + 1]; ++k) {
                const uint32_t shifted = len[k] == kChunkBytes ? shift_chunk.apply(r)
                                                               : lvgpu::shift_matrix(len[k]).apply(r);
                r = shifted ^ ~out[k];  // ^ R(0, piece k)
            }
            crc = ~r;
        }
        h_out[i] = (flags & LV_CRC_MASK) ? lv_crc32c_mask(crc) : crc;
    }
    return LV_OK;
}

int lv_crc32c_batch_host(const uint8_t *h_arena, size_t arena_bytes, const uint64_t *h_off,
                         const uint32_t *h_len, const uint32_t *h_seed, uint32_t *h_out, size_t n,
                         uint32_t flags, int device) {
    g_err.clear();
    if (n == 0) return LV_OK;
    if (!h_arena || !h_off || !h_len || !h_out) return set_err(LV_ERR_INVALID, "null host pointer");
    if (n > 0xffffffffull) return set_err(LV_ERR_INVALID, "more than 2^32-1 buffers per call");
    bool long_buffers = false;
    for (size_t i = 0; i < n; ++i) {
        if (h_off[i] > arena_bytes || h_len[i] > arena_bytes - h_off[i])
            return set_err(LV_ERR_INVALID, "buffer outside arena");
        long_buffers |= h_len[i] > kSplitBytes;
    }
    if (long_buffers) return batch_host_split(h_arena, arena_bytes, h_off, h_len, h_seed, h_out, n, flags, device);
    lvgpu_internal::DeviceGuard dg;  // the caller's current device comes back on return
    if (int rc = dg.set(device)) return rc;
    DevCtx *c = nullptr;
    if (int rc = current_ctx(&c)) return rc;
    std::lock_guard<std::mutex> lk(c->host_m);
    if (int rc = upload_locked(*c, h_arena, arena_bytes, 0)) return rc;
    hipStream_t s = c->stream;
    const size_t meta = n * (8 + 4 + 4 + 4);
    if (int rc = grow_dev(&c->d_meta, &c->d_meta_cap, meta)) return rc;
    if (int rc = grow_pinned(&c->h_meta, &c->h_meta_cap, meta)) return rc;
    uint64_t *d_off = reinterpret_cast<uint64_t *>(c->d_meta);
    uint32_t *d_len = reinterpret_cast<uint32_t *>(d_off + n);
    uint32_t *d_seed = d_len + n;
    uint32_t *d_out = d_seed + n;

    // metadata: one pinned staging copy, async
    std::memcpy(c->h_meta, h_off, n * 8);
    std::memcpy(c->h_meta + n * 8, h_len, n * 4);
    if (h_seed) std::memcpy(c->h_meta + n * 12, h_seed, n * 4);
    LV_HIP(hipMemcpyAsync(d_off, c->h_meta, n * (h_seed ? 16 : 12), hipMemcpyHostToDevice, s));
    counters().h2d += n * (h_seed ? 16 : 12);
    uint8_t *ws = nullptr;
    std::unique_lock<std::mutex> ws_lk;
    if (int rc = stream_ws(*c, s, n, &ws, &ws_lk)) return rc;
    // the lengths are on the host here: the join is launched only if needed
    lv_batch_hint hint{0, 0, 1};
    for (size_t i = 0; i < n; ++i) {
        hint.total_bytes += h_len[i];
        hint.max_len = std::max(hint.max_len, h_len[i]);
    }
    for (size_t i = 0; i < n && hint.uniform; ++i) hint.uniform = h_len[i] == hint.max_len;
    bool aligned = hint.uniform && hint.max_len && reinterpret_cast<uintptr_t>(c->d_arena) % 16 == 0;
    for (size_t i = 0; i < n && aligned; ++i) aligned = h_off[i] % 16 == 0;
    const UniformPlan pl = aligned ? uniform_plan(c->cus, 0, 0, hint.max_len, n, -1) : UniformPlan{0, -1, 0};
    if (pl.applies() && pl.scratch <= sort_ws_bytes(n)) {
        // aligned uniform blocks (LV_HINT_ALIGNED16): the strided API's kernels
        if (int rc = launch_uniform(*c, pl, c->d_arena, 0, d_off, d_len, nullptr, hint.max_len, n,
                                    h_seed ? d_seed : nullptr, d_out, flags, s, ws))
            return rc;
    } else if (int rc = launch_binned(*c, ws, c->d_arena, d_off, d_len, h_seed ? d_seed : nullptr, d_out, n, flags, s,
                                      hint_needs_join(hint, n, static_cast<uint32_t>(c->cus)))) {
        return rc;
    }
    if (int rc = check_launch()) return rc;
    LV_HIP(hipMemcpyAsync(c->h_meta, d_out, n * 4, hipMemcpyDeviceToHost, s));
    counters().d2h += n * 4;
    LV_HIP(hipStreamSynchronize(s));
    std::memcpy(h_out, c->h_meta, n * 4);
    return LV_OK;
}

int lv_fill_splitmix(uint8_t *d_dst, uint64_t begin, uint64_t nbytes, uint64_t seed, void *stream) {
    g_err.clear();
    if (nbytes == 0) return LV_OK;
    if (!d_dst) return set_err(LV_ERR_INVALID, "null device pointer");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool words = (reinterpret_cast<uintptr_t>(d_dst) % 8 == 0) && begin % 8 == 0 && nbytes % 8 == 0;
    const uint64_t items = words ? nbytes / 8 : nbytes;
    uint64_t grid = (items + 255) / 256;
    if (grid > 65536) grid = 65536;
    if (words)
        hipLaunchKernelGGL(lvk::fill_words_kernel, dim3(static_cast<uint32_t>(grid)), dim3(256), 0, s,
                           reinterpret_cast<uint64_t *>(d_dst), begin / 8, nbytes / 8, seed);
    else
        hipLaunchKernelGGL(lvk::fill_bytes_kernel, dim3(static_cast<uint32_t>(grid)), dim3(256), 0, s,
                           d_dst, begin, nbytes, seed);
    return check_launch();
}

}  // extern "C"
