// MI355X (gfx950 / CDNA4) batched CRC32C.
//
// Replaces, for many buffers at once, the per-record crc32c::extend /
// crc32c::value calls of the reference WAL (log_writer.rs:123-124,
// log_reader.rs:335-336) and the table-block checksum.  Output
// is bit-identical to crc32c.rs:42-63 (extend + optional mask).
//
// Kernel design (DESIGN.md "Kernel"):
//  * A group of G lanes (G in {1,4,16,64}) owns one buffer at a time; a
//    wave holds 64/G groups.  Lane i of a group loads the i-th 16-B granule of
//    every "row" of G granules with one global_load_dwordx4, so a row is one
//    contiguous, coalesced run of 16*G bytes.  Rows are aligned to the END of
//    the buffer; missing granules before the buffer start read as zeros
//    (leading zeros leave a zero CRC register unchanged).
//  * Per lane: p = R(0, granule) by four slice-by-4 steps; across rows
//    A = Shift_{16G}(A) ^ p (Horner).  Groups then combine lanes pairwise,
//    A_i = Shift_{16*2^k}(A_i) ^ A_{i+2^k}, k < log2 G.  The bytes after the
//    last aligned granule (<16) are folded in by one lane, bytewise.
//  * The seed enters by xoring (seed ^ ~0) into the first 4 buffer bytes:
//    R(s, w||D) = R(0, (s^w)||D).  Buffers shorter than 4 bytes go bytewise.
//  * Lookup tables live in LDS.  The slice tables T0..T3 and the row-shift
//    tables W0..W3 use a "Latin-square" replicated layout: entry e of table k,
//    copy c sits in dword (4c+k) (+32 for W) of a 256-B row e.  In lookup
//    instruction i, lane g (of a 32-lane LDS group; c = g&7, q = g>>3) reads
//    table (q+i)&3, so the 32 lanes of every ds_read_b32 hit 32 distinct
//    banks: conflict-free random lookups with 64 KiB of tables.  The address
//    (row e from a state byte, dword from the lane) is ONE v_perm_b32.
//  * Persistent grid: one 1024-thread workgroup per CU (88 KiB LDS image).
//
// No MFMA: the work is one table lookup per byte, bound by HBM read
// bandwidth (roofline in DESIGN.md).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/lvgpu/crc32c.h"
#include "crc32c_gf2.h"

namespace lvk {

constexpr int kThreads = 1024;                   // 16 waves: 4 per SIMD
constexpr int kWaves = kThreads / 64;
constexpr int kCombWords = 6 * 4 * 256;          // Shift_{16*2^k} byte tables, k = 0..5
constexpr int kLatinWords = 256 * 64;            // 256 rows x 256 B
constexpr int kImageWords = kCombWords + kLatinWords;  // 22528 dwords = 88 KiB
constexpr uint32_t kLatinBase = kCombWords * 4;  // 24576, fits the ds offset field
constexpr uint32_t kShiftOff = 128;              // W tables: dwords 32..63 of a row

__shared__ __attribute__((aligned(16))) uint32_t g_lds[kImageWords];

// Per-lane lookup constants: lv byte i = 4*beta_i (dword of the lane's table
// copy for instruction i); sel_i moves that byte to bits 0..7 and the state
// byte indexing table k_i to bits 8..15 (v_perm selector: 0-3 = S1 bytes,
// 4-7 = S0 bytes, 12 = 0x00).
struct Lut {
    uint32_t lv, sel0, sel1, sel2, sel3, c4;
};

__device__ __forceinline__ Lut make_lut(uint32_t lane) {
    const uint32_t g = lane & 31u, c = g & 7u, q = g >> 3;
    Lut L;
    L.lv = 0;
    uint32_t sel[4];
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
        const uint32_t k = (q + i) & 3u;
        L.lv |= ((4u * c + k) * 4u) << (8u * i);
        sel[i] = 0x0C0C0000u | ((4u + 3u - k) << 8) | i;
    }
    L.sel0 = sel[0];
    L.sel1 = sel[1];
    L.sel2 = sel[2];
    L.sel3 = sel[3];
    L.c4 = 4u * c;
    return L;
}

__device__ __forceinline__ uint32_t lds_word(uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(g_lds) + byte_addr);
}

// XOR of the four Latin-region tables at OFF (0: T, kShiftOff: W) indexed by
// the four bytes of s.  OFF = 0: one slice-by-4 step, T3[b0]^T2[b1]^T1[b2]^T0[b3].
template <uint32_t OFF>
__device__ __forceinline__ uint32_t lookup4(uint32_t s, const Lut &L) {
    const uint32_t a0 = __builtin_amdgcn_perm(s, L.lv, L.sel0);
    const uint32_t a1 = __builtin_amdgcn_perm(s, L.lv, L.sel1);
    const uint32_t a2 = __builtin_amdgcn_perm(s, L.lv, L.sel2);
    const uint32_t a3 = __builtin_amdgcn_perm(s, L.lv, L.sel3);
    return lds_word(a0 + kLatinBase + OFF) ^ lds_word(a1 + kLatinBase + OFF) ^
           lds_word(a2 + kLatinBase + OFF) ^ lds_word(a3 + kLatinBase + OFF);
}

// R(s, 16 bytes of v).
__device__ __forceinline__ uint32_t chain16(uint32_t s, uint4 v, const Lut &L) {
    s = lookup4<0>(s ^ v.x, L);
    s = lookup4<0>(s ^ v.y, L);
    s = lookup4<0>(s ^ v.z, L);
    return lookup4<0>(s ^ v.w, L);
}

// Shift_{16*2^k}(a) from the unreplicated combine tables.
__device__ __forceinline__ uint32_t comb_shift(uint32_t a, int k) {
    const uint32_t *t = g_lds + k * 1024;
    return t[a & 0xffu] ^ t[256 + ((a >> 8) & 0xffu)] ^ t[512 + ((a >> 16) & 0xffu)] ^
           t[768 + (a >> 24)];
}

// One byte through T0 (copy of this lane): crc32c.rs:81.
__device__ __forceinline__ uint32_t byte_step(uint32_t s, uint32_t b, uint32_t c4) {
    const uint32_t e = (s ^ b) & 0xffu;
    return g_lds[kCombWords + e * 64u + c4] ^ (s >> 8);
}

// Head fix-up of word d of a granule: rel = (word address) - (buffer start).
// Bytes before the buffer become 0; bytes 0..3 of the buffer get s0 xored in.
__device__ __forceinline__ uint32_t fix_word(uint32_t w, int64_t rel, uint32_t s0) {
    if (rel >= 4) return w;
    if (rel <= -4) return 0u;
    if (rel < 0) {
        const uint32_t sh = static_cast<uint32_t>(-rel) * 8u;
        return (w & (0xffffffffu << sh)) ^ (s0 << sh);
    }
    return w ^ (s0 >> (static_cast<uint32_t>(rel) * 8u));
}

// Global (address space 1) pointers: global_load_* counts only in vmcnt, so
// outstanding HBM loads never hold up the LDS lookups' lgkmcnt waits (a flat
// load would count in both).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 g_u32x4;
typedef const __attribute__((address_space(1))) uint8_t g_uint8;

__device__ __forceinline__ uint4 load_granule(uint64_t g) {
    const u32x4 v = *reinterpret_cast<g_u32x4 *>(g << 4);
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint32_t load_byte(uint64_t addr) {
    return *reinterpret_cast<g_uint8 *>(addr);
}

__device__ __forceinline__ uint32_t mask_crc(uint32_t c) {  // crc32c.rs:54-57
    return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}

// CRC of buffer [a, a+len) (absolute device address) with seed, computed by the
// G lanes of a group; the result is valid in lane gl == 0.
template <int G>
__device__ __forceinline__ uint32_t crc_group(uint64_t a, uint32_t len, uint32_t seed, uint32_t gl,
                                              const Lut &L) {
    const uint32_t s0 = ~seed;
    if (len < 4) {  // crc32c.rs:112-115 path: bytewise from the seeded state
        uint32_t s = s0;
        if (gl == 0)
            for (uint32_t i = 0; i < len; ++i)
                s = byte_step(s, load_byte(a + i), L.c4);
        return ~s;
    }
    const uint64_t e = a + len;
    const uint64_t g0 = a >> 4, gend = e >> 4;
    const uint32_t ng = static_cast<uint32_t>(gend - g0);
    const uint32_t nrows = (ng + G - 1) / G;
    const int64_t gs = static_cast<int64_t>(gend) - static_cast<int64_t>(G) * nrows;
    const uint64_t tail_base = gend << 4;
    const uint32_t tail_hi = static_cast<uint32_t>(e - tail_base);
    const uint32_t tail_lo = a > tail_base ? static_cast<uint32_t>(a - tail_base) : 0u;

    uint4 tail = make_uint4(0, 0, 0, 0);
    if (gl == 0 && tail_hi != 0) tail = load_granule(gend);

    // Rows are consumed in batches of U with the next batch's loads in flight
    // (software pipeline: 2*U granules = 2*U*16*64 B per wave outstanding).
    constexpr uint32_t U = 4;
    const int64_t g0s = static_cast<int64_t>(g0);
    auto load_row = [&](uint32_t r) -> uint4 {
        const int64_t g = gs + static_cast<int64_t>(G) * r + gl;
        if (r < nrows && g >= g0s) return load_granule(static_cast<uint64_t>(g));
        return make_uint4(0, 0, 0, 0);
    };
    uint4 cur[U], nxt[U];
#pragma unroll
    for (uint32_t j = 0; j < U; ++j) cur[j] = load_row(j);

    uint32_t A = 0;
    for (uint32_t r = 0; r < nrows; r += U) {
#pragma unroll
        for (uint32_t j = 0; j < U; ++j) nxt[j] = load_row(r + U + j);
        uint32_t p[U];
#pragma unroll
        for (uint32_t j = 0; j < U; ++j) {
            uint4 v = cur[j];
            const int64_t g = gs + static_cast<int64_t>(G) * (r + j) + gl;
            const int64_t rel = g * 16 - static_cast<int64_t>(a);
            if (rel < 4 && g >= g0s) {  // head granule(s): zero pre-buffer bytes, xor seed
                v.x = fix_word(v.x, rel, s0);
                v.y = fix_word(v.y, rel + 4, s0);
                v.z = fix_word(v.z, rel + 8, s0);
                v.w = fix_word(v.w, rel + 12, s0);
            }
            if constexpr (G == 1) {
                if (r + j < nrows) A = chain16(A, v, L);
            } else {
                p[j] = chain16(0u, v, L);
            }
        }
        if constexpr (G != 1) {
#pragma unroll
            for (uint32_t j = 0; j < U; ++j)
                if (r + j < nrows) A = lookup4<kShiftOff>(A, L) ^ p[j];
        }
#pragma unroll
        for (uint32_t j = 0; j < U; ++j) cur[j] = nxt[j];
    }
#pragma unroll
    for (int k = 0; (1 << k) < G; ++k) {
        const uint32_t other = __shfl_down(A, 1u << k, G);
        A = comb_shift(A, k) ^ other;
    }
    if (gl == 0) {
        const uint32_t tw[4] = {tail.x, tail.y, tail.z, tail.w};
        for (uint32_t i = tail_lo; i < tail_hi; ++i) {
            uint32_t b = (tw[i >> 2] >> (8u * (i & 3u))) & 0xffu;
            const uint64_t rel = tail_base + i - a;
            if (rel < 4) b ^= (s0 >> (8u * static_cast<uint32_t>(rel))) & 0xffu;
            A = byte_step(A, b, L.c4);
        }
    }
    return ~A;
}

__device__ __forceinline__ void stage_tables(const uint4 *__restrict__ image) {
    uint4 *l4 = reinterpret_cast<uint4 *>(g_lds);
    for (int i = threadIdx.x; i < kImageWords / 4; i += kThreads) l4[i] = image[i];
    __syncthreads();
}

template <int G, bool STRIDED>
__global__ __launch_bounds__(kThreads) void crc32c_batch_kernel(
    const uint8_t *__restrict__ arena, const uint64_t *__restrict__ off,
    const uint32_t *__restrict__ len, uint64_t stride, uint32_t blen,
    const uint32_t *__restrict__ seed, uint32_t *__restrict__ out, uint64_t n, uint32_t flags,
    const uint4 *__restrict__ image) {
    stage_tables(image);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    const Lut L = make_lut(lane);
    constexpr uint32_t kGroups = 64 / G;
    const uint32_t gl = lane % G;
    const uint64_t gid =
        (static_cast<uint64_t>(blockIdx.x) * kWaves + wave) * kGroups + lane / G;
    const uint64_t gstride = static_cast<uint64_t>(gridDim.x) * kWaves * kGroups;
    const uint64_t base = reinterpret_cast<uint64_t>(arena);
    for (uint64_t b = gid; b < n; b += gstride) {
        uint64_t a;
        uint32_t ln;
        if constexpr (STRIDED) {
            a = base + b * stride;
            ln = blen;
        } else {
            a = base + off[b];
            ln = len[b];
        }
        const uint32_t sd = seed ? seed[b] : 0u;
        const uint32_t crc = crc_group<G>(a, ln, sd, gl, L);
        if (gl == 0) out[b] = (flags & LV_CRC_MASK) ? mask_crc(crc) : crc;
    }
}

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

// ---------------------------------------------------------------------------
// Host side: per-device context, table images, launch and the C ABI.
// ---------------------------------------------------------------------------
namespace {

thread_local std::string g_err;

int set_err(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define LV_HIP(call)                                                                   \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess)                                                          \
            return set_err(static_cast<int>(e_), std::string(#call) + ": " +           \
                                                     hipGetErrorString(e_));           \
    } while (0)

constexpr int kGs[4] = {1, 4, 16, 64};

// Host copy of the LDS image for each G (index into kGs).
const std::vector<uint32_t> &host_image(int gi) {
    static std::vector<uint32_t> images[4];
    static std::once_flag once;
    std::call_once(once, [] {
        uint32_t T[4][256], C[6][4][256];
        lvgpu::slice_tables(T);
        for (int k = 0; k < 6; ++k) lvgpu::shift_tables(16ull << k, C[k]);
        for (int i = 0; i < 4; ++i) {
            std::vector<uint32_t> &im = images[i];
            im.assign(lvk::kImageWords, 0u);
            for (int k = 0; k < 6; ++k)
                for (int j = 0; j < 4; ++j)
                    for (int e = 0; e < 256; ++e) im[(k * 4 + j) * 256 + e] = C[k][j][e];
            uint32_t W[4][256];
            lvgpu::shift_tables(16ull * kGs[i], W);
            for (int e = 0; e < 256; ++e)
                for (int c = 0; c < 8; ++c)
                    for (int k = 0; k < 4; ++k) {
                        uint32_t *row = &im[lvk::kCombWords + e * 64];
                        row[4 * c + k] = T[k][e];           // T_k indexed by state byte 3-k
                        row[32 + 4 * c + k] = W[3 - k][e];  // W indexed the same way
                    }
        }
    });
    return images[gi];
}

struct DevCtx {
    std::mutex m;
    bool ready = false;
    int cus = 0;
    uint4 *image[4] = {nullptr, nullptr, nullptr, nullptr};
    // host-path staging (grown on demand)
    uint8_t *d_arena = nullptr;
    size_t d_arena_cap = 0;
    uint8_t *d_meta = nullptr;
    size_t d_meta_cap = 0;
    uint8_t *h_pinned = nullptr;
    size_t h_pinned_cap = 0;
    hipStream_t stream = nullptr;
};

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
        for (int i = 0; i < 4; ++i) {
            const auto &im = host_image(i);
            LV_HIP(hipMalloc(&c.image[i], im.size() * 4));
            LV_HIP(hipMemcpy(c.image[i], im.data(), im.size() * 4, hipMemcpyHostToDevice));
        }
        c.ready = true;
    }
    *out = &c;
    return 0;
}

// Buffers-per-group choice for a known (uniform) length.
int pick_gi(uint64_t len) {
    if (len <= 128) return 0;    // G = 1
    if (len <= 1024) return 1;   // G = 4
    if (len <= 16384) return 2;  // G = 16
    return 3;                    // G = 64
}

// Group-size override from flags (LV_CRC_GROUP), or -1.
int forced_gi(uint32_t flags) {
    const uint32_t f = (flags & LV_CRC_GROUP_MASK) >> 8;
    return f ? static_cast<int>(f) - 1 : -1;
}

template <int G, bool STRIDED>
void launch_one(const DevCtx &c, int gi, const uint8_t *arena, const uint64_t *off,
                const uint32_t *len, uint64_t stride, uint32_t blen, const uint32_t *seed,
                uint32_t *out, uint64_t n, uint32_t flags, hipStream_t s) {
    const uint64_t groups_per_wg = static_cast<uint64_t>(lvk::kWaves) * (64 / G);
    uint64_t grid = (n + groups_per_wg - 1) / groups_per_wg;
    if (grid > static_cast<uint64_t>(c.cus)) grid = c.cus;
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL((lvk::crc32c_batch_kernel<G, STRIDED>), dim3(static_cast<uint32_t>(grid)),
                       dim3(lvk::kThreads), 0, s, arena, off, len, stride, blen, seed, out, n,
                       flags, c.image[gi]);
}

template <bool STRIDED>
void launch_g(const DevCtx &c, int gi, const uint8_t *arena, const uint64_t *off,
              const uint32_t *len, uint64_t stride, uint32_t blen, const uint32_t *seed,
              uint32_t *out, uint64_t n, uint32_t flags, hipStream_t s) {
    switch (gi) {
        case 0: launch_one<1, STRIDED>(c, gi, arena, off, len, stride, blen, seed, out, n, flags, s); break;
        case 1: launch_one<4, STRIDED>(c, gi, arena, off, len, stride, blen, seed, out, n, flags, s); break;
        case 2: launch_one<16, STRIDED>(c, gi, arena, off, len, stride, blen, seed, out, n, flags, s); break;
        default: launch_one<64, STRIDED>(c, gi, arena, off, len, stride, blen, seed, out, n, flags, s); break;
    }
}

int check_launch() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return set_err(static_cast<int>(e), std::string("kernel launch: ") + hipGetErrorString(e));
    return 0;
}

}  // namespace

extern "C" {

const char *lv_last_error(void) { return g_err.c_str(); }

const char *lv_version(void) { return "lvgpu 0.1.0 gfx950"; }

int lv_device_init(void) {
    DevCtx *c = nullptr;
    return current_ctx(&c);
}

int lv_crc32c_batch_device(const uint8_t *d_arena, const uint64_t *d_off, const uint32_t *d_len,
                           const uint32_t *d_seed, uint32_t *d_out, size_t n, uint32_t flags,
                           void *stream) {
    g_err.clear();
    if (n == 0) return LV_OK;
    if (!d_arena || !d_off || !d_len || !d_out) return set_err(LV_ERR_INVALID, "null device pointer");
    DevCtx *c = nullptr;
    if (int rc = current_ctx(&c)) return rc;
    const int gi = forced_gi(flags);
    launch_g<false>(*c, gi >= 0 ? gi : 2, d_arena, d_off, d_len, 0, 0, d_seed, d_out, n, flags,
                    static_cast<hipStream_t>(stream));
    return check_launch();
}

int lv_crc32c_batch_strided(const uint8_t *d_base, uint64_t stride, uint32_t block_len, size_t n,
                            const uint32_t *d_seed, uint32_t *d_out, uint32_t flags, void *stream) {
    g_err.clear();
    if (n == 0) return LV_OK;
    if (!d_base || !d_out) return set_err(LV_ERR_INVALID, "null device pointer");
    DevCtx *c = nullptr;
    if (int rc = current_ctx(&c)) return rc;
    const int gi = forced_gi(flags);
    launch_g<true>(*c, gi >= 0 ? gi : pick_gi(block_len), d_base, nullptr, nullptr, stride, block_len, d_seed,
                   d_out, n, flags, static_cast<hipStream_t>(stream));
    return check_launch();
}

int lv_crc32c_batch_host(const uint8_t *h_arena, size_t arena_bytes, const uint64_t *h_off,
                         const uint32_t *h_len, const uint32_t *h_seed, uint32_t *h_out, size_t n,
                         uint32_t flags, int device) {
    g_err.clear();
    if (n == 0) return LV_OK;
    if (!h_arena || !h_off || !h_len || !h_out) return set_err(LV_ERR_INVALID, "null host pointer");
    for (size_t i = 0; i < n; ++i)
        if (h_off[i] > arena_bytes || h_len[i] > arena_bytes - h_off[i])
            return set_err(LV_ERR_INVALID, "buffer outside arena");
    LV_HIP(hipSetDevice(device));
    DevCtx *c = nullptr;
    if (int rc = current_ctx(&c)) return rc;
    std::lock_guard<std::mutex> lk(c->m);
    if (!c->stream) LV_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    const size_t meta = n * (8 + 4 + 4 + 4);
    const size_t need_dev = arena_bytes + 16;
    if (c->d_arena_cap < need_dev) {
        if (c->d_arena) LV_HIP(hipFree(c->d_arena));
        c->d_arena = nullptr;
        c->d_arena_cap = 0;
        LV_HIP(hipMalloc(&c->d_arena, need_dev));
        c->d_arena_cap = need_dev;
    }
    if (c->d_meta_cap < meta) {
        if (c->d_meta) LV_HIP(hipFree(c->d_meta));
        c->d_meta = nullptr;
        c->d_meta_cap = 0;
        LV_HIP(hipMalloc(&c->d_meta, meta));
        c->d_meta_cap = meta;
    }
    const size_t need_pin = arena_bytes > meta ? arena_bytes : meta;
    if (c->h_pinned_cap < need_pin) {
        if (c->h_pinned) LV_HIP(hipHostFree(c->h_pinned));
        c->h_pinned = nullptr;
        c->h_pinned_cap = 0;
        LV_HIP(hipHostMalloc(&c->h_pinned, need_pin, hipHostMallocDefault));
        c->h_pinned_cap = need_pin;
    }
    uint64_t *d_off = reinterpret_cast<uint64_t *>(c->d_meta);
    uint32_t *d_len = reinterpret_cast<uint32_t *>(d_off + n);
    uint32_t *d_seed = d_len + n;
    uint32_t *d_out = d_seed + n;
    hipStream_t s = c->stream;
    // metadata via pinned staging, then the payload
    std::memcpy(c->h_pinned, h_off, n * 8);
    std::memcpy(c->h_pinned + n * 8, h_len, n * 4);
    if (h_seed) std::memcpy(c->h_pinned + n * 12, h_seed, n * 4);
    LV_HIP(hipMemcpyAsync(d_off, c->h_pinned, n * (h_seed ? 16 : 12), hipMemcpyHostToDevice, s));
    LV_HIP(hipStreamSynchronize(s));
    std::memcpy(c->h_pinned, h_arena, arena_bytes);
    LV_HIP(hipMemcpyAsync(c->d_arena, c->h_pinned, arena_bytes, hipMemcpyHostToDevice, s));
    launch_g<false>(*c, 2, c->d_arena, d_off, d_len, 0, 0, h_seed ? d_seed : nullptr, d_out, n,
                    flags, s);
    if (int rc = check_launch()) return rc;
    LV_HIP(hipMemcpyAsync(c->h_pinned, d_out, n * 4, hipMemcpyDeviceToHost, s));
    LV_HIP(hipStreamSynchronize(s));
    std::memcpy(h_out, c->h_pinned, n * 4);
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
