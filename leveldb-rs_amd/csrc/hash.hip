// Batched leveldb hash (util/hash.rs:20-51) on MI355X, SURVEY 8f row 4.
//
// The hash is a serial, non-linear chain over 4-byte words
// (h = ((h + w) * m) ^ (h >> 16)), so unlike CRC32C it cannot be split
// inside a buffer: one lane owns one buffer.  Its keys are cache keys (tens of
// bytes), so a launch is bound by metadata + key bytes through HBM.  A wave
// whose 64 keys lie within 4 KiB stages those bytes through LDS with
// coalesced 16-B loads; otherwise each lane reads its key's dwords from
// memory.  Either way the words are dword-aligned reads funnel-shifted by the
// key's byte misalignment (v_alignbyte_b32), never touching a dword past the
// key's last byte, and keys of <= 64 B run the chain from registers.
// Round 4 (profiles/r04/hash_pmc/, hash_ab/): the kernel is not bound by its
// bytes -- packed keys fetch 15 % less (n + 1 bounds instead of an offset and
// a length per key) in the same time -- nor by its instruction stream: a
// branch-free chain and span staging (selects instead of exec-mask branches,
// ~180 scalar instructions per set of 64 keys fewer) measured the same.  The
// waves sit in s_waitcnt 56 % of their cycles (SQ_WAIT_ANY): each set's span
// load waits for the set's metadata, so a set costs one exposed memory round
// trip per wave at full occupancy.  Prefetching the next set's span one
// set ahead into a second LDS stage by LDS-DMA (global_load_lds_dwordx4, two
// 2.5 KiB stages per wave, 7 workgroups per CU) was correct but slower:
// 145 -> 172 us on the offsets API, packed u32 unchanged
// (profiles/r04/hash_glds/) -- so the round trip is not the bound either.
// Wait counts (round 4): the next set's metadata was loaded under an exec
// mask and a `more` branch, so the compiler could not count the loads in
// flight and waited vmcnt(0) -- for the prefetch just issued -- at the top of
// every set.  Every lane now loads its (clamped) metadata and the validity
// select waits until the set is hashed: offsets
// API unchanged (0.515 vs 0.516), packed u32 keys 0.504 -> 0.542
// (profiles/r04/hash_exact/).  A two-deep kernel with every load exact --
// the next set's span in registers while this set hashes, 80 VGPRs, 6
// workgroups per CU -- measured 0.46 against 0.52 on one box
// (profiles/r04/base_ab/) and was removed.  VALU: ~170 ops per set (wave64 =
// 4 cycles an op), ~100 of them the 17-word chain and its tail; taking the
// tail-word capture (a compare and a select per word) out of the chain --
// its two dwords re-read after it -- and reading the 17-dword LDS window
// unmasked: offsets 0.518 -> 0.53, packed u32 0.549 -> 0.575
// (profiles/r04/hash_tail/, hash_ldsall/).  The multiply is not the bound:
// a full-rate 24-bit one (a timing-only build, wrong hashes) ran the same
// (profiles/r04/hash_mul/).
// The grid is persistent (8 workgroups per CU): a wave walks sets of 64 keys,
// requests the next set's metadata ahead, and stores each result one set
// late, after the next set's loads, so no wait includes a store.  (A
// two-deep form -- the next set's span in flight in registers while this
// set hashes from LDS, metadata two sets ahead, 64 VGPRs at 8 waves/SIMD --
// measured 106 vs 117 G keys/s, three interleaved reps: not kept.)
// Round 5 (profiles/r05/hash_kpl2/, hash_glds2/, valu/): two keys per lane,
// chains interleaved in one loop over a 128-key set (95 VGPRs, 5 waves per
// SIMD): 0.41-0.49 vs 0.53 by key bytes; the LDS-DMA prefetch again, with
// every memory operation of a set issued before its chains and one vmcnt(0)
// a set (the round-4 version waited on its own prefetch): 0.41 vs 0.53.
// Neither kept.  Nor is the VALU the bound: SQ_INSTS_VALU = 43.4 M per
// launch (165 per set), at the 2.44 cycles a simple wave64 op measures on
// this part (tools/pmc_calib.hip) 0.30 of the launch's issue capacity.
// What the launch moves -- keys + 12 B of metadata + 4 B of output per key,
// 0.87 GB -- runs at 0.77 of 8 TB/s: HBM binds.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstring>

#include "../../include/lvgpu/crc32c.h"
#include "../../include/lvgpu/hash.h"
#include "lv_internal.h"
#include "lvk/knobs.h"


namespace lvh {

constexpr uint32_t kM = 0xc6a4a793u;  // hash.rs:23
constexpr uint32_t kFastDw = 17;      // dwords of the register fast path (keys <= 64 B + misalignment)

typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

__device__ __forceinline__ uint32_t mix(uint32_t h, uint32_t w) {  // hash.rs:31-35
    h += w;
    h *= kM;
    return h ^ (h >> 16);
}

// bytes [bs, bs+4) of the 8-byte little-endian pair (lo, hi)
__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t bs) {
    return __builtin_amdgcn_alignbyte(hi, lo, bs);
}

// One wave's staged key bytes: the 16-B granules spanning its 64 keys.


constexpr uint32_t kSpanBytes = 4096;
constexpr uint64_t kWgsPerCu = LVK_HASH_WGS_PER_CU;
constexpr uint32_t kSpanPad = 20;  // dwords past the span a masked fast-path read may address

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        const uint64_t o = __shfl_xor(v, m);
        v = o < v ? o : v;
    }
    return v;
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        const uint64_t o = __shfl_xor(v, m);
        v = o > v ? o : v;
    }
    return v;
}

// hash.rs:25-48 of one key of any length read straight from memory
// (dword-aligned reads, funnel-shifted by the key's misalignment, never a
// dword past its last byte); h arrives as seed ^ (kM * L).
__device__ __forceinline__ uint32_t key_from_mem(const uint8_t *__restrict__ base, uint64_t o, uint32_t L,
                                                 uint32_t h) {
    const uint32_t bs = static_cast<uint32_t>(o & 3u);
    const uint32_t nw = L >> 2;
    const uint32_t ndw = (bs + L + 3) >> 2;
    const uint32_t *d = reinterpret_cast<const uint32_t *>(base + (o - bs));
    uint32_t cur = d[0];
    uint32_t k = 0;
    // The first 4 quads (keys up to ~64 B: cache keys) are requested
    // together, so a key costs one memory latency rather than one per
    // quad; the loop below continues for longer keys.
    constexpr uint32_t kPre = 4;
    u32x4a4 pre[kPre];
#pragma unroll
    for (uint32_t m = 0; m < kPre; ++m)
        if (4 * m + 4 <= nw && 4 * m + 4 < ndw) pre[m] = *reinterpret_cast<const u32x4a4 *>(d + 4 * m + 1);
#pragma unroll
    for (uint32_t m = 0; m < kPre; ++m) {
        if (!(k + 4 <= nw && k + 4 < ndw)) break;
        const u32x4a4 v = pre[m];
        h = mix(h, funnel(v.x, cur, bs));
        h = mix(h, funnel(v.y, v.x, bs));
        h = mix(h, funnel(v.z, v.y, bs));
        h = mix(h, funnel(v.w, v.z, bs));
        cur = v.w;
        k += 4;
    }
    // 4 words per step from d[k+1 .. k+4], all inside the buffer's dwords
    for (; k + 4 <= nw && k + 4 < ndw; k += 4) {
        const u32x4a4 v = *reinterpret_cast<const u32x4a4 *>(d + k + 1);
        h = mix(h, funnel(v.x, cur, bs));
        h = mix(h, funnel(v.y, v.x, bs));
        h = mix(h, funnel(v.z, v.y, bs));
        h = mix(h, funnel(v.w, v.z, bs));
        cur = v.w;
    }
    for (; k < nw; ++k) {
        const uint32_t hi = k + 1 < ndw ? d[k + 1] : 0u;
        h = mix(h, funnel(hi, cur, bs));
        cur = hi;
    }
    const uint32_t diff = L - 4 * nw;          // hash.rs:38-48
    if (diff) {
        const uint32_t hi = nw + 1 < ndw ? d[nw + 1] : 0u;
        const uint32_t t = funnel(hi, cur, bs);
        if (diff >= 3) h += ((t >> 16) & 0xffu) << 16;
        if (diff >= 2) h += ((t >> 8) & 0xffu) << 8;
        h += t & 0xffu;
        h *= kM;
        h ^= h >> 24;
    }
    return h;
}

// Hash of this lane's key of one wave-set of 64 keys (metadata already
// loaded); span is the wave's LDS stage.
__device__ __forceinline__ uint32_t hash_set(const uint8_t *__restrict__ base, uint32_t *span, bool valid,
                                             uint64_t o, uint32_t L, uint32_t sdv, uint32_t lane,
                                             uint32_t *pout, uint32_t pval, bool pst) {
    uint32_t h = sdv ^ (kM * L);  // hash.rs:25
    const uint32_t bs = static_cast<uint32_t>(o & 3u);
    const uint32_t nw = L >> 2;               // whole words, hash.rs:29
    const uint32_t ndw = (bs + L + 3) >> 2;   // dwords covering the buffer
    // Keys of a batch are usually packed (cache keys, log keys): the wave
    // stages the granules spanning its 64 keys through LDS with coalesced
    // 16-B loads, instead of 64 lanes gathering byte-aligned keys.  Waves
    // whose keys span more than kSpanBytes read keys straight from memory.
    // Candidate span from the first and the last lane of the wave (keys are
    // usually packed in order); the wave stages it only if every key lies
    // inside it.  Two lane reads and one ballot instead of two 64-bit
    // six-step shuffle reductions.
    const uint64_t act = __ballot(valid);
    const int last = act ? 63 - __builtin_clzll(act) : 0;
    const uint64_t lo = __shfl(o, 0), hi = __shfl(o + L, last);
    const uint64_t lo16 = lo & ~15ull;
    const bool inside = !L || (o >= lo && o + L <= hi);
    const bool staged = act && hi > lo && hi - lo16 <= kSpanBytes && __all(inside);  // wave-uniform
    if (staged) {
        const uint32_t nch = static_cast<uint32_t>((hi - lo16 + 15) >> 4);
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 *src = reinterpret_cast<const u32x4 *>(base + lo16);
        u32x4 *dst = reinterpret_cast<u32x4 *>(span);
        constexpr uint32_t kCh = kSpanBytes / 16 / 64;
        u32x4 t[kCh];
#pragma unroll
        for (uint32_t k = 0; k < kCh; ++k) {
            const uint32_t c = lane + 64u * k;
            if (c < nch) t[k] = __builtin_nontemporal_load(src + c);
        }
        // the previous set's result leaves after this set's loads: waiting
        // for them (vmcnt is in order) then does not wait for the store
        if (pst) *pout = pval;
#pragma unroll
        for (uint32_t k = 0; k < kCh; ++k) {
            const uint32_t c = lane + 64u * k;
            if (c < nch) dst[c] = t[k];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else if (pst) {
        *pout = pval;
    }
    if (valid && L && ndw <= kFastDw) {
        // Keys of up to ~64 B (cache keys): every dword of the key is read at
        // once (from the wave's staged span, or whole quads from memory where
        // they fit and single dwords at its end), zeros past the key; the
        // chain then runs from registers, predicated per lane.
        uint32_t w[kFastDw + 1];
        if (staged) {
            const uint32_t *sd = span + ((o - bs - lo16) >> 2);
            // every dword of the window (the span's pad keeps it inside the
            // stage): no compare and select per dword; bytes past the key
            // never reach the chain (funnel shifts by bs < 4 only take
            // bytes of w[j + 1] below 4 nw + bs, and the tail word is
            // re-read or masked to its diff bytes)
#pragma unroll
            for (uint32_t j = 0; j < kFastDw; ++j) w[j] = sd[j];
        } else {
            const uint32_t *d = reinterpret_cast<const uint32_t *>(base + (o - bs));
            w[0] = d[0];
#pragma unroll
            for (uint32_t m = 0; m < 4; ++m) {
                const uint32_t b = 4 * m + 1;
                if (b + 3 < ndw) {
                    const u32x4a4 v = *reinterpret_cast<const u32x4a4 *>(d + b);
                    w[b] = v.x;
                    w[b + 1] = v.y;
                    w[b + 2] = v.z;
                    w[b + 3] = v.w;
                } else {
#pragma unroll
                    for (uint32_t t = 0; t < 4; ++t) w[b + t] = b + t < ndw ? d[b + t] : 0u;
                }
            }
        }
        w[kFastDw] = 0u;
        uint32_t tw = 0;
        const uint32_t diff = L - 4 * nw;          // hash.rs:38-48
        // The loop is VALU-bound (wave64: 4 cycles an op): capturing the
        // tail word in it cost a compare and a select per word, so the
        // tail's two dwords are read again after it (LDS or L1)
#pragma unroll
        for (uint32_t j = 0; j < kFastDw; ++j)
            if (j < nw) h = mix(h, funnel(w[j + 1], w[j], bs));
        if (diff) {  // then nw < ndw
            uint32_t t0, t1;
            if (staged) {
                const uint32_t *sd = span + ((o - bs - lo16) >> 2);
                t0 = sd[nw];
                t1 = nw + 1 < ndw ? sd[nw + 1] : 0u;
            } else {
                const uint32_t *d = reinterpret_cast<const uint32_t *>(base + (o - bs));
                t0 = d[nw];
                t1 = nw + 1 < ndw ? d[nw + 1] : 0u;
            }
            tw = funnel(t1, t0, bs);
        }
        if (diff) {
            if (diff >= 3) h += ((tw >> 16) & 0xffu) << 16;
            if (diff >= 2) h += ((tw >> 8) & 0xffu) << 8;
            h += tw & 0xffu;
            h *= kM;
            h ^= h >> 24;
        }
    } else if (valid && L) {
        h = key_from_mem(base, o, L, h);
    }
    return h;
}

// Metadata of one wave-set: load() requests this lane's words (issued one
// set ahead), get() turns them into (offset, length, seed) when the set is
// hashed -- any cross-lane step sits there, so the prefetch never waits.
struct MetaRaw {
    uint64_t o, x;
    uint32_t L, sd;
};

// Offsets API: off[] / len[] / seed[] per key.
struct OffsetsMeta {
    const uint64_t *off;
    const uint32_t *len;
    const uint32_t *seed;
    __device__ __forceinline__ MetaRaw load(uint64_t i, uint32_t n, uint32_t) const {
        const bool v = i < n;
        MetaRaw r;
        // every lane loads (clamped; get() zeroes lanes past n)
        const uint64_t ic = v ? i : n - 1u;
        r.o = off[ic];
        r.L = len[ic];
        r.sd = seed ? seed[ic] : 0u;  // (wave-uniform)
        r.x = 0;
        return r;
    }
    __device__ __forceinline__ void get(const MetaRaw &r, uint64_t i, uint32_t n, uint32_t, uint64_t &o, uint32_t &L,
                                        uint32_t &sd) const {
        const bool v = i < n;
        o = v ? r.o : 0u;
        L = v ? r.L : 0u;
        sd = v ? r.sd : 0u;
    }
};

// Packed keys (lv_hash_batch_packed): key i = arena[b[i], b[i+1]) with n + 1
// bounds of B bytes (u32: an Arrow-style string array, u64: a large one).  A
// lane reads its start; its end is the next lane's start, and lane 63 (or
// the last key) reads the bound after it -- 4 or 8 B of metadata per key
// instead of 12.
template <typename B>
struct PackedMeta {
    const B *b;
    const uint32_t *seed;
    __device__ __forceinline__ MetaRaw load(uint64_t i, uint32_t n, uint32_t lane) const {
        const bool v = i < n;
        MetaRaw r;
        // every lane loads (clamped; get() zeroes lanes past n)
        const uint64_t ic = v ? i : n - 1u;
        r.o = static_cast<uint64_t>(b[ic]);
        r.x = static_cast<uint64_t>(b[ic + 1]);  // used by lane 63 and the last key
        r.sd = seed ? seed[ic] : 0u;
        r.L = 0;
        return r;
    }
    __device__ __forceinline__ void get(const MetaRaw &r, uint64_t i, uint32_t n, uint32_t lane, uint64_t &o,
                                        uint32_t &L, uint32_t &sd) const {
        const uint64_t nx = __shfl_down(r.o, 1);
        const uint64_t e = (lane == 63u || i + 1 >= n) ? r.x : nx;
        const bool v = i < n;
        o = v ? r.o : 0u;
        L = v ? static_cast<uint32_t>(e - r.o) : 0u;
        sd = v ? r.sd : 0u;
    }
};

// Persistent: wave w of the grid hashes wave-sets w, w + W, ... of 64 keys.
// The next set's metadata is requested before this set's keys, so its
// latency overlaps theirs: one memory round trip per set instead of two
// (a one-set-per-wave grid: meta, then span, then compute, 65 -> 71 % of
// 8 TB/s was the ceiling of that shape).
// (Round 4: an XCD-aware set order -- the logical workgroup (b % 8) * (G / 8)
// + b / 8, so that neighbouring sets, which share the 128-B lines at their
// span and metadata edges, sit on one XCD's L2 -- measured 1 % slower on the
// offsets API and 3 % on packed keys, three interleaved reps each:
// profiles/r04/ab1/.)
template <typename Meta>
__global__ void __launch_bounds__(256) hash_kernel(const uint8_t *__restrict__ base, Meta meta,
                                                   uint32_t *__restrict__ out, uint32_t n, uint32_t flags) {
    __shared__ __attribute__((aligned(16))) uint32_t span[4][kSpanBytes / 4 + kSpanPad];
    const uint32_t lane = threadIdx.x & 63u, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t W = static_cast<uint64_t>(gridDim.x) * 4u;
    uint64_t set = static_cast<uint64_t>(blockIdx.x) * 4u + wv;
    if (set * 64u >= n) return;  // wave-uniform
    MetaRaw cur = meta.load(set * 64u + lane, n, lane), nx{};
    uint32_t *pout = out, pval = 0;  // the previous set's result, stored one set late
    bool pst = false;
    for (;;) {
        const uint64_t nxt = set + W;
        const bool more = nxt * 64u < n;  // wave-uniform
        nx = meta.load(nxt * 64u + lane, n, lane);  // every lane, every set (clamped): exact waits
        const uint64_t i = set * 64u + lane;
        const bool valid = i < n;
        uint64_t o;
        uint32_t L, sd;
        meta.get(cur, i, n, lane, o, L, sd);
        const uint32_t h = hash_set(base, span[wv], valid, o, L, sd, lane, pout, pval, pst);
        pout = out + (valid ? i : 0u);
        pval = (flags & LV_HASH_SHARD) ? (h >> 28) : h;
        pst = valid;
        if (!more) {
            if (pst) *pout = pval;
            break;
        }
        __builtin_amdgcn_wave_barrier();  // this set's LDS reads precede the next stage
        set = nxt;
        cur = nx;
    }
}

// persistent grid: 8 workgroups (32 waves) per CU at most
uint32_t hash_grid(size_t n) {
    static std::atomic<int> cus_cache[64];
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64) cus = cus_cache[dev].load(std::memory_order_relaxed);
    if (cus == 0) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
        if (dev >= 0 && dev < 64) cus_cache[dev].store(cus, std::memory_order_relaxed);
    }
    const uint64_t want = (n + 255) / 256, cap = static_cast<uint64_t>(cus) * kWgsPerCu;
    return static_cast<uint32_t>(want < cap ? want : cap);
}

}  // namespace lvh

extern "C" {

uint32_t lv_hash(const uint8_t *data, size_t n, uint32_t seed) {
    uint32_t h = seed ^ (lvh::kM * static_cast<uint32_t>(n));
    size_t i = 0;
    for (; i + 4 <= n; i += 4) {
        uint32_t w;
        std::memcpy(&w, data + i, 4);  // decode_fixed_32 (little-endian host)
        h += w;
        h *= lvh::kM;
        h ^= h >> 16;
    }
    const size_t diff = n - i;
    if (diff >= 3) h += static_cast<uint32_t>(data[i + 2]) << 16;
    if (diff >= 2) h += static_cast<uint32_t>(data[i + 1]) << 8;
    if (diff >= 1) {
        h += data[i];
        h *= lvh::kM;
        h ^= h >> 24;
    }
    return h;
}

uint32_t lv_cache_shard(uint32_t hash) { return hash >> 28; }

int lv_hash_batch_device(const uint8_t *d_arena, const uint64_t *d_off, const uint32_t *d_len,
                         const uint32_t *d_seed, uint32_t *d_out, size_t n, uint32_t flags, void *stream) {
    lvgpu_internal::clear_error();
    if (n == 0) return LV_OK;
    if (!d_arena || !d_off || !d_len || !d_out) return lvgpu_internal::set_error(LV_ERR_INVALID, "null device pointer");
    if (n > 0xffffffffull) return lvgpu_internal::set_error(LV_ERR_INVALID, "more than 2^32-1 buffers per call");
    if (flags & ~LV_HASH_SHARD) return lvgpu_internal::set_error(LV_ERR_INVALID, "unknown flags");
    hipLaunchKernelGGL(lvh::hash_kernel<lvh::OffsetsMeta>, dim3(lvh::hash_grid(n)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), d_arena, lvh::OffsetsMeta{d_off, d_len, d_seed}, d_out,
                       static_cast<uint32_t>(n), flags);
    return lvgpu_internal::launch_status();
}

int lv_hash_batch_packed(const uint8_t *d_arena, const void *d_bounds, uint32_t bound_bytes, const uint32_t *d_seed,
                         uint32_t *d_out, size_t n, uint32_t flags, void *stream) {
    lvgpu_internal::clear_error();
    if (n == 0) return LV_OK;
    if (!d_arena || !d_bounds || !d_out) return lvgpu_internal::set_error(LV_ERR_INVALID, "null device pointer");
    if (n > 0xffffffffull - 1) return lvgpu_internal::set_error(LV_ERR_INVALID, "more than 2^32-2 keys per call");
    if (flags & ~LV_HASH_SHARD) return lvgpu_internal::set_error(LV_ERR_INVALID, "unknown flags");
    if (bound_bytes != 4 && bound_bytes != 8) return lvgpu_internal::set_error(LV_ERR_INVALID, "bound_bytes must be 4 or 8");
    if (reinterpret_cast<uintptr_t>(d_bounds) % bound_bytes)
        return lvgpu_internal::set_error(LV_ERR_INVALID, "bounds must be aligned to bound_bytes");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (bound_bytes == 4)
        hipLaunchKernelGGL(lvh::hash_kernel<lvh::PackedMeta<uint32_t>>, dim3(lvh::hash_grid(n)), dim3(256), 0, s, d_arena,
                           lvh::PackedMeta<uint32_t>{static_cast<const uint32_t *>(d_bounds), d_seed}, d_out,
                           static_cast<uint32_t>(n), flags);
    else
        hipLaunchKernelGGL(lvh::hash_kernel<lvh::PackedMeta<uint64_t>>, dim3(lvh::hash_grid(n)), dim3(256), 0, s, d_arena,
                           lvh::PackedMeta<uint64_t>{static_cast<const uint64_t *>(d_bounds), d_seed}, d_out,
                           static_cast<uint32_t>(n), flags);
    return lvgpu_internal::launch_status();
}

}  // extern "C"
