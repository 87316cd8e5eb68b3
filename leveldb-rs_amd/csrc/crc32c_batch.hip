// MI355X (gfx950 / CDNA4) batched CRC32C.
//
// Replaces, for many buffers at once, the per-record crc32c::extend /
// crc32c::value calls of the reference WAL (log_writer.rs:123-124,
// log_reader.rs:335-336) and the table-block checksum.  Output
// is bit-identical to crc32c.rs:42-63 (extend + optional mask).
//
// Kernel design:
//  * A group of G lanes (G in {1,4,16,64}) owns one buffer at a time; a
//    wave holds 64/G groups.  Lane i of a group loads the i-th 16-B granule of
//    every "row" of G granules with one global_load_dwordx4, so a row is one
//    contiguous, coalesced run of 16*G bytes.  Rows are aligned to the END of
//    the buffer, except in the offsets API's G = 16 walk, where they sit on
//    the absolute 256-B grid (merge_al); granules outside the buffer read as
//    zeros (leading zeros leave a zero CRC register unchanged).
//  * Per lane: p = R(0, granule) by four slice-by-4 steps; across batches of
//    U rows A_i = Shift_{16GU}(A_i) ^ p_i (Horner), then the rows merge and
//    the lanes combine pairwise, X_l = Shift_{16*2^k}(X_l) ^ X_{l+2^k},
//    k < log2 G.  The < 16 bytes after the last whole granule fold in as one
//    shifted granule (fold_tail).
//  * The seed enters by xoring (seed ^ ~0) into the first 4 buffer bytes:
//    R(s, w||D) = R(0, (s^w)||D).  Buffers shorter than 4 bytes go bytewise.
//  * Lookup tables live in LDS.  The slice tables T0..T3 and the row-shift
//    tables use a "Latin-square" replicated layout: entry e of table k, copy
//    c sits in dword (4c+k) (+32 for the second set) of a 256-B row e.  In
//    lookup instruction i, lane g (of a 32-lane LDS group; c = g&7, q = g>>3)
//    reads table (q+i)&3, so the 32 lanes of every ds_read_b32 hit 32
//    distinct banks: conflict-free random lookups.  The address (row e from a
//    state byte, dword from the lane) is ONE v_perm_b32.
//  * Persistent grid: one 1024-thread workgroup per CU; the 152 KiB table
//    image plus 8 KiB of result staging fill the CU's 160 KiB of LDS.
//
// No MFMA: the work is one table lookup per byte, bound by HBM read
// bandwidth (roofline in DESIGN.md).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "../../include/lvgpu/crc32c.h"
#include "../../include/lvgpu/table.h"
#include "../../include/lvgpu/wal.h"
#include "crc32c_gf2.h"
#include "lv_internal.h"

namespace lvk {

constexpr int kThreads = 1024;  // 16 waves: 4 per SIMD, one workgroup per CU
constexpr int kWaves = kThreads / 64;
constexpr uint32_t U = 4;       // rows per batch (= interleaved Horner accumulators)

// LDS image (bytes):
//   [0, 64K)      region A, 256 rows x 256 B: dwords 0..31 T0..T3 (Latin),
//                 dwords 32..63 W4 = Shift_{16*G*U} (Latin)
//   [64K, 128K)   region B: dwords 0..31 W1 = Shift_{16*G}, 32..63 W2 = Shift_{32*G}
//   [128K, 152K)  combine tables Shift_{16*2^k}, k = 0..5, plain byte tables
constexpr uint32_t kRegionA = 0;
constexpr uint32_t kRegionB = 65536;
constexpr uint32_t kHalf = 128;  // second table set of a region: +32 dwords
constexpr uint32_t kComb = 131072;
constexpr int kImageWords = (131072 + 6 * 4 * 1024) / 4;  // 38912 dwords = 152 KiB

__shared__ __attribute__((aligned(16))) uint32_t g_lds[kImageWords];

// Per-wave output staging (8 KiB; with the image, exactly the 160 KiB of a
// CU).  Results go to LDS and leave in one global store per wave every few
// rounds.  A global store in the batch loop costs a pipeline drain: on gfx9
// stores count in vmcnt, the register allocator soon reuses the store's
// registers, and waiting for the store waits (in order) for every prefetch
// load issued before it.
__shared__ uint32_t g_oidx[kWaves][64];
__shared__ uint32_t g_ocrc[kWaves][64];
static_assert(sizeof(uint32_t) * (kImageWords + 2 * kWaves * 64) <= 163840, "LDS budget");

// Per-lane lookup constants: lv byte i = 4*beta_i (dword of the lane's table
// copy for lookup instruction i); sel_i moves that byte to bits 0..7 and the
// state byte that indexes table k_i to bits 8..15 (v_perm selector: 0-3 = S1
// bytes, 4-7 = S0 bytes, 12 = 0x00).
struct Lut {
    uint32_t lv, sel0, sel1, sel2, sel3;
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
    return L;
}

__device__ __forceinline__ uint32_t lds_word(uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(g_lds) + byte_addr);
}

// a ^ b ^ c in ONE v_bitop3_b32 (gfx950; truth table 0x96).  The lookup XOR
// trees are most of the kernel's VALU work, and VALU issue (4 cycles per
// wave64 instruction per SIMD) is one of the resources that bound it.
#ifndef LVK_XOR3
#define LVK_XOR3 1
#endif
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if LVK_XOR3
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
    return a ^ b ^ c;
#endif
}

// XOR of the four Latin tables at byte offset OFF indexed by the bytes of s.
// OFF = 0 is one slice-by-4 step T3[b0]^T2[b1]^T1[b2]^T0[b3]; the shift
// regions hold S[3-k] at table slot k so the same selectors index them.
template <uint32_t OFF>
__device__ __forceinline__ uint32_t lookup4(uint32_t s, const Lut &L) {
    const uint32_t a0 = __builtin_amdgcn_perm(s, L.lv, L.sel0);
    const uint32_t a1 = __builtin_amdgcn_perm(s, L.lv, L.sel1);
    const uint32_t a2 = __builtin_amdgcn_perm(s, L.lv, L.sel2);
    const uint32_t a3 = __builtin_amdgcn_perm(s, L.lv, L.sel3);
    return xor3(lds_word(a0 + OFF), lds_word(a1 + OFF), lds_word(a2 + OFF)) ^ lds_word(a3 + OFF);
}

// lookup4 ^ x with two 3-input XORs.
template <uint32_t OFF>
__device__ __forceinline__ uint32_t lookup4x(uint32_t s, uint32_t x, const Lut &L) {
    const uint32_t a0 = __builtin_amdgcn_perm(s, L.lv, L.sel0);
    const uint32_t a1 = __builtin_amdgcn_perm(s, L.lv, L.sel1);
    const uint32_t a2 = __builtin_amdgcn_perm(s, L.lv, L.sel2);
    const uint32_t a3 = __builtin_amdgcn_perm(s, L.lv, L.sel3);
    return xor3(xor3(lds_word(a0 + OFF), lds_word(a1 + OFF), lds_word(a2 + OFF)), lds_word(a3 + OFF), x);
}

// R(0, 16 bytes of v): four slice-by-4 steps.
__device__ __forceinline__ uint32_t r0_granule(uint4 v, const Lut &L) {
    uint32_t s = lookup4x<kRegionA>(v.x, v.y, L);
    s = lookup4x<kRegionA>(s, v.z, L);
    s = lookup4x<kRegionA>(s, v.w, L);
    return lookup4<kRegionA>(s, L);
}

// Address of lookup i of state s (one v_perm_b32).
template <int I>
__device__ __forceinline__ uint32_t lut_addr(uint32_t s, const Lut &L) {
    const uint32_t sel = I == 0 ? L.sel0 : I == 1 ? L.sel1 : I == 2 ? L.sel2 : L.sel3;
    return __builtin_amdgcn_perm(s, L.lv, sel);
}

// Shift_{16*2^k}(a) from the plain combine tables.
__device__ __forceinline__ uint32_t comb_shift(uint32_t a, int k) {
    const uint32_t *t = g_lds + (kComb / 4) + k * 1024;
    return t[a & 0xffu] ^ t[256 + ((a >> 8) & 0xffu)] ^ t[512 + ((a >> 16) & 0xffu)] ^
           t[768 + (a >> 24)];
}

// The U granules of a batch folded step-major: every slice-by-4 step issues
// the 4U lookups of all U chains (plus, in step 0, the U row-shift lookups of
// the accumulators) before consuming any, so 4U+ LDS reads are in flight per
// wave instead of one chain's 4.  p[i] = R(0, v[i]); A[i] = W4(A[i]) ^ p[i]
// (or A[i] = p[i] when FIRST).
// W4K < 0: W4 = the Latin half of region A (Shift_{64G} for the image's G);
// W4K = k >= 0: W4 = plain combine table k (Shift_{16*2^k}) -- how groups of
// G = 1 and 4 run on a G = 16 image (Shift_64 = k 2, Shift_256 = k 4).
// Experiment switches (wrong CRCs; timing studies only, never built into
// the product library, tools/build_variant.sh): LVK_EXP_NOSHIFT drops the
// row-shift lookups, LVK_EXP_NOFOLD all lookups (the load structure alone),
// LVK_EXP_NOSTAGE the blocks kernel's table staging.
#ifndef LVK_EXP_NOSHIFT
#define LVK_EXP_NOSHIFT 0
#endif
#ifndef LVK_EXP_NOFOLD
#define LVK_EXP_NOFOLD 0
#endif
#ifndef LVK_STAGGER  // s_sleep(32) units between the start of successive waves (blocks kernel, >= 8 KiB)
#define LVK_STAGGER 1u
#endif
#ifndef LVK_EXP_NOSTAGE
#define LVK_EXP_NOSTAGE 0
#endif
// The LVK_EXP_* switches compute WRONG CRCs: a build that sets one must say
// so explicitly (tools/build_variant.sh passes LVK_EXPERIMENT_BUILD=1 and
// names the library a variant), so they can never reach the product library.
// Sorted-walk studies: LVK_EXP_NOTAIL skips the tail granule's fold,
// LVK_EXP_NOFIX the head/end fix-ups of a round's rows, LVK_EXP_NOMERGE the
// merge lookups (rows XORed) and the lane rotation.
#ifndef LVK_EXP_NOTAIL
#define LVK_EXP_NOTAIL 0
#endif
#ifndef LVK_EXP_NOFIX
#define LVK_EXP_NOFIX 0
#endif
#ifndef LVK_EXP_NOMERGE
#define LVK_EXP_NOMERGE 0
#endif
#ifndef LVK_EXP_NOSEALWRITE  // the seal computes its trailers but stores none
#define LVK_EXP_NOSEALWRITE 0
#endif
#if (LVK_EXP_NOSHIFT || LVK_EXP_NOFOLD || LVK_EXP_NOSTAGE || LVK_EXP_NOTAIL || LVK_EXP_NOFIX || LVK_EXP_NOMERGE || \
     LVK_EXP_NOSEALWRITE) && \
    !defined(LVK_EXPERIMENT_BUILD)
#error "LVK_EXP_* timing switches compute wrong CRCs; define LVK_EXPERIMENT_BUILD for an experiment variant"
#endif
// NU rows per batch; W4OFF = LDS offset of the Latin row-shift table (the
// image's W4 = Shift_{64G}, or region B's W2 = Shift_{32G} for NU = 2).
// SKIP (FIRST batches only): the leading rows that hold no buffer byte for
// any group of the wave are not folded (their accumulators start at 0, as a
// fold of zero granules would leave them).
template <bool FIRST, int W4K = -1, uint32_t NU = U, uint32_t W4OFF = kRegionA + kHalf, uint32_t SKIP = 0>
__device__ __forceinline__ void fold_batch(const uint4 (&v)[NU], uint32_t (&A)[NU], const Lut &L) {
    static_assert(SKIP == 0 || FIRST, "only a first batch skips rows");
    static_assert(SKIP < NU, "at least one row");
#if LVK_EXP_NOFOLD  // experiment only: no lookups at all (load-structure bound)
#pragma unroll
    for (uint32_t i = 0; i < NU; ++i) A[i] = (FIRST ? 0u : A[i]) ^ xor3(v[i].x, v[i].y, v[i].z) ^ v[i].w;
    return;
#endif
    uint32_t s[NU], w[NU], w3[NU];
#pragma unroll
    for (uint32_t i = 0; i < NU; ++i) s[i] = v[i].x;
    if constexpr (SKIP > 0) {
#pragma unroll
        for (uint32_t i = 0; i < SKIP; ++i) A[i] = 0u;
    }
    if constexpr (!FIRST && W4K >= 0) {
#pragma unroll
        for (uint32_t i = 0; i < NU; ++i) {
            w[i] = comb_shift(A[i], W4K);
            w3[i] = 0u;
        }
    } else if constexpr (!FIRST && LVK_EXP_NOSHIFT) {  // experiment only: wrong CRCs
#pragma unroll
        for (uint32_t i = 0; i < NU; ++i) {
            w[i] = A[i];
            w3[i] = 0u;
        }
    } else if constexpr (!FIRST) {
        uint32_t aa[NU][4];
#pragma unroll
        for (uint32_t i = 0; i < NU; ++i) {
            aa[i][0] = lut_addr<0>(A[i], L);
            aa[i][1] = lut_addr<1>(A[i], L);
            aa[i][2] = lut_addr<2>(A[i], L);
            aa[i][3] = lut_addr<3>(A[i], L);
        }
#pragma unroll
        for (uint32_t i = 0; i < NU; ++i) {
            w[i] = xor3(lds_word(aa[i][0] + W4OFF), lds_word(aa[i][1] + W4OFF),
                        lds_word(aa[i][2] + W4OFF));
            w3[i] = lds_word(aa[i][3] + W4OFF);
        }
    }
#pragma unroll
    for (uint32_t step = 0; step < 4; ++step) {
        uint32_t ad[NU][4];
#pragma unroll
        for (uint32_t i = SKIP; i < NU; ++i) {
            ad[i][0] = lut_addr<0>(s[i], L);
            ad[i][1] = lut_addr<1>(s[i], L);
            ad[i][2] = lut_addr<2>(s[i], L);
            ad[i][3] = lut_addr<3>(s[i], L);
        }
        uint32_t t[NU][4];
#pragma unroll
        for (uint32_t i = SKIP; i < NU; ++i)
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) t[i][k] = lds_word(ad[i][k] + kRegionA);
#pragma unroll
        for (uint32_t i = SKIP; i < NU; ++i) {
            const uint32_t x = xor3(t[i][0], t[i][1], t[i][2]);
            if (step < 3) {
                const uint32_t nw = step == 0 ? v[i].y : step == 1 ? v[i].z : v[i].w;
                s[i] = xor3(x, t[i][3], nw);
            } else if constexpr (FIRST) {
                A[i] = x ^ t[i][3];
            } else {  // A = W4(A) ^ R(0, granule): 8 terms in four ops
                A[i] = x ^ xor3(t[i][3], w[i], w3[i]);
            }
        }
    }
}


// One byte through T0 (this lane's copy): crc32c.rs:81.
__device__ __forceinline__ uint32_t byte_step(uint32_t s, uint32_t b) {
    const uint32_t c4 = (__lane_id() & 7u) * 4u;
    const uint32_t e = (s ^ b) & 0xffu;
    return g_lds[e * 64u + c4] ^ (s >> 8);
}

// Head fix-up of one word at byte offset rel from the buffer start: bytes
// before the buffer become 0 and buffer bytes 0..3 get s0 xored in.
// Branch-free (selects); only executed for lanes that hold head bytes.
__device__ __forceinline__ uint32_t fix_word(uint32_t w, int32_t rel, uint32_t s0) {
    const int32_t z = -rel;  // leading bytes of the word that precede the buffer
    const uint32_t keep = z <= 0 ? 0xffffffffu : (z >= 4 ? 0u : 0xffffffffu << (8 * z));
    const uint32_t sx =
        (rel >= 4 || rel <= -4) ? 0u : (rel >= 0 ? s0 >> (8 * rel) : s0 << (8 * z));
    return (w & keep) ^ sx;
}

// Global (address space 1) loads: global_load_* counts only in vmcnt, so
// outstanding HBM loads never hold up the LDS lookups' lgkmcnt waits (a flat
// load would count in both).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 g_u32x4;

__device__ __forceinline__ uint4 to_uint4(u32x4 v) { return make_uint4(v.x, v.y, v.z, v.w); }

// Payload loads are non-temporal (global_load_dwordx4 ... nt): every byte is
// read exactly once, and keeping the stream out of L2/MALL measured +13-15 %
// on the 1 GiB configuration (tools/crc_ideal_probe.hip).
__device__ __forceinline__ uint4 load16(uint64_t addr) {
    return to_uint4(__builtin_nontemporal_load(reinterpret_cast<g_u32x4 *>(addr)));
}

// Default-policy (L2-allocating) 16-B load.
__device__ __forceinline__ uint4 load16_rt(uint64_t addr) {
    return to_uint4(*reinterpret_cast<g_u32x4 *>(addr));
}

// Row loads of the general kernels: non-temporal, except the last row of a
// batch, whose last 128-B line the next batch's first row shares when the
// buffer end is not line aligned (rows are aligned to the buffer END): a
// default-policy load keeps that line in L2 for the second reader (C2 HBM
// traffic 1.146x -> 1.045x of the payload).
template <uint32_t I>
__device__ __forceinline__ uint4 load_row(uint64_t addr) {
    if constexpr (I == U - 1) return load16_rt(addr);
    return load16(addr);
}

__device__ __forceinline__ uint32_t mask_crc(uint32_t c) {  // crc32c.rs:54-57
    return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}

struct Params {
    uint64_t base;  // arena address
    const uint64_t *off;
    const uint32_t *len;
    const uint32_t *seed;
    uint32_t *out;
    uint64_t n;
    uint64_t stride;
    uint32_t blen;
    uint32_t flags;
    uint64_t plen;    // long-block split (blocks kernel, PIECES): bytes per piece
    uint32_t pshift;  // log2 pieces per block
    const uint4 *ent;       // optional: sorted entries {off lo, off hi, len, buffer index}
    const uint32_t *sseed;  // optional: seeds in sorted-entry order
    uint64_t nplain;        // sorted walk: entries [nplain, n) are long-buffer pieces
    uint32_t *part;         // piece registers (long-buffer split of the offsets API)
    const uint32_t *mats;   // blocks kernel, FUSE: Shift_{j plen}, j < 2^pshift (32 column words each)
};

// Geometry of one buffer [a, a+len) on the 16-B granule grid.  Batches of
// U rows x G granules end at the last whole granule, so every batch is full;
// granules of batch 0 that precede the buffer are fixed up to zero.
// Granule index g is expressed relative to g0 = a >> 4: d = g - g0.
struct Geo {
    uint64_t abase;  // a & ~15 (address of granule g0)
    uint32_t bid;    // buffer index (output slot)
    uint32_t len;
    uint32_t seed;
    uint32_t nb;     // batches, >= 1
    int32_t hoff;    // d of batch 0 row 0 lane 0, in (-G*U, 0]
    uint32_t alow;   // a & 15, | 16 if batch 1 also holds head bytes
};

template <int G>
__device__ __forceinline__ Geo make_geo(uint64_t a, uint32_t len, uint32_t seed) {
    constexpr int32_t GU = G * static_cast<int32_t>(U);
    Geo q;
    q.abase = a & ~static_cast<uint64_t>(15);
    q.len = len;
    q.seed = seed;
    const uint32_t alow = static_cast<uint32_t>(a & 15u);
    const int32_t ng = static_cast<int32_t>(((alow + len) >> 4));  // whole granules from g0
    const int32_t nb = ng > 0 ? (ng + GU - 1) / GU : 1;
    q.nb = static_cast<uint32_t>(nb);
    q.hoff = ng - GU * nb;
    const bool fix2 = nb > 1 && q.hoff == -(GU - 1) && alow > 12u;  // seed spills into batch 1
    q.alow = alow | (fix2 ? 16u : 0u);
    return q;
}

template <int G, bool STRIDED>
__device__ __forceinline__ Geo fetch_geo(const Params &P, uint64_t i) {
    Geo q;
    uint64_t b = i;
    if constexpr (STRIDED) {
        q = make_geo<G>(P.base + b * P.stride, P.blen, P.seed ? P.seed[b] : 0u);
    } else if (P.ent) {  // one sequential 16-B load instead of idx -> off/len
        const uint4 e = P.ent[i];
        b = e.w;
        q = make_geo<G>(P.base + ((static_cast<uint64_t>(e.y) << 32) | e.x), e.z, P.seed ? P.seed[b] : 0u);
    } else {
        q = make_geo<G>(P.base + P.off[b], P.len[b], P.seed ? P.seed[b] : 0u);
    }
    q.bid = static_cast<uint32_t>(b);
    return q;
}

// Batch j >= 1: all rows lie inside the buffer.
template <int G>
__device__ __forceinline__ void load_batch(const Geo &q, uint32_t j, uint32_t gl, uint4 (&v)[U]) {
    const int32_t d = q.hoff + static_cast<int32_t>(G * U * j + gl);
    const uint64_t p = q.abase + (static_cast<int64_t>(d) << 4);
    v[0] = load_row<0>(p);
    v[1] = load_row<1>(p + 16u * G);
    v[2] = load_row<2>(p + 32u * G);
    v[3] = load_row<3>(p + 48u * G);
}

// Batch 0: rows before the buffer are clamped to granule g0 (a valid
// address); fix_head zeroes them afterwards.
template <int G>
__device__ __forceinline__ void load_batch0(const Geo &q, uint32_t gl, uint4 (&v)[U]) {
#pragma unroll
    for (uint32_t i = 0; i < U; ++i) {
        int32_t d = q.hoff + static_cast<int32_t>(G * i + gl);
        d = d < 0 ? 0 : d;
        const uint64_t a = q.abase + (static_cast<uint32_t>(d) << 4);
        v[i] = i == U - 1 ? load16_rt(a) : load16(a);
    }
}

// The tail granule (bytes after the last whole granule), lane 0 only.
__device__ __forceinline__ uint4 load_tail(const Geo &q, uint32_t gl) {
    const uint32_t end = (q.alow & 15u) + q.len;
    if (gl == 0 && (end & 15u)) return load16(q.abase + (end & ~15u));
    return make_uint4(0, 0, 0, 0);
}

// Head bytes of batch j: the granule g0 (d == 0) loses its pre-buffer bytes
// and takes the seed in buffer bytes 0..3; g0+1 (d == 1) takes the seed bytes
// that spill past g0 when a % 16 > 12.  Only those lanes run the fix-up.
template <int G>
__device__ __forceinline__ void fix_head(const Geo &q, uint32_t j, uint32_t gl, uint4 (&v)[U]) {
    const uint32_t s0 = q.len >= 4 ? ~q.seed : 0u;
    const int32_t alow = static_cast<int32_t>(q.alow & 15u);
#pragma unroll
    for (uint32_t i = 0; i < U; ++i) {
        const int32_t d = q.hoff + static_cast<int32_t>(G * (U * j + i) + gl);
        if (d == 0 || (d == 1 && alow > 12)) {
            const int32_t rel = d * 16 - alow;
            v[i].x = fix_word(v[i].x, rel, s0);
            v[i].y = fix_word(v[i].y, rel + 4, s0);
            v[i].z = fix_word(v[i].z, rel + 8, s0);
            v[i].w = fix_word(v[i].w, rel + 12, s0);
        }
    }
}

// Batch 0 rows that lie wholly before the buffer (d < 0) were loaded from a
// clamped address; they contribute nothing.
template <int G>
__device__ __forceinline__ void drop_pre_rows(const Geo &q, uint32_t gl, uint32_t (&A)[U]) {
#pragma unroll
    for (uint32_t i = 0; i < U; ++i)
        if (q.hoff + static_cast<int32_t>(G * i + gl) < 0) A[i] = 0u;
}

// Finish a buffer: merge the U row accumulators, combine the G lanes, fold
// the tail bytes, apply the short-buffer seed and store (lane 0).
template <int G>
__device__ __forceinline__ void finish(const Params &P, const Geo &q, const uint32_t (&A)[U],
                                       const uint4 &tail, uint32_t gl, const Lut &L) {
    // X = W3(A0) ^ W2(A1) ^ W1(A2) ^ A3 = W2(W1(A0) ^ A1) ^ (W1(A2) ^ A3)
    const uint32_t x01 = lookup4<kRegionB>(A[0], L) ^ A[1];
    const uint32_t x23 = lookup4<kRegionB>(A[2], L) ^ A[3];
    uint32_t X = lookup4<kRegionB + kHalf>(x01, L) ^ x23;
#pragma unroll
    for (int k = 0; (1 << k) < G; ++k) {
        const uint32_t other = __shfl_down(X, 1u << k, G);
        X = comb_shift(X, k) ^ other;
    }
    const uint32_t alow = q.alow & 15u;
    const uint32_t end = alow + q.len;
    if (gl == 0 && ((end & 15u) != 0 || q.len < 4)) {
        const uint32_t tb = end & ~15u;  // tail granule start, relative to abase
        const uint32_t hi = end - tb;
        const uint32_t lo = alow > tb ? alow - tb : 0u;
        const uint32_t s0 = q.len >= 4 ? ~q.seed : 0u;
        const uint32_t tw[4] = {tail.x, tail.y, tail.z, tail.w};
        for (uint32_t i = lo; i < hi; ++i) {
            uint32_t by = (tw[i >> 2] >> (8u * (i & 3u))) & 0xffu;
            const uint32_t rel = tb + i - alow;
            if (rel < 4) by ^= (s0 >> (8u * rel)) & 0xffu;
            X = byte_step(X, by);
        }
        if (q.len < 4) {  // R(s, D) = R(0, D) ^ Shift_|D|(s) for the unseeded short path
            uint32_t s = ~q.seed;
            for (uint32_t i = 0; i < q.len; ++i) s = byte_step(s, 0u);
            X ^= s;
        }
    }
    if (gl == 0) {
        const uint32_t crc = ~X;
        P.out[q.bid] = (P.flags & LV_CRC_MASK) ? mask_crc(crc) : crc;
    }
}

// Per-group streaming state.  The load side runs exactly one batch ahead of
// the fold side: batch j+1 of the current buffer, or batch 0 of the next
// buffer when j is the last batch.
template <int G>
struct Stream {
    Geo q, qn;        // current / next buffer (qn valid iff b + gstride < n)
    uint64_t b;       // logical index of q
    uint4 tail;       // tail granule of q (lane 0 only)
    uint32_t A[U];
    uint32_t j;
};

template <int G, bool STRIDED>
__device__ __forceinline__ bool stream_step(const Params &P, uint64_t gstride, uint32_t gl, const Lut &L,
                                            Stream<G> &S, uint4 (&cur)[U], uint4 (&nxt)[U]) {
    const bool last = S.j + 1 == S.q.nb;
    const bool has_next = S.b + gstride < P.n;
    if (!last)
        load_batch<G>(S.q, S.j + 1, gl, nxt);
    else if (has_next)
        load_batch0<G>(S.qn, gl, nxt);
    // One fold variant for every batch (accumulators start at 0 and
    // Shift(0) = 0), so groups of a wave at different batch indices never
    // run two fold bodies; only the light head fix-up is divergent.
    if (S.j == 0)
        fix_head<G>(S.q, 0, gl, cur);
    else if (S.j == 1 && (S.q.alow & 16u))
        fix_head<G>(S.q, 1, gl, cur);
    fold_batch<false>(cur, S.A, L);
    if (S.j == 0) drop_pre_rows<G>(S.q, gl, S.A);
    if (!last) {
        ++S.j;
        return false;
    }
    finish<G>(P, S.q, S.A, S.tail, gl, L);
#pragma unroll
    for (uint32_t i = 0; i < U; ++i) S.A[i] = 0u;
    if (!has_next) return true;
    S.b += gstride;
    S.q = S.qn;
    S.tail = load_tail(S.q, gl);  // needed only at this buffer's finish
    if (S.b + gstride < P.n) S.qn = fetch_geo<G, STRIDED>(P, S.b + gstride);
    S.j = 0;
    return false;
}

// One group streams buffers gid, gid + gstride, ...  The loop shape is the
// one that fits 128 VGPRs (16 waves/CU) without spills for each G: a
// ping-pong of two register slots for G = 1, a copy of the prefetched batch
// (16 moves) for G > 1, where the doubled inlined fold of a ping-pong spills.
template <int G, bool STRIDED>
__device__ __forceinline__ void group_stream(const Params &P, uint64_t gid, uint64_t gstride,
                                             uint32_t gl, const Lut &L) {
    if (gid >= P.n) return;
    Stream<G> S;
#pragma unroll
    for (uint32_t i = 0; i < U; ++i) S.A[i] = 0u;
    S.b = gid;
    S.q = fetch_geo<G, STRIDED>(P, S.b);
    if (gid + gstride < P.n) S.qn = fetch_geo<G, STRIDED>(P, gid + gstride);
    S.tail = load_tail(S.q, gl);
    S.j = 0;
    uint4 cur[U], nxt[U];
    load_batch0<G>(S.q, gl, cur);
    if constexpr (G == 1) {  // ping-pong: slots swap roles, no copies
        for (;;) {
            if (stream_step<G, STRIDED>(P, gstride, gl, L, S, cur, nxt)) break;
            if (stream_step<G, STRIDED>(P, gstride, gl, L, S, nxt, cur)) break;
        }
    } else {
        for (;;) {
            if (stream_step<G, STRIDED>(P, gstride, gl, L, S, cur, nxt)) break;
#pragma unroll
            for (uint32_t i = 0; i < U; ++i) cur[i] = nxt[i];
        }
    }
}

// Copy the 152 KiB table image into LDS: every thread issues all of its
// (<= 10) 16-B loads before the first LDS store, so the copy costs about one
// L2 round trip rather than ten.
__device__ __forceinline__ void stage_tables(const uint4 *__restrict__ image) {
    constexpr int kVec = kImageWords / 4;
    constexpr int kPer = (kVec + kThreads - 1) / kThreads;
    uint4 *l4 = reinterpret_cast<uint4 *>(g_lds);
    g_u32x4 *src = reinterpret_cast<g_u32x4 *>(reinterpret_cast<uint64_t>(image));
    u32x4 r[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = threadIdx.x + k * kThreads;
        if (i < kVec) r[k] = src[i];
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = threadIdx.x + k * kThreads;
        if (i < kVec) l4[i] = to_uint4(r[k]);
    }
    __syncthreads();
}

template <int G, bool STRIDED>
__global__ __launch_bounds__(kThreads) void crc32c_batch_kernel(Params P, const uint4 *__restrict__ image) {
    // Workgroups without work leave before staging the tables (empty classes).
    if (static_cast<uint64_t>(blockIdx.x) * kWaves * (64 / G) >= P.n) return;
    stage_tables(image);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    const Lut L = make_lut(lane);
    constexpr uint32_t kGroups = 64 / G;
    const uint64_t gid = (static_cast<uint64_t>(blockIdx.x) * kWaves + wave) * kGroups + lane / G;
    const uint64_t gstride = static_cast<uint64_t>(gridDim.x) * kWaves * kGroups;
    group_stream<G, STRIDED>(P, gid, gstride, lane % G, L);
}

// Uniform-block kernel (SSTable-style fixed-size blocks): block k is
// base[k*stride, k*stride + blen) with base, stride 16-B aligned and blen a
// multiple of 16*G*U, so every block is `nb` whole batches and every group
// of a wave walks the same (block round, batch) sequence: the batch control
// is wave-uniform (scalar), there is no head/tail work, and the seed enters
// as lane 0's first word.
// Merge the U row accumulators and the G lanes of a group; lane 0 of the
// group returns the (optionally masked) CRC.
// W1K/W2K < 0: the image's Latin W1/W2 (region B); k >= 0: plain combine
// table k (for G = 1, 4 on a G = 16 image: Shift_16G, Shift_32G).
// x of lane l + 2^k.  DPP: within 16-lane rows (k < 4) one row_shl move
// (VALU, no LDS round trip); lanes past the row end read 0, and only lanes
// whose tree stays inside their group use the value, so G <= 16 groups never
// see it.  Wider steps go through ds_bpermute.  Measured: blocks kernel
// +0.4 % with DPP; class kernel -1 % (C2) / -2 % (C4), so it keeps bpermute.
template <int G, bool DPP>
__device__ __forceinline__ uint32_t lanes_down(uint32_t x, int k) {
    if constexpr (DPP) {
        switch (k) {
        case 0: return __builtin_amdgcn_mov_dpp(x, 0x101, 0xf, 0xf, true);
        case 1: return __builtin_amdgcn_mov_dpp(x, 0x102, 0xf, 0xf, true);
        case 2: return __builtin_amdgcn_mov_dpp(x, 0x104, 0xf, 0xf, true);
        case 3: return __builtin_amdgcn_mov_dpp(x, 0x108, 0xf, 0xf, true);
        default: break;
        }
    }
    return __shfl_down(x, 1u << k, G);
}

template <int G, int W1K = -1, int W2K = -1, bool DPP = false>
__device__ __forceinline__ uint32_t merge_group(const uint32_t (&A)[U], const Lut &L) {
    uint32_t x01, x23, X;
    if constexpr (W1K >= 0) {
        x01 = comb_shift(A[0], W1K) ^ A[1];
        x23 = comb_shift(A[2], W1K) ^ A[3];
    } else {
        x01 = lookup4<kRegionB>(A[0], L) ^ A[1];
        x23 = lookup4<kRegionB>(A[2], L) ^ A[3];
    }
    if constexpr (W2K >= 0)
        X = comb_shift(x01, W2K) ^ x23;
    else
        X = lookup4<kRegionB + kHalf>(x01, L) ^ x23;
#pragma unroll
    for (int k = 0; (1 << k) < G; ++k) {
        const uint32_t other = lanes_down<G, DPP>(X, k);
        X = comb_shift(X, k) ^ other;
    }
    return X;
}

__device__ __forceinline__ uint32_t final_crc(const Params &P, uint32_t X) {
    const uint32_t crc = ~X;
    return (P.flags & LV_CRC_MASK) ? mask_crc(crc) : crc;
}

// Every step issues the SAME loads (next batch, and for seeded calls the
// next block's seed) whether or not a next batch exists -- the last one
// reads the arena's first row.  The compiler's s_waitcnt counts are static:
// if one path through a step skips the prefetch, the fold of the current
// batch waits with the count of that path (vmcnt(2)..(0) after a 4-load
// prefetch) and so for the prefetch itself, serialising load and compute in
// every step.
// PIECES: the long-block split of the strided API.  Virtual block v is piece
// v & (2^pshift - 1) of block v >> pshift (plen bytes each); piece 0 takes
// the block's seed, the others start from a zero register, and the output is
// the raw register R (no final xor, no mask) for combine_pieces_kernel.
// FUSE (PIECES, <= kFuseMax pieces per block, one round: n <= 64 x grid):
// a workgroup's 64 virtual blocks are whole blocks, so it joins their pieces
// itself after one barrier -- the matrices Shift_{j plen} wait in g_oidx
// (unused by this kernel), staged with the tables -- and there is no second
// launch.
constexpr uint32_t kFuseMax = 16;  // pieces per block; kFuseMax x 33 words fit g_oidx
#ifndef LVK_FUSE_INFLIGHT
#define LVK_FUSE_INFLIGHT 1
#endif

// R = sum of the columns of m selected by the bits of v (a GF(2) matrix-vector product).
__device__ __forceinline__ uint32_t gf2_apply(const uint32_t *m, uint32_t v) {
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) r ^= (v >> j & 1u) ? m[j] : 0u;
    return r;
}

// The fused combine (FUSE): wave 0 lane l holds WG-local piece l (wave l/4,
// group l%4) -- piece k = l mod s of its block -- shifts it by Shift_{(s-1-k)
// plen} and the s lanes of a block xor; the block's first lane stores.
__device__ __forceinline__ void fuse_pieces(const Params &P, const uint32_t *fm, uint32_t (&res)[kWaves][64],
                                            uint32_t lane, uint32_t wave) {
    __syncthreads();  // every wave's piece registers are in res[w][0..3] (one round)
    if (wave != 0) return;
    const uint32_t s = 1u << P.pshift;
    const uint64_t v = static_cast<uint64_t>(blockIdx.x) * 64u + lane;
    const uint32_t k = lane & (s - 1u);
    uint32_t acc = v < P.n ? gf2_apply(fm + (s - 1u - k) * 33u, res[lane >> 2][lane & 3u]) : 0u;
    for (uint32_t d = s >> 1; d >= 1; d >>= 1) acc ^= __shfl_xor(acc, d);
    if (v < P.n && k == 0) P.out[v >> P.pshift] = final_crc(P, acc);
}
static_assert(kFuseMax * 33 <= kWaves * 64, "fused combine matrices fit g_oidx");
template <int G, bool SEEDED, bool PIECES = false, bool FUSE = false>
__global__ __launch_bounds__(kThreads) void crc32c_blocks_kernel(Params P, uint32_t nb,
                                                                 const uint4 *__restrict__ image) {
    static_assert(!FUSE || (PIECES && G == 16), "fused combine: pieces of the G = 16 kernel");
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
    constexpr uint32_t kGroups = 64 / G;
    constexpr uint64_t kRow = 16ull * G;       // bytes between rows of a batch
    constexpr uint64_t kBatch = kRow * U;      // bytes per batch
    const uint32_t gl = lane % G;
    constexpr uint32_t kW = kWaves;  // (8-16 streaming waves per CU measured alike)
    uint64_t blk = (static_cast<uint64_t>(blockIdx.x) * kW + wave) * kGroups + lane / G;
    const uint64_t gstride = static_cast<uint64_t>(gridDim.x) * kW * kGroups;
    // Rounds of blocks are wave-uniform: the wave runs while its first group
    // has a block; groups past the end are masked.
    const uint64_t wblk0 = (static_cast<uint64_t>(blockIdx.x) * kW + wave) * kGroups;
    const uint64_t pmask = (1ull << P.pshift) - 1;
    auto block_ptr = [&](uint64_t k) {
        const uint64_t kk = k < P.n ? k : 0;
        if constexpr (PIECES) return P.base + (kk >> P.pshift) * P.stride + (kk & pmask) * P.plen + 16u * gl;
        return P.base + kk * P.stride + 16u * gl;
    };
    // the word xored into lane 0's first word of block k: ~seed (0 -> ~0)
    // for a whole block or a first piece, 0 for a later piece (raw R(0, .))
    auto seed_ld = [&](uint64_t k) -> uint32_t {
        const uint64_t kk = k < P.n ? k : 0;
        if constexpr (PIECES) {
            const uint32_t sd = SEEDED ? ~P.seed[kk >> P.pshift] : 0xffffffffu;
            return (kk & pmask) ? 0u : sd;
        }
        return ~P.seed[kk];
    };
    constexpr bool kVarS0 = SEEDED || PIECES;

    // The first batch (and seed) is requested before the table image is
    // staged, so its HBM latency overlaps the staging.
    uint64_t ptr = block_ptr(blk);
    uint32_t s0 = kVarS0 ? seed_ld(blk) : 0xffffffffu;
    uint32_t s0n = s0;
    uint4 slot0[U], slot1[U];
#pragma unroll
    for (uint32_t i = 0; i < U; ++i) slot0[i] = load16(ptr + kRow * i);
    uint32_t *const fm = &g_oidx[0][0];  // FUSE: matrix j at word 33 j (distinct banks per lane)
    if constexpr (FUSE) {
        const uint32_t nw = (1u << P.pshift) * 32u;
        for (uint32_t i = threadIdx.x; i < nw; i += kThreads) fm[(i >> 5) * 33 + (i & 31u)] = P.mats[i];
    }
#if !LVK_EXP_NOSTAGE
    stage_tables(image);
#endif
    if (wblk0 >= P.n) {
        if constexpr (FUSE) fuse_pieces(P, fm, g_ocrc, lane, wave);  // the barrier is workgroup-wide
        return;
    }
    if constexpr (PIECES && LVK_FUSE_INFLIGHT) {
        // One round of <= 4 batches per group (pieces of <= 4 KiB): every
        // batch's loads in flight at once -- one memory round trip for the
        // whole walk, where the one-ahead prefetch of the loop below pays one
        // per batch (a 64 MiB call is 4 batches per wave).  1,024 x 64 KiB:
        // 17.4 -> 16.8 us.  (Requesting batches 1-3 before the table staging
        // too spills 68-80 VGPRs.)  The fused join always has one round; the
        // two-launch split has one when the pieces fill at most one pass.
        if (nb <= U && (FUSE || wblk0 + gstride >= P.n)) {
            uint4 v1[U], v2[U], v3[U];
#pragma unroll
            for (uint32_t i = 0; i < U; ++i) {
                v1[i] = load16(ptr + kBatch * (nb > 1 ? 1u : 0u) + kRow * i);
                v2[i] = load16(ptr + kBatch * (nb > 2 ? 2u : 0u) + kRow * i);
                v3[i] = load16(ptr + kBatch * (nb > 3 ? 3u : 0u) + kRow * i);
            }
            const Lut L = make_lut(lane);
            uint32_t A[U];
            if (gl == 0) slot0[0].x ^= kVarS0 ? seed_ld(blk) : 0xffffffffu;
            fold_batch<true>(slot0, A, L);
            if (nb > 1) fold_batch<false>(v1, A, L);
            if (nb > 2) fold_batch<false>(v2, A, L);
            if (nb > 3) fold_batch<false>(v3, A, L);
            const uint32_t X = merge_group<G, -1, -1, true>(A, L);
            if constexpr (FUSE) {
                if (gl == 0) g_ocrc[wave][lane / G] = X;
                fuse_pieces(P, fm, g_ocrc, lane, wave);
            } else {
                if (gl == 0 && blk < P.n) P.out[blk] = X;  // the raw register, for combine_pieces_*
            }
            return;
        }
    }
    // Blocks of >= 8 KiB: the waves of a CU start ~0.85 us apart.  Waves that
    // start together walk their blocks in lockstep, so all 16 K concurrent
    // streams sit at the same offset within their blocks, and at 8-64 KiB
    // strides that address pattern reads 2-4 % slower (HBM address mapping:
    // padding the stride has the same effect).  4 KiB blocks run best in
    // lockstep (a stagger cost 0.5-1 % there).  Strided 8 / 16 / 64 KiB: 76.8 ->
    // 79.8, 77.7 -> 80.0, 79.8 -> 81.6 % of 8 TB/s; 32 KiB within noise.
    // Only waves with >= 64 batches to walk stagger (the last wave's delay,
    // ~13 us, is then a few batches of its work): a small batch would
    // otherwise wait out the delay.
    const uint64_t rounds = (P.n - 1 - wblk0) / gstride + 1;
    if (G == 16 && nb >= 8 && rounds * nb >= 64)
        for (uint32_t k = 0; k < wave * LVK_STAGGER; ++k) __builtin_amdgcn_s_sleep(32);
    const Lut L = make_lut(lane);
    uint32_t A[U];
    // The flush store's operands live in registers of their own for the whole
    // loop (kept live past it below), so no loop temporary reuses them: a
    // write to a pending store's source register waits for the store, i.e.
    // (vmcnt is in order) for every prefetch load issued before it.
    uint32_t st_val = 0;
    uint64_t st_ptr = 0;

    // one batch: prefetch the next batch into `nxt`, fold `cur`
    auto step = [&](uint64_t r, uint32_t j, uint4(&cur)[U], uint4(&nxt)[U]) {
        const bool lastj = j + 1 == nb;
        const bool more = !lastj || r + 1 < rounds;
        const uint64_t nptr = lastj ? block_ptr(blk + gstride) : ptr + kBatch;
        // no next batch: a dummy read of the arena's first row, the same lines
        // for every wave (L2 hits)
        const uint64_t lptr = more ? nptr : P.base + 16u * gl;
        if constexpr (kVarS0) s0n = seed_ld(blk + gstride);
#pragma unroll
        for (uint32_t i = 0; i < U; ++i) nxt[i] = load16(lptr + kRow * i);
        if (j == 0) {
            if (gl == 0) cur[0].x ^= s0;
            fold_batch<true>(cur, A, L);
        } else {
            fold_batch<false>(cur, A, L);
        }
        if (lastj) {
            // round r's K results -> LDS slot (r % G)*K + group; one store of
            // the wave's 64 slots every G rounds (and after the last round)
            const uint32_t X = merge_group<G, -1, -1, true>(A, L);
            if (gl == 0) g_ocrc[wave][(r % G) * kGroups + lane / G] = PIECES ? X : final_crc(P, X);
            if (!FUSE && ((r + 1) % G == 0 || r + 1 == rounds)) {
                __builtin_amdgcn_wave_barrier();
                const uint64_t r0 = r - r % G;
                const uint64_t k = wblk0 + (r0 + lane / kGroups) * gstride + lane % kGroups;
                st_val = g_ocrc[wave][lane];
                st_ptr = reinterpret_cast<uint64_t>(P.out + (k < P.n ? k : 0));
                if (lane < (r - r0 + 1) * kGroups && k < P.n) *reinterpret_cast<uint32_t *>(st_ptr) = st_val;
                __builtin_amdgcn_wave_barrier();
            }
            blk += gstride;
            if constexpr (kVarS0) s0 = s0n;
        }
        ptr = nptr;
    };

    const uint64_t total = rounds * nb;  // batches this wave walks
    uint64_t t = 0;
    uint64_t r = 0;
    uint32_t j = 0;
    for (;;) {
        step(r, j, slot0, slot1);
        if (++t == total) break;
        if (++j == nb) { j = 0; ++r; }
        step(r, j, slot1, slot0);
        if (++t == total) break;
        if (++j == nb) { j = 0; ++r; }
    }
    asm volatile("" ::"v"(st_val), "v"(st_ptr));
    if constexpr (FUSE) fuse_pieces(P, fm, g_ocrc, lane, wave);
}

// Length classes of the offsets API.  Buffers are counting-sorted by key =
// (class, batches descending): each class runs with the group size that keeps
// ~1-32 batches per buffer, and consecutive list entries -- the groups of one
// wave -- have the same batch count, so they finish buffers in lockstep.
constexpr uint32_t kBuckets = 64;                 // batch-count buckets per class
constexpr uint32_t kKeys = 4 * kBuckets;
constexpr uint32_t kSortThreads = 256;
constexpr uint32_t kSortE = 16;  // elements per thread per register block in the sort passes

__device__ __forceinline__ uint32_t len_class(uint32_t len) {
    return len <= 256u ? 0u : len <= 2048u ? 1u : len <= 32768u ? 2u : 3u;
}

// Rows per batch of the G = 16 classes' aligned-row walk (sorted_stream).
#ifndef LVK_AL_ROWS
#define LVK_AL_ROWS 4
#endif
#ifndef LVK_ALIGNED_ROWS
#define LVK_ALIGNED_ROWS 1
#endif
constexpr uint32_t kAlRows = LVK_ALIGNED_ROWS ? LVK_AL_ROWS : U;

__device__ __forceinline__ uint32_t sort_key(uint32_t len) {
    const uint32_t c = len_class(len);
    const uint32_t gu16 = 16u * (c >= 2 ? kAlRows : U) * (c == 0 ? 1u : c == 1 ? 4u : 16u);
    uint32_t nb = (len + gu16 - 1) / gu16;  // batches, ignoring start alignment
    nb = nb < kBuckets - 1 ? nb : kBuckets - 1;
    return c * kBuckets + (kBuckets - 1 - nb);
}

// Sort workspace, 16-B aligned.  Header (u32 words): [0, 4) the long-buffer
// split's piece and long-buffer counters and the batch's payload bytes (u64);
// [4, 256) unused; [256, 264) class start x4, count x4; [264, 520) per-key
// totals; [520, 528) unused.  Then the per-workgroup histogram matrix
// M[wgs][256], the per-workgroup payload sums (u64), n + kPieceBudget sorted
// 16-B entries (the pieces of split long buffers follow the n sorted ones),
// as many seeds in entry order, kPieceBudget piece registers and
// kPieceBudget / 2 long-buffer records {buffer, first piece, pieces, log2 piece}.
constexpr uint32_t kWsPieces = 0;
constexpr uint32_t kWsLongs = 1;
constexpr uint32_t kWsBytes = 2;
#ifndef LVK_IDENT
#define LVK_IDENT 1
#endif
constexpr uint32_t kWsIdent = 4;  // 1: the sorted list is the identity (one key, no split): see sort_scatter
constexpr uint32_t kPieceBudget = 65536;  // piece entries per call (each split buffer takes <= kMaxPieces)
#ifndef LVK_MAX_PIECES  // pieces per split buffer (a lone 16 MiB buffer: 4,096 of 4 KiB, as the strided API cuts it)
#define LVK_MAX_PIECES 4096
#endif
constexpr uint32_t kMaxPieces = LVK_MAX_PIECES;
constexpr uint32_t kPieceFlag = 0x80000000u;  // output slot flag of a piece entry (slot < kPieceBudget)
constexpr uint32_t kWsCls = kKeys;
constexpr uint32_t kWsTot = kKeys + 8;
constexpr uint32_t kWsHeader = kWsTot + kKeys + 8;  // 528 words, 16-B multiple
constexpr uint32_t kSortChunk = kSortThreads * kSortE;  // elements per sorting workgroup (n <= 4M)
constexpr uint32_t kSortMaxWgs = 1024;
constexpr uint32_t kScanWgs = kKeys / 16;  // 16 keys per scan workgroup
constexpr uint32_t kScanThreads = 1024;    // 16 keys x 64 row ranges
static_assert(kSortMaxWgs <= 64 * 16, "scan: 64 row ranges of <= 16 rows");

// h[k] += 1 for each valid lane's key k.  A wave whose valid lanes share one
// key (a uniform batch: thousands of same-address LDS atomics would
// serialize) adds its count with one atomic; otherwise each lane adds its own.
__device__ __forceinline__ void wave_count(uint32_t *h, uint32_t k, bool valid, uint32_t lane) {
    const uint64_t act = __ballot(valid);
    if (!act) return;  // wave-uniform
    const int leader = __ffsll(static_cast<long long>(act)) - 1;
    const uint32_t kl = __shfl(k, leader);
    if (__ballot(valid && k != kl) == 0) {
        if (static_cast<int>(lane) == leader) atomicAdd(&h[kl], static_cast<uint32_t>(__popcll(act)));
    } else if (valid) {
        atomicAdd(&h[k], 1u);
    }
}

// Like wave_count, but returns each valid lane's claimed slot h[k]++.
__device__ __forceinline__ uint32_t wave_claim(uint32_t *h, uint32_t k, bool valid, uint32_t lane) {
    const uint64_t act = __ballot(valid);
    if (!act) return 0;  // wave-uniform
    const int leader = __ffsll(static_cast<long long>(act)) - 1;
    const uint32_t kl = __shfl(k, leader);
    if (__ballot(valid && k != kl) == 0) {
        uint32_t base = 0;
        if (static_cast<int>(lane) == leader) base = atomicAdd(&h[kl], static_cast<uint32_t>(__popcll(act)));
        base = __shfl(base, leader);
        return base + static_cast<uint32_t>(__popcll(act & ((1ull << lane) - 1ull)));
    }
    return valid ? atomicAdd(&h[k], 1u) : 0u;
}

// Pass 1: per-workgroup key histogram of a contiguous chunk, in LDS, stored
// as row blockIdx.x of M.  No global atomics: same-address device atomics
// from hundreds of workgroups serialize (one key for a uniform batch).
__global__ __launch_bounds__(kSortThreads) void sort_hist(const uint32_t *__restrict__ len, uint64_t n,
                                                          uint64_t chunk, uint32_t *__restrict__ M,
                                                          uint32_t *__restrict__ ws, uint64_t *__restrict__ wgb) {
    static_assert(kSortThreads == kKeys, "one thread per key");
    __shared__ uint32_t h[kKeys];
    __shared__ uint64_t bsum[kSortThreads / 64];
    const uint32_t t = threadIdx.x, lane = t & 63u;
    h[t] = 0;
    if (blockIdx.x == 0 && t == 0) {  // counters of the long-buffer split (read by later launches)
        ws[kWsPieces] = 0;
        ws[kWsLongs] = 0;
    }
    uint64_t mybytes = 0;
    __syncthreads();
    const uint64_t lo = blockIdx.x * chunk, hi = lo + chunk < n ? lo + chunk : n;
    for (uint64_t b0 = lo; b0 < hi; b0 += kSortChunk) {
        uint32_t l[kSortE];  // all loads of the block first: one memory latency, not kSortE
#pragma unroll
        for (uint32_t e = 0; e < kSortE; ++e) {
            const uint64_t i = b0 + e * kSortThreads + t;
            l[e] = i < hi ? len[i] : 0u;
        }
#pragma unroll
        for (uint32_t e = 0; e < kSortE; ++e) {
            mybytes += l[e];
            if (b0 + e * kSortThreads >= hi) break;  // block-uniform
            wave_count(h, sort_key(l[e]), b0 + e * kSortThreads + t < hi, lane);
        }
    }
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) mybytes += __shfl_xor(mybytes, k);
    if (lane == 0) bsum[t >> 6] = mybytes;
    __syncthreads();
    M[static_cast<uint64_t>(blockIdx.x) * kKeys + t] = h[t];
    if (t == 0) wgb[blockIdx.x] = bsum[0] + bsum[1] + bsum[2] + bsum[3];
}

// Pass 2: column scan of M.  Workgroup b owns keys [16b, 16b+16); thread
// (sub, kl) sums rows [sub*R, sub*R+R) of key 16b+kl, the 64 partial sums
// per key are scanned in LDS (Hillis-Steele over sub), and M[w][k] becomes
// the offset of workgroup w's first key-k entry within key k; the key totals
// go to the header.  No fence or ticket: the key starts are scanned by each
// scatter workgroup after the kernel boundary (a device-scope release here
// writes back the L2 and cost more than this whole pass).
__global__ __launch_bounds__(kScanThreads) void sort_scan(uint32_t *__restrict__ M, uint32_t wgs,
                                                          uint32_t *__restrict__ ws, const uint64_t *__restrict__ wgb) {
    __shared__ uint32_t part[64][16];
    __shared__ uint64_t bsum[kScanThreads / 64];
    if (blockIdx.x == 0) {  // the batch's payload bytes (sizes the long-buffer split's pieces)
        uint64_t b = threadIdx.x < wgs ? wgb[threadIdx.x] : 0u;
#pragma unroll
        for (int k = 32; k >= 1; k >>= 1) b += __shfl_xor(b, k);
        if ((threadIdx.x & 63u) == 0) bsum[threadIdx.x >> 6] = b;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint64_t tot = 0;
            for (uint32_t w = 0; w < kScanThreads / 64; ++w) tot += bsum[w];
            ws[kWsBytes] = static_cast<uint32_t>(tot);
            ws[kWsBytes + 1] = static_cast<uint32_t>(tot >> 32);
        }
    }
    const uint32_t t = threadIdx.x, kl = t & 15u, sub = t >> 4;
    const uint32_t k = blockIdx.x * 16u + kl;
    const uint32_t R = (wgs + 63u) / 64u;  // <= 16
    const uint32_t r0 = sub * R;
    uint32_t v[16];
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t r = 0; r < 16; ++r) {
        v[r] = (r < R && r0 + r < wgs) ? M[static_cast<uint64_t>(r0 + r) * kKeys + k] : 0u;
        sum += v[r];
    }
    part[sub][kl] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < 64; d <<= 1) {  // inclusive scan over sub
        const uint32_t x = sub >= d ? part[sub - d][kl] : 0u;
        __syncthreads();
        part[sub][kl] += x;
        __syncthreads();
    }
    if (sub == 63) ws[kWsTot + k] = part[63][kl];
    uint32_t run = part[sub][kl] - sum;  // exclusive
#pragma unroll
    for (uint32_t r = 0; r < 16; ++r) {
        if (r < R && r0 + r < wgs) M[static_cast<uint64_t>(r0 + r) * kKeys + k] = run;
        run += v[r];
    }
}

// Exclusive scan of the 256 key totals (one per thread of a 256-thread
// workgroup) into sc[]; returns this thread's key start.
__device__ __forceinline__ uint32_t key_starts(const uint32_t *ws, uint32_t *sc) {
    const uint32_t t = threadIdx.x;
    const uint32_t mine = ws[kWsTot + t];
    sc[t] = mine;
    __syncthreads();
    for (uint32_t d = 1; d < kKeys; d <<= 1) {
        const uint32_t x = t >= d ? sc[t - d] : 0u;
        __syncthreads();
        sc[t] += x;
        __syncthreads();
    }
    return sc[t] - mine;
}

// Pass 3: same chunks as pass 1.  Workgroup w's slots for key k start at
// key_start[k] + M[w][k]; buffers claim them with wave-aggregated LDS
// atomics (order within a workgroup's run is not stable, which keeps metadata
// reads and CRC stores within one 4096-buffer window).  Entries carry
// off/len/index so the CRC kernel reads one 16-B record per buffer; seeds are
// permuted alongside.
// Long-buffer split of the offsets API (verdict r01: a batch of a few long
// buffers left most of the grid idle, one 16-lane group walking each).  A
// buffer longer than the larger of 16 KiB and twice its piece length is cut
// into m <= kMaxPieces pieces of P = 2^p bytes, aligned to its END (piece 0
// holds the ragged rest), with P the smallest power of two >= 4 KiB, >=
// L / kMaxPieces and >= (payload bytes of the batch) / 16,384 (one pass of
// the grid's 16-lane groups): buffers that are long relative to the batch
// are split, C2/C4-sized ones are not.  The pieces go after the n sorted
// entries (claimed with a device counter, at most kPieceBudget per call;
// a buffer that does not fit stays whole), the walk stores their raw
// registers, and combine_long_kernel joins them.  The buffer's own sorted
// entry becomes an empty one with no output.
__device__ __forceinline__ uint32_t ceil_log2(uint64_t x) {
    return x <= 1 ? 0u : 64u - static_cast<uint32_t>(__clzll(static_cast<long long>(x - 1)));
}

// Per-wave staging of the claiming lanes' geometry (sort_scatter's 4 waves).
__shared__ uint4 g_split[kSortThreads / 64][64];     // {offset lo, hi, length, seed}
__shared__ uint32_t g_split_pre[kSortThreads / 64][64];  // inclusive prefix of the piece counts
__shared__ uint32_t g_split_p[kSortThreads / 64][64];    // log2 piece length

// Called by every lane of a wave (valid: the lane holds buffer i).  Counter
// claims are wave-aggregated (one device atomic per wave and counter: the
// same-address atomics of one per buffer serialized, ~40 us for 1,024
// buffers) and each split buffer's pieces are written by the whole wave.
// Returns true on lanes whose buffer was split.
__device__ __forceinline__ bool split_wave(bool valid, uint64_t o, uint32_t L, uint32_t s, uint32_t i, uint64_t n,
                                           uint64_t total, uint32_t *__restrict__ ws, uint4 *__restrict__ ent,
                                           uint32_t *__restrict__ sseed, bool seeded, uint4 *__restrict__ longs,
                                           uint32_t lane) {
    if (!longs) return false;  // splitting is off for this call (wave-uniform)
    uint32_t m = 0, p = 0;
    if (valid && L > 16384u) {
        p = ceil_log2(total / 16384u);
        const uint32_t pl = ceil_log2((static_cast<uint64_t>(L) + kMaxPieces - 1) / kMaxPieces);
        p = p > pl ? p : pl;
        p = p > 12u ? p : 12u;
        // No lower cap than 31: P >= batch bytes / 16,384 must hold for every
        // batch (it bounds sum m <= 16,384 + 8,192 and the split buffers <= 8,192,
        // inside kPieceBudget and kPieceBudget / 2).  A split needs L > 2P and
        // L < 2^32, so split buffers have p <= 30, and the join's shifts
        // Shift_{2^i}, i <= p + lc + 5 <= 30 + 6 + 5, stay below kBaseMats.
        p = p < 31u ? p : 31u;
        if (L > (2ull << p)) m = static_cast<uint32_t>((L + (1ull << p) - 1) >> p);
    }
    const uint64_t want = __ballot(m > 0);
    if (!want) return false;  // wave-uniform
    uint32_t incl = m;  // inclusive prefix of m over the wave
#pragma unroll
    for (uint32_t k = 1; k < 64; k <<= 1) {
        const uint32_t t = __shfl_up(incl, k);
        if (lane >= k) incl += t;
    }
    const uint32_t tot = __shfl(incl, 63);
    const uint32_t nlong = static_cast<uint32_t>(__popcll(want));
    uint32_t pb = 0, lb = 0;
    if (lane == 0) {
        pb = atomicAdd(&ws[kWsPieces], tot);
        lb = atomicAdd(&ws[kWsLongs], nlong);
    }
    pb = __shfl(pb, 0);
    lb = __shfl(lb, 0);
    const uint32_t base = pb + incl - m;
    // (both limits hold by construction, since P >= batch bytes / 16,384 for
    // every batch: sum of m <= 16,384 + 8,192 and at most 8,192 buffers longer
    // than 2P >= batch bytes / 8,192 -- and are checked anyway: a claim past
    // them leaves its buffer whole)
    const uint32_t li = lb + static_cast<uint32_t>(__popcll(want & ((1ull << lane) - 1ull)));
    const bool fits = m > 0 && static_cast<uint64_t>(base) + m <= kPieceBudget && li < kPieceBudget / 2;
    if (m > 0 && li < kPieceBudget / 2)  // long record (m = 0 when not split: combine_long_kernel skips it)
        longs[li] = make_uint4(i, base, fits ? m : 0u, p);
    // the wave writes every claimed buffer's piece entries (or blanks for
    // claims past the budget, so every slot below min(counter, budget) is
    // set), lane-parallel over the wave's pieces: the claiming lanes park
    // their geometry in LDS; lane l writes slots l, l + 64, ... and walks a
    // cursor over the wave's inclusive prefix (slots only grow, so the
    // cursor moves ~once per slot: a loop over the buffers with broadcasts
    // ran ~75 us for 1,024 split buffers, a binary search per slot -- six
    // dependent LDS reads -- ~90 us for 64 x 256 pieces)
    const uint32_t w = threadIdx.x >> 6;
    g_split[w][lane] = make_uint4(static_cast<uint32_t>(o), static_cast<uint32_t>(o >> 32), L, s);
    g_split_pre[w][lane] = incl;
    g_split_p[w][lane] = p | (fits ? 0x100u : 0u);
    __builtin_amdgcn_wave_barrier();
    // Buffer j's prefix pair and geometry stay in registers and are re-read
    // only when the cursor moves (every m / 64 slots), so a slot costs no
    // dependent LDS read (with one per slot: 62 us for 64 x 256 pieces).
    uint32_t j = 0;                        // first lane with incl > u (u grows, so j only moves forward)
    uint32_t pre = g_split_pre[w][0], prv = 0;  // incl of lanes j and j - 1
    uint4 gj = g_split[w][0];
    uint32_t pj = g_split_p[w][0];
    for (uint32_t u = lane; u < tot; u += 64) {
        if (pre <= u) {
            do {
                prv = pre;
                pre = g_split_pre[w][++j];
            } while (pre <= u);
            gj = g_split[w][j];
            pj = g_split_p[w][j];
        }
        const uint32_t mj = pre - prv;
        const uint32_t k = u - prv;  // piece index within buffer j
        const uint32_t slot = pb + u;
        if (pj & 0x100u) {  // buffer j was split
            const uint64_t P = 1ull << (pj & 0xffu);
            const uint64_t first = gj.z - (static_cast<uint64_t>(mj) - 1) * P;  // piece 0: [0, first)
            // every piece is walked like a seed-0 buffer except piece 0,
            // which takes the buffer's seed: piece k > 0 yields R(~0, piece)
            // and combine_long_kernel removes the constant Shift_P(~0)
            const uint64_t a = ((static_cast<uint64_t>(gj.y) << 32) | gj.x) + (k ? first + (k - 1) * P : 0);
            ent[n + slot] = make_uint4(static_cast<uint32_t>(a), static_cast<uint32_t>(a >> 32),
                                       static_cast<uint32_t>(k ? P : first), slot | kPieceFlag);
            if (seeded) sseed[n + slot] = k ? 0u : gj.w;
        } else if (slot < kPieceBudget) {
            ent[n + slot] = make_uint4(0, 0, 0, 0xffffffffu);
        }
    }
    __builtin_amdgcn_wave_barrier();
    return fits;
}

__global__ __launch_bounds__(kSortThreads) void sort_scatter(const uint64_t *__restrict__ off,
                                                             const uint32_t *__restrict__ len, uint64_t n,
                                                             uint64_t chunk, uint32_t *__restrict__ ws,
                                                             const uint32_t *__restrict__ M,
                                                             uint4 *__restrict__ ent,
                                                             const uint32_t *__restrict__ seed,
                                                             uint32_t *__restrict__ sseed, uint4 *__restrict__ longs) {
    __shared__ uint32_t cur[kKeys];
    __shared__ uint32_t sc[kKeys];
    const uint32_t t = threadIdx.x, lane = t & 63u;
    const uint32_t mrow = M[static_cast<uint64_t>(blockIdx.x) * kKeys + t];
    const uint32_t ks = key_starts(ws, sc);
    cur[t] = ks + mrow;
    // A batch whose buffers all share one key (uniform lengths: the C3-like
    // case) is already "sorted" in index order; if none of them can be split
    // (classes 0-1 never are; class 2 only above 16 KiB and only in batches
    // of < 16,384 buffers, since a split needs L > 2P >= batch bytes / 8,192)
    // the class kernel reads off/len/seed directly and the scatter is skipped.
    const uint32_t tk = ws[kWsTot + t];
    const bool ident_key = tk == static_cast<uint32_t>(n);  // this thread's key holds every buffer
    const uint32_t kc = t / kBuckets, knb = kBuckets - 1 - t % kBuckets;
    const bool ident_ok = ident_key && (kc <= 1 || (kc == 2 && (knb <= 16 || n >= 16384)));
    const bool ident = __syncthreads_or(LVK_IDENT && ident_ok);
    if (blockIdx.x == 0 && t % kBuckets == 0) {  // per-class [start, count) for the CRC kernel
        const uint32_t c = t / kBuckets;
        ws[kWsCls + c] = ks;
        ws[kWsCls + 4 + c] = sc[t + kBuckets - 1] - ks;
    }
    if (blockIdx.x == 0 && t == 0) ws[kWsIdent] = ident ? 1u : 0u;
    if (ident) return;  // block-uniform
    __syncthreads();
    const uint64_t total = (static_cast<uint64_t>(ws[kWsBytes + 1]) << 32) | ws[kWsBytes];
    const uint64_t lo = blockIdx.x * chunk, hi = lo + chunk < n ? lo + chunk : n;
    for (uint64_t b0 = lo; b0 < hi; b0 += kSortChunk) {
        uint32_t lb[kSortE];
        uint64_t ob[kSortE];
#pragma unroll
        for (uint32_t e = 0; e < kSortE; ++e) {
            const uint64_t i = b0 + e * kSortThreads + t;
            lb[e] = i < hi ? len[i] : 0u;
            ob[e] = i < hi ? off[i] : 0u;
        }
#pragma unroll
        for (uint32_t e = 0; e < kSortE; ++e) {
            const uint64_t r0 = b0 + e * kSortThreads;
            if (r0 >= hi) break;  // block-uniform
            const uint64_t i = r0 + t;
            const bool valid = i < hi;
            const uint32_t pos = wave_claim(cur, sort_key(lb[e]), valid, lane);
            const uint32_t sd = (seed && valid) ? seed[i] : 0u;
            const bool split = split_wave(valid, ob[e], lb[e], sd, static_cast<uint32_t>(i), n, total, ws, ent, sseed,
                                          seed != nullptr, longs, lane);
            if (valid) {
                // a split buffer's own entry: empty, no output (combine_long_kernel stores it)
                ent[pos] = make_uint4(static_cast<uint32_t>(ob[e]), static_cast<uint32_t>(ob[e] >> 32),
                                      split ? 0u : lb[e], split ? 0xffffffffu : static_cast<uint32_t>(i));
                if (seed) sseed[pos] = sd;
            }
        }
    }
}

// Small batches (n <= kSmallSort): the three passes in ONE launch.  Every
// workgroup reads all n lengths (<= 4 KiB), so it knows the whole key
// histogram, the histogram of the buffers before its chunk, the batch's
// payload bytes and every buffer's split (pieces m_i, log2 piece length p_i);
// piece slots and long-record indices are index-order prefix sums instead of
// device-atomic claims, so no pass waits for another and no counter needs
// zeroing.  (By construction every split fits: P >= batch bytes / 16,384,
// so sum m <= 16,384 + n pieces and <= n long records, below the budgets.)  Each workgroup then claims its
// chunk's sorted slots, and writes an equal share of ALL the piece slots (a
// binary search over the LDS prefix finds a slot's buffer): a lone 16 MiB
// buffer is 4,096 pieces, 16 dependent rounds for the one workgroup of its
// chunk.  The chunks are the three-pass sort's; the grid is at least
// kSmallSortWgs workgroups (the extra ones write pieces only).
#ifndef LVK_SMALL_SORT
#define LVK_SMALL_SORT 1
#endif
constexpr uint32_t kSmallSort = 4 * kSortThreads;  // buffers
constexpr uint32_t kSmallSortWgs = 64;
__global__ __launch_bounds__(kSortThreads) void sort_small(const uint64_t *__restrict__ off,
                                                           const uint32_t *__restrict__ len, uint64_t n,
                                                           uint64_t chunk, uint32_t *__restrict__ ws,
                                                           uint4 *__restrict__ ent, const uint32_t *__restrict__ seed,
                                                           uint32_t *__restrict__ sseed, uint4 *__restrict__ longs) {
    __shared__ uint32_t hall[kKeys], hpre[kKeys], sc[kKeys];
    __shared__ uint32_t mpre[kSmallSort + 1];  // exclusive prefix of m over buffer index (+ total)
    __shared__ uint32_t lpre[kSmallSort + 1];  // exclusive prefix of split buffers
    __shared__ uint32_t pp[kSmallSort];        // log2 piece length of a split buffer
    __shared__ uint64_t red[kSortThreads / 64];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint64_t lo = blockIdx.x * chunk, hi = lo + chunk < n ? lo + chunk : n;
    hall[t] = 0;
    hpre[t] = 0;
    uint32_t l[4];
    uint64_t mine = 0;
#pragma unroll
    for (uint32_t e = 0; e < 4; ++e) {
        const uint64_t i = e * kSortThreads + t;
        l[e] = i < n ? len[i] : 0u;
        mine += l[e];
    }
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) mine += __shfl_xor(mine, k);
    if (lane == 0) red[w] = mine;
    __syncthreads();
    const uint64_t total = red[0] + red[1] + red[2] + red[3];
    // histograms, splits and their index-order prefixes
    uint32_t run_m = 0, run_l = 0;
#pragma unroll
    for (uint32_t e = 0; e < 4; ++e) {
        const uint64_t i = e * kSortThreads + t;
        const bool valid = i < n;
        const uint32_t k = sort_key(l[e]);
        wave_count(hall, k, valid, lane);
        wave_count(hpre, k, valid && i < lo, lane);
        uint32_t m = 0, p = 0;
        if (longs && valid && l[e] > 16384u) {  // split_wave's rule
            p = ceil_log2(total / 16384u);
            const uint32_t pl = ceil_log2((static_cast<uint64_t>(l[e]) + kMaxPieces - 1) / kMaxPieces);
            p = p > pl ? p : pl;
            p = p > 12u ? p : 12u;
            p = p < 31u ? p : 31u;  // split_wave's bound (see there)
            if (l[e] > (2ull << p)) m = static_cast<uint32_t>((l[e] + (1ull << p) - 1) >> p);
        }
        // exclusive scans over t of m and (m > 0), plus the running totals of rows e' < e
        uint32_t im = m, il = m > 0 ? 1u : 0u;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t xm = __shfl_up(im, d), xl = __shfl_up(il, d);
            if (lane >= d) {
                im += xm;
                il += xl;
            }
        }
        __syncthreads();  // red / sc reuse
        if (lane == 63) {
            sc[w] = im;
            sc[4 + w] = il;
        }
        __syncthreads();
        uint32_t bm = run_m, bl = run_l;
        for (uint32_t v = 0; v < w; ++v) {
            bm += sc[v];
            bl += sc[4 + v];
        }
        pp[i] = p;  // i < kSmallSort: e < 4, t < kSortThreads
        mpre[i] = bm + im - m;
        lpre[i] = bl + il - (m > 0 ? 1u : 0u);
        run_m += sc[0] + sc[1] + sc[2] + sc[3];
        run_l += sc[4] + sc[5] + sc[6] + sc[7];
    }
    __syncthreads();
    if (t == 0) {
        mpre[kSmallSort] = run_m;
        lpre[kSmallSort] = run_l;
    }
    // key starts (exclusive scan of the whole histogram) and this chunk's
    // slots: a wave scan, then the earlier waves' totals (2 barriers, where a
    // Hillis-Steele scan over LDS took 16)
    static_assert(kKeys == kSortThreads, "one key per thread");
    __shared__ uint32_t wtot[kSortThreads / 64];
    const uint32_t mineh = hall[t];
    uint32_t inc = mineh;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t x = __shfl_up(inc, d);
        if (lane >= d) inc += x;
    }
    if (lane == 63) wtot[w] = inc;
    __syncthreads();
    for (uint32_t v = 0; v < w; ++v) inc += wtot[v];
    sc[t] = inc;  // inclusive (block 0 reads other keys' entries below)
    __syncthreads();
    const uint32_t ks = inc - mineh;
    const uint32_t kc = t / kBuckets, knb = kBuckets - 1 - t % kBuckets;
    const bool ident_ok = mineh == static_cast<uint32_t>(n) && (kc <= 1 || (kc == 2 && (knb <= 16 || n >= 16384)));
    const bool ident = __syncthreads_or(LVK_IDENT && ident_ok && run_l == 0);
    if (blockIdx.x == 0) {
        ws[kWsTot + t] = mineh;
        if (t % kBuckets == 0) {  // per-class [start, count) for the CRC kernel
            ws[kWsCls + kc] = ks;
            ws[kWsCls + 4 + kc] = sc[t + kBuckets - 1] - ks;
        }
        if (t == 0) {
            ws[kWsIdent] = ident ? 1u : 0u;
            ws[kWsBytes] = static_cast<uint32_t>(total);
            ws[kWsBytes + 1] = static_cast<uint32_t>(total >> 32);
            ws[kWsPieces] = run_m;
            ws[kWsLongs] = run_l;
        }
    }
    if (ident) return;  // block-uniform
    __syncthreads();  // sc (inclusive) is read above; hpre becomes the claim cursor
    hpre[t] += ks;
    __syncthreads();
    // this chunk's buffers: sorted slots, entries, long records
    const uint64_t i = lo + t;
    const bool valid = i < hi;  // chunk <= 16 <= kSortThreads for n <= kSmallSort
    const uint32_t L = valid ? len[i] : 0u;
    const uint64_t o = valid ? off[i] : 0u;
    const uint32_t sd = (seed && valid) ? seed[i] : 0u;
    const uint32_t pos = wave_claim(hpre, sort_key(L), valid, lane);
    const uint32_t m = valid ? mpre[i + 1] - mpre[i] : 0u;
    if (valid) {
        ent[pos] = make_uint4(static_cast<uint32_t>(o), static_cast<uint32_t>(o >> 32), m ? 0u : L,
                              m ? 0xffffffffu : static_cast<uint32_t>(i));
        if (seed) sseed[pos] = sd;
        if (m) longs[lpre[i]] = make_uint4(static_cast<uint32_t>(i), mpre[i], m, pp[i]);
    }
    // this workgroup's share of the piece slots [0, run_m), one per thread
    const uint32_t per = (run_m + gridDim.x - 1) / gridDim.x;
    const uint32_t s0 = min(blockIdx.x * per, run_m), s1 = min(s0 + per, run_m);
    for (uint32_t u = s0 + t; u < s1; u += kSortThreads) {
        uint32_t j = 0, jh = static_cast<uint32_t>(n);  // the buffer holding slot u: the last j with mpre[j] <= u
        while (jh - j > 1) {
            const uint32_t mid = (j + jh) >> 1;
            if (mpre[mid] <= u) j = mid; else jh = mid;
        }
        const uint32_t mj = mpre[j + 1] - mpre[j], k = u - mpre[j];
        const uint32_t Lj = len[j];
        const uint64_t P = 1ull << pp[j];
        const uint64_t first = Lj - (static_cast<uint64_t>(mj) - 1) * P;  // piece 0: [0, first)
        const uint64_t a = off[j] + (k ? first + (k - 1) * P : 0);
        ent[n + u] = make_uint4(static_cast<uint32_t>(a), static_cast<uint32_t>(a >> 32),
                                static_cast<uint32_t>(k ? P : first), u | kPieceFlag);
        if (seed) sseed[n + u] = k ? 0u : seed[j];
    }
}

// ---------------------------------------------------------------------------
// WAL scan with the framing fused into the sort passes (the
// reader side, log_reader.rs:271-364).  Records never straddle a 32 KiB block
// (log_writer.rs:67-80), so every block's header chain can be walked on its
// own, exactly as read_physical_record frames it (log_reader.rs:271-331):
// stop when fewer than HEADER_SIZE bytes remain, at a length that overruns
// the block (BAD_LENGTH) or at a ZERO/0 header (ZERO).  wal_hist walks each
// block (one thread per block) and counts the records' CRC units
// [type || payload] (log_reader.rs:336) into the length-sort histogram, plus
// the records per block, and keeps each block's first kHdrCache headers; sort_scan
// is shared; wal_scatter takes those headers from the cache, one thread per
// record (no dependent chain step), walks on only for blocks with more
// records, and writes every record straight into its sorted slot, plus its
// log-order header offset and info word.  The class kernel then checksums the
// units.  Four launches, no host synchronisation (round 1: count pass, hipCUB
// scan, host readback of the total, emit pass, then the whole offsets API).
constexpr uint32_t kWalBlock = 32768;  // log_format.rs:63
constexpr uint32_t kWalHeader = 7;     // log_format.rs:66
constexpr uint32_t kHdrCache = 64;     // headers per block wal_hist keeps for wal_scatter

// A cached header: position in its block | length << 16 | type << 32.
__device__ __forceinline__ uint64_t hdr_pack(uint32_t pos, uint32_t len, uint32_t type) {
    return pos | (static_cast<uint64_t>(len) << 16) | (static_cast<uint64_t>(type) << 32);
}

// The 8 bytes at log offset pos (bytes past the log read as 0): aligned
// 8-B words, each read only if it holds a byte of the log (an aligned word
// never crosses a page), and a funnel shift.  (A per-thread 64-B LDS window
// of the log, which would keep several short records' headers per load,
// measured slower: wal_hist 36.6 -> 41.6 us; so did a 64-B register window
// parsed divergently, one load per record that leaves it: 38.9 -> 49.6 us;
// and 32-B / 64-B register windows in the uniform one-header-per-step loop:
// scan -1.5 / -2.8 %.
// The chains that bound the walk are hops over longer records, one HBM
// round trip each.)
__device__ __forceinline__ uint64_t wal_load8(const uint8_t *log, uint64_t size, uint64_t pos) {
    const uint64_t a = pos & ~7ull;
    const uint64_t *w = reinterpret_cast<const uint64_t *>(log + a);
    const uint64_t lo = a < size ? w[0] : 0ull;
    const uint32_t sh = static_cast<uint32_t>(pos & 7u) * 8u;
    if (!sh) return lo;
    const uint64_t hi = a + 8 < size ? w[1] : 0ull;
    return (lo >> sh) | (hi << (64u - sh));
}

// One step of a block's header chain: the record at pos (status, unit
// length); the next header is at pos + HEADER_SIZE + len.
struct WalRec {
    uint32_t len, type, status, ulen;
};

__device__ __forceinline__ WalRec wal_decode(uint64_t h, uint32_t blen, uint32_t pos) {  // crc(4) | length(2) | type(1)
    WalRec r;
    r.len = static_cast<uint32_t>(h >> 32) & 0xffffu;
    r.type = static_cast<uint32_t>(h >> 48) & 0xffu;
    r.status = LV_WAL_REC_OK;
    if (kWalHeader + r.len > blen - pos)
        r.status = LV_WAL_REC_BAD_LENGTH;  // log_reader.rs:312-324
    else if (r.type == 0 && r.len == 0)
        r.status = LV_WAL_REC_ZERO;        // log_reader.rs:326-331
    r.ulen = r.status == LV_WAL_REC_OK ? r.len + 1 : 0u;
    return r;
}

__device__ __forceinline__ WalRec wal_record(const uint8_t *log, uint64_t size, uint64_t start, uint32_t blen,
                                             uint32_t pos) {
    return wal_decode(wal_load8(log, size, start + pos), blen, pos);
}

// Long chains: after LVK_WAL_TOUCH_HOPS hops, the wave loads one dword of
// every 128-B line of the rest of each block still being walked (a block with
// that many records has short ones: its remaining headers are close
// together), four blocks at a time (16 loads per lane in flight, one HBM round
// trip per four blocks), so the remaining hops hit L2 (~200 cycles) instead
// of HBM (~900).  In the bench log 5 % of the blocks hold > 16 records and the
// longest chain is 54.
#ifndef LVK_WAL_TOUCH_HOPS
#define LVK_WAL_TOUCH_HOPS 16
#endif
__device__ __forceinline__ uint32_t wal_touch(const uint8_t *log, uint64_t b0, uint32_t pos, uint32_t blen,
                                              bool active, uint32_t lane) {
    uint64_t dm = __ballot(active);
    uint32_t x = 0;
    while (dm) {  // wave-uniform
        uint32_t v[4][4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int l0 = dm ? __ffsll(static_cast<long long>(dm)) - 1 : 0;
            const bool on = dm != 0;
            dm &= dm - 1;
            const uint32_t p0 = __shfl(pos, l0), bl = on ? __shfl(blen, l0) : 0u;
            const uint8_t *blk = log + (b0 + static_cast<uint64_t>(l0)) * kWalBlock;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t o = (p0 & ~127u) + 128u * (lane + 64u * k);
                v[g][k] = o < bl ? *reinterpret_cast<const uint32_t *>(blk + o) : 0u;
            }
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) x ^= xor3(v[g][0], v[g][1], v[g][2]) ^ v[g][3];
    }
    return x;
}

__global__ __launch_bounds__(kSortThreads) void wal_hist(const uint8_t *__restrict__ log, uint64_t size,
                                                         uint64_t nblocks, uint64_t chunk, uint32_t *__restrict__ M,
                                                         uint64_t *__restrict__ wgrec, uint32_t *__restrict__ blkcnt,
                                                         uint64_t *__restrict__ hcache) {
    __shared__ uint32_t h[kKeys];
    __shared__ uint64_t wsum[kSortThreads / 64];
    __shared__ uint64_t hcl[kSortThreads * (kHdrCache + 1)];  // per-thread header cache (130 KiB)
    const uint32_t t = threadIdx.x, lane = t & 63u;
    h[t] = 0;
    __syncthreads();
    const uint64_t lo = blockIdx.x * chunk, hi = lo + chunk < nblocks ? lo + chunk : nblocks;
    uint64_t mine = 0;
    uint32_t touched = 0;
    for (uint64_t b0 = lo; b0 < hi; b0 += kSortThreads) {  // block-uniform
        const uint64_t b = b0 + t;
        const uint64_t start = b * kWalBlock;
        const uint32_t blen = b < hi ? static_cast<uint32_t>(size - start < kWalBlock ? size - start : kWalBlock) : 0u;
        uint32_t pos = 0, cnt = 0, hops = 0;
        bool active = blen >= kWalHeader;
        // The header cache is filled in LDS and stored after the walk: a
        // global store in the hop (vmcnt counts stores too, in order) made
        // every hop's wait for its header load also wait for the previous
        // hop's store.
        uint64_t *const hl = hcl + t * (kHdrCache + 1);  // stride 65 words: lanes spread over the banks
        while (__any(active)) {  // wave-uniform: the longest chain of the wave
            if (LVK_WAL_TOUCH_HOPS && hops++ == LVK_WAL_TOUCH_HOPS)
                touched ^= wal_touch(log, b0 + (t & ~63u), pos, blen, active, lane);
            uint32_t key = 0;
            const bool rec = active;
            if (active) {
                const WalRec r = wal_record(log, size, start, blen, pos);
                key = sort_key(r.ulen);
                if (cnt < kHdrCache) hl[cnt] = hdr_pack(pos, r.len, r.type);
                ++cnt;
                pos += kWalHeader + r.len;
                active = r.status == LV_WAL_REC_OK && blen - pos >= kWalHeader;
            }
            wave_count(h, key, rec, lane);
        }
        for (uint32_t c = 0; c < cnt && c < kHdrCache; ++c) hcache[b * kHdrCache + c] = hl[c];
        if (b < hi) blkcnt[b] = cnt;
        mine += cnt;
    }
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) mine += __shfl_xor(mine, k);
    if (lane == 0) wsum[t >> 6] = mine;
    asm volatile("" ::"v"(touched));  // the touches are kept
    __syncthreads();
    M[static_cast<uint64_t>(blockIdx.x) * kKeys + t] = h[t];
    if (t == 0) wgrec[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];  // sort_scan sums these
}

// Output of the WAL scan, in log order (lv_wal_scan_device).
struct WalOut {
    uint64_t *hdr_off;
    uint32_t *info;  // type | status << 8 | length << 16
    uint64_t *count;
    uint64_t cap;
};

__global__ __launch_bounds__(kSortThreads) void wal_scatter(const uint8_t *__restrict__ log, uint64_t size,
                                                            uint64_t nblocks, uint64_t chunk, uint32_t *__restrict__ ws,
                                                            const uint32_t *__restrict__ M,
                                                            const uint64_t *__restrict__ wgrec,
                                                            const uint32_t *__restrict__ blkcnt,
                                                            const uint64_t *__restrict__ hcache, uint4 *__restrict__ ent,
                                                            WalOut o) {
    __shared__ uint32_t cur[kKeys];
    __shared__ uint32_t sc[kKeys];
    __shared__ uint64_t red[kSortThreads];
    const uint32_t t = threadIdx.x, lane = t & 63u;
    const uint64_t total = (static_cast<uint64_t>(ws[kWsBytes + 1]) << 32) | ws[kWsBytes];  // records
    const bool over = total > o.cap;  // nothing is written past the capacity: the caller retries
    const uint32_t mrow = M[static_cast<uint64_t>(blockIdx.x) * kKeys + t];
    const uint32_t ks = key_starts(ws, sc);
    cur[t] = ks + mrow;
    if (blockIdx.x == 0 && t % kBuckets == 0) {  // per-class [start, count) for the CRC kernel
        const uint32_t c = t / kBuckets;
        ws[kWsCls + c] = over ? 0u : ks;
        ws[kWsCls + 4 + c] = over ? 0u : sc[t + kBuckets - 1] - ks;
    }
    if (blockIdx.x == 0 && t == 0) {
        *o.count = total;
        ws[kWsIdent] = 0u;  // the class kernel reads the sorted entries
    }
    // this workgroup's first record in log order: the records of the ones before
    uint64_t pre = 0;
    for (uint32_t v = t; v < blockIdx.x; v += kSortThreads) pre += wgrec[v];
    red[t] = pre;
    __syncthreads();
    for (uint32_t d = kSortThreads / 2; d >= 1; d >>= 1) {
        if (t < d) red[t] += red[t + d];
        __syncthreads();
    }
    uint64_t run = red[0];
    __syncthreads();
    if (over) return;  // block-uniform
    const uint64_t lo = blockIdx.x * chunk, hi = lo + chunk < nblocks ? lo + chunk : nblocks;
    for (uint64_t b0 = lo; b0 < hi; b0 += kSortThreads) {  // block-uniform
        const uint64_t b = b0 + t;
        const uint32_t c = b < hi ? blkcnt[b] : 0u;
        red[t] = c;  // inclusive scan of the block counts (Hillis-Steele in LDS)
        __syncthreads();
        for (uint32_t d = 1; d < kSortThreads; d <<= 1) {
            const uint64_t x = t >= d ? red[t - d] : 0u;
            __syncthreads();
            red[t] += x;
            __syncthreads();
        }
        const uint32_t tot = static_cast<uint32_t>(red[kSortThreads - 1]);  // records of these blocks
        // The chunk's cached records, thread-parallel in log order: record q
        // belongs to the block j whose inclusive prefix first exceeds q (a
        // binary search over red), as its record k = q - excl(j).  (Round 2
        // first ran one thread per block over its records: a wave then took
        // as many claim-and-store steps as its longest block has records,
        // ~30 us for the bench log.)
        for (uint32_t q0 = 0; q0 < tot; q0 += kSortThreads) {  // block-uniform
            const uint32_t q = q0 + t;
            uint32_t j = 0;
            for (uint32_t step = kSortThreads / 2; step >= 1; step >>= 1)
                if (red[j + step - 1] <= q) j += step;
            const uint32_t ex = j ? static_cast<uint32_t>(red[j - 1]) : 0u;
            const uint32_t k = q - ex;
            const bool rec = q < tot && k < kHdrCache;
            const uint64_t bj = b0 + j;
            const uint64_t start = bj * kWalBlock;
            WalRec r{};
            uint32_t pos = 0;
            if (rec) {
                const uint64_t h = hcache[bj * kHdrCache + k];
                const uint32_t blen = static_cast<uint32_t>(size - start < kWalBlock ? size - start : kWalBlock);
                pos = static_cast<uint32_t>(h) & 0xffffu;
                r.len = static_cast<uint32_t>(h >> 16) & 0xffffu;
                r.type = static_cast<uint32_t>(h >> 32) & 0xffu;
                r.status = kWalHeader + r.len > blen - pos ? LV_WAL_REC_BAD_LENGTH
                                                           : (r.type == 0 && r.len == 0 ? LV_WAL_REC_ZERO : LV_WAL_REC_OK);
                r.ulen = r.status == LV_WAL_REC_OK ? r.len + 1 : 0u;
            }
            const uint32_t slot = wave_claim(cur, sort_key(r.ulen), rec, lane);
            if (rec) {
                const uint64_t rid = run + q;  // log order: blocks in order, records in chain order
                const uint64_t ua = start + pos + 6;  // [type || payload], log_reader.rs:336
                ent[slot] = make_uint4(static_cast<uint32_t>(ua), static_cast<uint32_t>(ua >> 32), r.ulen,
                                       static_cast<uint32_t>(rid));
                o.hdr_off[rid] = start + pos;
                o.info[rid] = r.type | (r.status << 8) | (r.len << 16);
            }
        }
        // blocks with more records than the cache holds walk on from there
        // (one thread per block; rare: a 32 KiB block holds > 64 records only
        // when most of them are a few bytes long)
        {
            const uint64_t start = b * kWalBlock;
            const uint32_t blen = b < hi ? static_cast<uint32_t>(size - start < kWalBlock ? size - start : kWalBlock) : 0u;
            bool active = c > kHdrCache;
            uint32_t pos = 0;
            uint64_t rid = run + static_cast<uint64_t>(red[t]) - c + kHdrCache;
            if (active) {
                const uint64_t h = hcache[b * kHdrCache + kHdrCache - 1];
                pos = (static_cast<uint32_t>(h) & 0xffffu) + kWalHeader + (static_cast<uint32_t>(h >> 16) & 0xffffu);
            }
            while (__any(active)) {
                WalRec r{};
                const bool rec = active;
                if (active) r = wal_record(log, size, start, blen, pos);
                const uint32_t slot = wave_claim(cur, sort_key(r.ulen), rec, lane);
                if (rec) {
                    const uint64_t ua = start + pos + 6;  // [type || payload], log_reader.rs:336
                    ent[slot] = make_uint4(static_cast<uint32_t>(ua), static_cast<uint32_t>(ua >> 32), r.ulen,
                                           static_cast<uint32_t>(rid));
                    o.hdr_off[rid] = start + pos;
                    o.info[rid] = r.type | (r.status << 8) | (r.len << 16);
                    ++rid;
                    pos += kWalHeader + r.len;
                    active = r.status == LV_WAL_REC_OK && blen - pos >= kWalHeader;
                }
            }
        }
        run += tot;
        __syncthreads();  // red is rewritten by the next chunk
    }
}

// ---------------------------------------------------------------------------
// Wave-uniform walk of length-sorted entries (offsets API).  The K = 64/G
// groups of a wave take K consecutive sorted entries per round; sorting by
// (class, batch count) makes their batch counts (nearly) equal, so the wave
// runs max_i(nb_i) batches for all of them under SCALAR control -- the
// uniform-block kernel's loop shape, ping-pong register slots and all.  A
// group with fewer batches starts early: its granules before the buffer start
// load from a clamped address and are zeroed in registers (leading zeros
// leave a zero CRC register unchanged).  The bytes after the last whole
// granule fold in as ONE granule (seed trick, below) instead of bytewise.
struct RGeo {
    uint64_t a;     // buffer start address (an empty buffer: the arena start)
    uint32_t len;
    uint32_t seed;
    uint32_t bid;   // output slot, or ~0u for a lane past the end of the list
    uint32_t aux;   // per-source extra (table units: in-range flag | type byte << 8)
    __device__ __forceinline__ uint64_t abase() const { return a & ~static_cast<uint64_t>(15); }
    __device__ __forceinline__ uint32_t alow() const { return static_cast<uint32_t>(a) & 15u; }
    __device__ __forceinline__ uint32_t ng() const { return (alow() + len) >> 4; }  // whole granules from g0
};

// Max over lanes l ^ m, m = from .. 32.  The 16- and 32-lane steps are
// gfx950's v_permlane16/32_swap (VALU; each swap returns v at l and at l ^ m
// in its two results) instead of ds_bpermute round trips through LDS.
#ifndef LVK_PERMLANE
#define LVK_PERMLANE 1
#endif
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v, int from) {
    for (int m = from; m < 64; m <<= 1) {
        uint32_t o;
#if LVK_PERMLANE
        if (m == 16) {
            const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
            o = r[0] > r[1] ? r[0] : r[1];
        } else if (m == 32) {
            const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
            o = r[0] > r[1] ? r[0] : r[1];
        } else
#endif
        {
            o = __shfl_xor(v, m);
        }
        v = o > v ? o : v;
    }
    return __builtin_amdgcn_readfirstlane(v);
}

// Geometry of sorted entry e (clamped to the last entry for lanes past the
// end, so every address stays valid).  Seeds come pre-sorted (sort_scatter),
// so no load depends on another.
template <bool SEEDED>
__device__ __forceinline__ RGeo load_rgeo(const Params &P, uint64_t e) {
    const bool valid = e < P.n;
    const uint64_t ec = valid ? e : P.n - 1;
    const uint4 v = P.ent[ec];
    RGeo q;
    // an empty buffer reads nothing of its own: point it at the arena start
    // so its (masked) loads stay inside the caller's allocation
    q.a = v.z ? P.base + ((static_cast<uint64_t>(v.y) << 32) | v.x) : P.base;
    q.len = v.z;
    q.seed = SEEDED ? P.sseed[ec] : 0u;
    q.bid = valid ? v.w : 0xffffffffu;
    q.aux = 0;
    return q;
}

// Wave max of the groups' batch counts (>= 1).
template <int G>
__device__ __forceinline__ uint32_t round_nbw(const RGeo &q) {
    constexpr uint32_t GU = G * U;
    const uint32_t nb = (q.ng() + GU - 1) / GU;
    return wave_max_u32(nb < 1u ? 1u : nb, G);
}

// Last batch index that holds head granules (d <= 1) for any group.
template <int G>
__device__ __forceinline__ uint32_t round_jfix(const RGeo &q, uint32_t nbw) {
    constexpr uint32_t GU = G * U;
    const uint32_t ng = q.ng();
    const uint32_t jh = (GU * nbw - ng) / GU + ((q.alow() > 12u && ng >= 2u) ? 1u : 0u);
    return wave_max_u32(jh, G);
}

// d (granule index relative to g0) of batch j, row 0, this lane.
template <int G>
__device__ __forceinline__ int32_t row_d(const RGeo &q, uint32_t nbw, uint32_t j, uint32_t gl) {
    return static_cast<int32_t>(q.ng()) - static_cast<int32_t>(G * U * (nbw - j)) + static_cast<int32_t>(gl);
}

// Batch j of a round: rows before the buffer clamp to granule g0.
template <int G>
__device__ __forceinline__ void load_rbatch(const RGeo &q, uint32_t nbw, uint32_t j, uint32_t gl, uint4 (&v)[U]) {
    const int32_t d0 = row_d<G>(q, nbw, j, gl);
    const uint64_t ab = q.abase();
#pragma unroll
    for (uint32_t i = 0; i < U; ++i) {
        int32_t d = d0 + static_cast<int32_t>(G * i);
        d = d < 0 ? 0 : d;
        const uint64_t ad = ab + (static_cast<uint32_t>(d) << 4);
        // the last row's 128-B line is shared with the next batch's first
        // row when the buffer end is not line aligned: keep it in L2
        v[i] = i == U - 1 ? load16_rt(ad) : load16(ad);
    }
}

// Head fix-up of batch j: zero granules before the buffer (d < 0), clear the
// pre-buffer bytes of g0 and xor the seed into buffer bytes 0..3.
template <int G>
__device__ __forceinline__ void fix_rbatch(const RGeo &q, uint32_t nbw, uint32_t j, uint32_t gl, uint4 (&v)[U]) {
    const uint32_t s0 = q.len >= 4 ? ~q.seed : 0u;
    const int32_t alow = static_cast<int32_t>(q.alow());
    const int32_t d0 = row_d<G>(q, nbw, j, gl);
#pragma unroll
    for (uint32_t i = 0; i < U; ++i) {
        const int32_t d = d0 + static_cast<int32_t>(G * i);
        if (d < 0) {
            v[i] = make_uint4(0, 0, 0, 0);
        } else if (d == 0 || (d == 1 && alow > 12)) {
            const int32_t rel = d * 16 - alow;
            v[i].x = fix_word(v[i].x, rel, s0);
            v[i].y = fix_word(v[i].y, rel + 4, s0);
            v[i].z = fix_word(v[i].z, rel + 8, s0);
            v[i].w = fix_word(v[i].w, rel + 12, s0);
        }
    }
}

// The granule after the last whole granule (k = (alow+len) & 15 bytes of it
// belong to the buffer).
__device__ __forceinline__ uint4 load_rtail(const RGeo &q, uint32_t gl) {
    if (gl == 0 && ((q.alow() + q.len) & 15u)) return load16_rt(q.abase() + (static_cast<uint64_t>(q.ng()) << 4));
    return make_uint4(0, 0, 0, 0);
}

// X = R(X, tail bytes).  With V the tail granule (pre-buffer bytes zeroed,
// seed applied, bytes >= k zeroed) and k >= 4:
//   R(X, V[0..k)) = R(0, V'[0..k)) with V'.x = V.x ^ X      (seed trick)
//                 = R(0, 0^(16-k) || V'[0..k))              (leading zeros)
// i.e. one granule fold of V' shifted up by 16-k bytes.  k < 4 goes bytewise.
__device__ __forceinline__ uint32_t fold_tail(uint32_t X, uint4 V, const RGeo &q, const Lut &L) {
    const uint32_t alow = q.alow();
    const uint32_t end = alow + q.len;
    const uint32_t k = end & 15u;
    if (k == 0) return X;
    const uint32_t s0 = q.len >= 4 ? ~q.seed : 0u;
    const int32_t rel = static_cast<int32_t>(end & ~15u) - static_cast<int32_t>(alow);
    uint32_t w[4] = {fix_word(V.x, rel, s0), fix_word(V.y, rel + 4, s0), fix_word(V.z, rel + 8, s0),
                     fix_word(V.w, rel + 12, s0)};
#pragma unroll
    for (uint32_t m = 0; m < 4; ++m) {  // zero bytes >= k
        const int32_t nb = static_cast<int32_t>(k) - static_cast<int32_t>(4 * m);
        w[m] &= nb >= 4 ? 0xffffffffu : (nb <= 0 ? 0u : (0xffffffffu >> (32 - 8 * nb)));
    }
    if (k >= 4) {
        w[0] ^= X;
        const uint64_t lo = (static_cast<uint64_t>(w[1]) << 32) | w[0];
        const uint64_t hi = (static_cast<uint64_t>(w[3]) << 32) | w[2];
        const uint32_t b = 8u * (16u - k);  // 8 .. 96
        uint64_t h2, l2;
        if (b >= 64) {
            h2 = lo << (b - 64);
            l2 = 0;
        } else {
            h2 = (hi << b) | (lo >> (64 - b));
            l2 = lo << b;
        }
        return r0_granule(make_uint4(static_cast<uint32_t>(l2), static_cast<uint32_t>(l2 >> 32),
                                     static_cast<uint32_t>(h2), static_cast<uint32_t>(h2 >> 32)),
                          L);
    }
    for (uint32_t i = 0; i < k; ++i) X = byte_step(X, (w[0] >> (8u * i)) & 0xffu);
    return X;
}

// ---- 256-B-aligned rows (the G = 16 classes) ----
// End-aligned rows of byte-packed buffers sit off the 128-B line grid: a
// 256-B group row then touches 3 lines instead of 2, and such rows read 11 %
// slower (6.12 vs 6.86 TB/s, tools/hbm_read_probe).  The G = 16 walk
// therefore puts rows on the absolute 256-B grid.  u = granule index from the
// 256-B boundary at or below the buffer start (g0 = u ph); the last whole
// granule u_e = ph + ng - 1 sits in row R_e, lane e, and R_e is row 3 of the
// last batch.  Granules before g0 and after u_e are zero in registers.  With
// lanes l > e read as belonging to the row BEFORE (their last data row is
// R_e - 1), every lane's distance to the end is 16 * (15 - l') for the
// rotated lane index l' = (l - e - 1) mod 16, so one lane rotation per buffer
// turns the ordinary merge tree into the exact CRC (merge_al).
#ifndef LVK_AL_RT_LAST
#define LVK_AL_RT_LAST 0
#endif
struct AGeo {
    int32_t ph;  // granule phase of g0 in its 256-B row
    int32_t re;  // row of the last whole granule (from ph's row)
    int32_t e;   // its lane
};

__device__ __forceinline__ AGeo al_geo(const RGeo &q) {
    AGeo g;
    g.ph = static_cast<int32_t>((q.abase() >> 4) & 15u);
    const int32_t ue = g.ph + static_cast<int32_t>(q.ng()) - 1;
    g.re = ue >> 4;
    g.e = ue & 15;
    return g;
}

// Wave max of the groups' batch counts (>= 1) at NU rows per batch.
template <uint32_t NU>
__device__ __forceinline__ uint32_t round_nbw_al(const AGeo &g) {
    const int32_t nb = (g.re + static_cast<int32_t>(NU)) / static_cast<int32_t>(NU);
    return wave_max_u32(nb < 1 ? 1u : static_cast<uint32_t>(nb), 16);
}

// Abs row rho of batch j, row i, in a round of nbw batches of NU rows.
template <uint32_t NU>
__device__ __forceinline__ int32_t al_row(const AGeo &g, uint32_t nbw, uint32_t j, uint32_t i) {
    return g.re + static_cast<int32_t>(NU * j + i + 1u) - static_cast<int32_t>(NU * nbw);
}

// Last batch that holds head granules (d <= 1) for any group.
template <uint32_t NU>
__device__ __forceinline__ uint32_t round_jfix_al(const RGeo &q, uint32_t nbw) {
    const AGeo g = al_geo(q);
    const int32_t uh = g.ph + ((q.alow() > 12u && q.ng() >= 2u) ? 1 : 0);
    const int32_t jh = ((uh >> 4) - g.re - 1 + static_cast<int32_t>(NU * nbw)) / static_cast<int32_t>(NU);
    return wave_max_u32(static_cast<uint32_t>(jh), 16);
}

// Granules outside the buffer's whole granules (d < 0: before its first
// 256-B row's start, or padding rows; d > dmax: past its end) load from a
// zero block instead of being zeroed after the load, so only the head batches
// need a fix-up pass (fix_rbatch_al); the load address costs the same selects
// a clamp would.
#ifndef LVK_ZERO_PAGE
#define LVK_ZERO_PAGE 1
#endif
__device__ __attribute__((aligned(256))) uint4 g_zero_granules[16];  // zero-initialised

template <uint32_t NU>
__device__ __forceinline__ void load_rbatch_al(const RGeo &q, uint32_t nbw, uint32_t j, uint32_t gl,
                                               uint4 (&v)[NU]) {
    const AGeo g = al_geo(q);
    const uint64_t ab = q.abase();
    const int32_t dmax = static_cast<int32_t>(q.ng()) - 1;
#pragma unroll
    for (uint32_t i = 0; i < NU; ++i) {
        int32_t d = 16 * al_row<NU>(g, nbw, j, i) + static_cast<int32_t>(gl) - g.ph;
#if LVK_ZERO_PAGE
        const uint64_t ad = (d < 0 || d > dmax) ? reinterpret_cast<uint64_t>(&g_zero_granules[gl])
                                                : ab + (static_cast<uint32_t>(d) << 4);
#else
        d = d > dmax ? dmax : d;  // upper clamp first: a buffer with no whole granule has dmax = -1
        d = d < 0 ? 0 : d;
        const uint64_t ad = ab + (static_cast<uint32_t>(d) << 4);
#endif
        v[i] = (LVK_AL_RT_LAST && i == NU - 1) ? load16_rt(ad) : load16(ad);
    }
}

// Head fix-up (as fix_rbatch) plus, without the zero block, the zero
// granules outside the buffer.
template <uint32_t NU>
__device__ __forceinline__ void fix_rbatch_al(const RGeo &q, uint32_t nbw, uint32_t j, uint32_t gl,
                                              uint4 (&v)[NU]) {
    const AGeo g = al_geo(q);
    const uint32_t s0 = q.len >= 4 ? ~q.seed : 0u;
    const int32_t alow = static_cast<int32_t>(q.alow());
    const int32_t dmax = static_cast<int32_t>(q.ng()) - 1;
#pragma unroll
    for (uint32_t i = 0; i < NU; ++i) {
        const int32_t d = 16 * al_row<NU>(g, nbw, j, i) + static_cast<int32_t>(gl) - g.ph;
#if LVK_ZERO_PAGE  // granules outside [0, dmax] were loaded from the zero block
        if ((d == 0 || (d == 1 && alow > 12)) && d <= dmax) {
#else
        if (d < 0 || d > dmax) {
            v[i] = make_uint4(0, 0, 0, 0);
        } else if (d == 0 || (d == 1 && alow > 12)) {
#endif
            const int32_t rel = d * 16 - alow;
            v[i].x = fix_word(v[i].x, rel, s0);
            v[i].y = fix_word(v[i].y, rel + 4, s0);
            v[i].z = fix_word(v[i].z, rel + 8, s0);
            v[i].w = fix_word(v[i].w, rel + 12, s0);
        }
    }
}

// Row merge by Horner with W1 = Shift_256: X = W1(W1(W1(A0)^A1)^A2)^A3.
// Lanes past e end one row earlier: their last row is row 2 of the last
// batch, and their row-3 accumulator must be taken BEFORE the last batch's
// W4 step (a3p), so their Horner runs (a3p, A0, A1, A2).  Then the lane
// rotation by e + 1 (one ds_bpermute) and the ordinary tree: lane 0 of the
// group holds R over the buffer's whole granules.
// (In the depth-2 form W2(W1(h0)^h1) ^ (W1(h2)^h3).)  `rot` (wave-uniform)
// is false when every group of the wave ends at lane 15 (e.g. aligned table
// blocks): no early lanes, no rotation.
template <uint32_t NU>
__device__ __forceinline__ uint32_t merge_al(const uint32_t (&A)[NU], uint32_t a3p, const Lut &L, const RGeo &q,
                                             uint32_t gl, uint32_t lane, bool rot) {
    const AGeo g = al_geo(q);
    const bool early = static_cast<int32_t>(gl) > g.e;
    uint32_t X;
    if constexpr (LVK_EXP_NOMERGE) {
        X = early ? a3p : 0u;
#pragma unroll
        for (uint32_t i = 0; i < NU; ++i) X ^= A[i];
        return X;
    } else if constexpr (NU == 4) {
        const uint32_t x01 = lookup4<kRegionB>(early ? a3p : A[0], L) ^ (early ? A[0] : A[1]);
        const uint32_t x23 = lookup4<kRegionB>(early ? A[1] : A[2], L) ^ (early ? A[2] : A[3]);
        X = lookup4<kRegionB + kHalf>(x01, L) ^ x23;
    } else if constexpr (NU == 3) {  // W1(W1(h0) ^ h1) ^ h2
        const uint32_t x01 = lookup4<kRegionB>(early ? a3p : A[0], L) ^ (early ? A[0] : A[1]);
        X = lookup4<kRegionB>(x01, L) ^ (early ? A[1] : A[2]);
    } else {  // NU = 2: W1(h0) ^ h1
        static_assert(NU == 2, "aligned rows: 2, 3 or 4 rows per batch");
        X = lookup4<kRegionB>(early ? a3p : A[0], L) ^ (early ? A[0] : A[1]);
    }
    if (rot) X = __shfl(X, static_cast<int32_t>((lane & ~15u) | ((gl + static_cast<uint32_t>(g.e) + 1u) & 15u)));
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t other = lanes_down<16, false>(X, k);
        X = comb_shift(X, k) ^ other;
    }
    return X;
}

// Leading rows of a round's first batch that hold no buffer byte for any
// group of the wave (wave-uniform, <= NU - 1): the first fold skips them.
#ifndef LVK_SKIP_PAD
#define LVK_SKIP_PAD 1
#endif
template <int G, uint32_t NU>
__device__ __forceinline__ uint32_t round_pad(const RGeo &q, uint32_t nbw) {
    uint32_t padg;
    if constexpr (LVK_ALIGNED_ROWS && G == 16) {
        const int32_t p = static_cast<int32_t>(NU * nbw) - al_geo(q).re - 1;
        padg = p <= 0 ? 0u : static_cast<uint32_t>(p);
    } else {  // end-aligned rows: row i is empty for every lane iff ng - G*NU*nbw + G*(i+1) - 1 < 0
        const uint32_t gu = G * NU * nbw, ng = q.ng();
        padg = gu > ng ? (gu - ng) / G : 0u;
    }
    padg = padg < NU - 1 ? padg : NU - 1;
    return (NU - 1) - wave_max_u32((NU - 1) - padg, G);
}

template <int W4K, uint32_t NU, uint32_t W4OFF>
__device__ __forceinline__ void fold_first(const uint4 (&v)[NU], uint32_t (&A)[NU], const Lut &L, uint32_t pad) {
#if LVK_SKIP_PAD
    if constexpr (NU >= 3) {
        if constexpr (NU == 4) {
            if (pad == 3) {
                fold_batch<true, W4K, NU, W4OFF, 3>(v, A, L);
                return;
            }
        }
        if (pad == 2) {
            fold_batch<true, W4K, NU, W4OFF, 2>(v, A, L);
            return;
        }
        if (pad == 1) {
            fold_batch<true, W4K, NU, W4OFF, 1>(v, A, L);
            return;
        }
    }
#endif
    fold_batch<true, W4K, NU, W4OFF>(v, A, L);
}

// The raw register R(~seed, buffer) (lane 0 of the group), before the final
// xor and mask: the tail bytes, then the short-buffer seed.
__device__ __forceinline__ uint32_t finish_raw(const RGeo &q, uint32_t X, const uint4 &tail, uint32_t gl,
                                               const Lut &L) {
    if (!LVK_EXP_NOTAIL) X = fold_tail(X, tail, q, L);
    if (gl == 0 && q.len < 4) {  // R(s, D) = R(0, D) ^ Shift_|D|(s) for short buffers
        uint32_t s = ~q.seed;
        for (uint32_t i = 0; i < q.len; ++i) s = byte_step(s, 0u);
        X ^= s;
    }
    return X;
}

// Entry source and result sink of the sorted walk: the offsets API's
// length-sorted list.  load() reads entry e; trailer() issues any extra
// per-unit loads with the tail load; stage() parks a unit's result in the
// wave's LDS slots (lane 0 of the group); flush() stores the parked results
// of the last rounds, one global store per lane, every kFlush rounds.
template <bool SEEDED>
struct SortedList {
    static constexpr uint32_t kFlush = 16;  // 64 slots of one word pair
    bool ident;  // the list is the identity (kWsIdent): entry e is buffer e of off/len/seed
    __device__ __forceinline__ RGeo load(const Params &P, uint64_t e) const {
        if (!ident) return load_rgeo<SEEDED>(P, e);
        const bool valid = e < P.n;
        const uint64_t ec = valid ? e : P.n - 1;
        RGeo q;
        q.len = P.len[ec];
        q.a = q.len ? P.base + P.off[ec] : P.base;  // an empty buffer reads nothing of its own
        q.seed = SEEDED ? P.seed[ec] : 0u;
        q.bid = valid ? static_cast<uint32_t>(ec) : 0xffffffffu;
        q.aux = 0;
        return q;
    }
    __device__ __forceinline__ uint2 trailer(const RGeo &, uint32_t) const { return make_uint2(0, 0); }
    // A piece parks its raw register for combine_long_kernel; its output slot
    // is its piece slot with the top bit set (piece slots are < kPieceBudget,
    // and a list with pieces has buffer indices < 2^31: launch_binned).
    __device__ __forceinline__ void stage(const Params &P, uint32_t wave, uint32_t slot, const RGeo &q, uint32_t X,
                                          uint2) const {
        const bool piece = P.nplain < P.n && q.bid != 0xffffffffu && (q.bid & kPieceFlag);
        g_oidx[wave][slot] = q.bid;
        g_ocrc[wave][slot] = piece ? X : final_crc(P, X);
    }
    __device__ __forceinline__ void flush(const Params &P, uint32_t wave, uint32_t lane, uint32_t nslots) const {
        const uint32_t bi = g_oidx[wave][lane], cv = g_ocrc[wave][lane];
        if (lane >= nslots || bi == 0xffffffffu) return;
        // piece slots (flagged in the entry) occur only in the pieces' sub-list (P.nplain < P.n)
        if (P.nplain < P.n && (bi & kPieceFlag))
            P.part[bi & ~kPieceFlag] = cv;
        else
            P.out[bi] = cv;
    }
};

// One wave walks rounds of the sorted list: round rho holds entries
// rho*K + group (K = 64/G groups).  The rounds come from `next()` (a static
// stride, or a workgroup's shared pool) until it returns rho >= nr.  Batches
// are prefetched one ahead, across rounds, in two ping-pong register slots;
// all control is wave-uniform.  Results are staged in LDS (g_oidx/g_ocrc)
// and stored every G rounds.  (Issuing the same loads in every step --
// entries and tail re-read each batch -- measured 4-5 % slower: the extra
// loads and spills cost more than the conservative wait counts they remove.)
// The image is always the G = 16 one: groups of G = 1 and 4 take their
// row-shift and merge tables from the plain combine tables.
template <int G, class Src, class Next, uint32_t ALR = kAlRows>
__device__ __forceinline__ void sorted_stream(const Params &P, const Src &src, uint32_t lane, const Lut &L,
                                              uint64_t rho, Next next) {
    constexpr bool AL = LVK_ALIGNED_ROWS && G == 16;  // 256-B-aligned rows (merge_al)
    constexpr uint32_t NU = AL ? ALR : U;              // rows per batch
    // Latin row shift Shift_{16 G NU}: region A's second half (the image's W4
    // for NU = 4; Shift_768 in the table image for NU = 3) or region B's W2
    // (NU = 2)
    constexpr uint32_t W4OFF = NU >= 3 ? kRegionA + kHalf : kRegionB + kHalf;
    constexpr uint32_t K = 64 / G;
    constexpr int W4K = G == 16 ? -1 : (G == 4 ? 4 : 2);  // Shift_{64G}
    constexpr int W1K = G == 16 ? -1 : (G == 4 ? 2 : 0);  // Shift_{16G}
    constexpr int W2K = G == 16 ? -1 : (G == 4 ? 3 : 1);  // Shift_{32G}
    const uint32_t gl = lane % G, grp = lane / G;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nr = (P.n + K - 1) / K;  // rounds in the list
    if (rho >= nr) return;
    uint64_t rhon = next();

    RGeo q = src.load(P, rho * K + grp);
    // (AL) some group of the round ends before lane 15.  The row geometry
    // (al_geo) is recomputed from q where it is used: fewer live registers.
    bool rot = AL && __any(al_geo(q).e != 15);
    uint32_t nbw = AL ? round_nbw_al<NU>(al_geo(q)) : round_nbw<G>(q);
    uint32_t jfix = AL ? round_jfix_al<NU>(q, nbw) : round_jfix<G>(q, nbw);
    uint32_t pad = round_pad<G, NU>(q, nbw);
    RGeo qn = q;
    if (rhon < nr) qn = src.load(P, rhon * K + grp);
    uint32_t nbwn = 0;
    uint4 tail;
    uint2 tr;
    uint4 slot0[NU], slot1[NU];
    if constexpr (AL)
        load_rbatch_al<NU>(q, nbw, 0, gl, slot0);
    else
        load_rbatch<G>(q, nbw, 0, gl, slot0);
    uint32_t A[NU];
    uint32_t a3p = 0;  // (AL) the last row's accumulator before the last batch
    uint32_t c = 0;  // rounds finished (output staging slot)
    uint32_t j = 0;

    auto step = [&](uint4(&cur)[NU], uint4(&nxt)[NU]) -> bool {
        const bool lastj = j + 1 == nbw;
        const bool more = rhon < nr;
        if (!lastj) {
            if constexpr (AL)
                load_rbatch_al<NU>(q, nbw, j + 1, gl, nxt);
            else
                load_rbatch<G>(q, nbw, j + 1, gl, nxt);
        } else {
            tail = load_rtail(q, gl);  // consumed after this batch's fold
            tr = src.trailer(q, gl);
            if (more) {
                if constexpr (AL) {
                    nbwn = round_nbw_al<NU>(al_geo(qn));
                    load_rbatch_al<NU>(qn, nbwn, 0, gl, nxt);
                } else {
                    nbwn = round_nbw<G>(qn);
                    load_rbatch<G>(qn, nbwn, 0, gl, nxt);
                }
            }
        }
        if constexpr (AL) {
            if (!LVK_EXP_NOFIX && (j <= jfix || (!LVK_ZERO_PAGE && lastj && rot))) fix_rbatch_al<NU>(q, nbw, j, gl, cur);
        } else if (j <= jfix) {
            fix_rbatch<G>(q, nbw, j, gl, cur);
        }
        if constexpr (AL) {
            if (lastj) a3p = j == 0 ? 0u : A[NU - 1];
        }
        if (j == 0)
            fold_first<W4K, NU, W4OFF>(cur, A, L, pad);
        else
            fold_batch<false, W4K, NU, W4OFF>(cur, A, L);
        if (!lastj) {
            ++j;
            return false;
        }
        uint32_t X;
        if constexpr (AL)
            X = merge_al<NU>(A, a3p, L, q, gl, lane, rot);
        else
            X = merge_group<G, W1K, W2K>(A, L);
        X = finish_raw(q, X, tail, gl, L);
        // slots: rounds per flush x groups per wave <= 64
        constexpr uint32_t kF = Src::kFlush * K <= 64 ? Src::kFlush : 64 / K;
        const uint32_t slot = (c % kF) * K + grp;
        if (gl == 0) src.stage(P, wave, slot, q, X, tr);
        if ((c + 1) % kF == 0 || !more) {
            __builtin_amdgcn_wave_barrier();
            src.flush(P, wave, lane, (c % kF + 1) * K);
            __builtin_amdgcn_wave_barrier();
        }
        if (!more) return true;
        ++c;
        q = qn;
        nbw = nbwn;
        if constexpr (AL) {
            rot = __any(al_geo(q).e != 15);
            jfix = round_jfix_al<NU>(q, nbw);
        } else {
            jfix = round_jfix<G>(q, nbw);
        }
        pad = round_pad<G, NU>(q, nbw);
        rhon = next();
        if (rhon < nr) qn = src.load(P, rhon * K + grp);
        j = 0;
        return false;
    };
    for (;;) {
        if (step(slot0, slot1)) break;
        if (step(slot1, slot0)) break;
    }
}

// The sorted sub-list [start, start+count) followed by `pieces` piece
// entries (the long-buffer split; they sit right after the n sorted entries,
// i.e. after the last class).
__device__ __forceinline__ Params sub_list(const Params &P0, uint32_t start, uint32_t count, uint32_t pieces = 0) {
    Params P = P0;
    P.ent = P0.ent + start;
    P.sseed = P0.sseed ? P0.sseed + start : nullptr;
    P.n = static_cast<uint64_t>(count) + pieces;
    P.nplain = count;
    return P;
}

// Waves per workgroup that walk the small classes (<= 2 KiB) before joining
// the large-buffer pool.  Measured on C2/C4: class 0 runs as fast on 4 waves
// per CU as on 16 (it is bound by per-buffer VALU work and random line
// reads, not latency), and classes 2+3 run FASTER on 12 waves than on 16.
#ifndef LVK_SMALL_WAVES
#define LVK_SMALL_WAVES 4
#endif
constexpr uint32_t kSmallWaves = LVK_SMALL_WAVES;
#ifndef LVK_SMALL_ALL
#define LVK_SMALL_ALL 1
#endif

// Next round of the workgroup's large-buffer share: a word of combine table
// k = 5 (Shift_512), which no group of the class kernel uses, since the LDS
// is full (image + output staging = 160 KiB).
constexpr uint32_t kPoolWord = (kComb + 5 * 4096) / 4;

// The offsets API in ONE persistent launch over the length-sorted list, on
// the G = 16 table image (staged once).  Waves [0, kSmallWaves) of every
// workgroup walk class 0 (G = 1) and then class 1 (G = 4), each class spread
// over those waves of the whole grid; meanwhile the other waves stream
// classes 2+3 (G = 16; one contiguous list).  Workgroup b owns the large
// rounds rho = b + k*grid, which its waves take from an LDS counter, so the
// small-class waves join the large work when they are done and no wave idles
// while its workgroup has rounds left.  (Earlier: a static split of the grid
// by class, 3-8 % slower -- a class that finishes early idles its CUs; then
// every workgroup walking every class in turn, with the image restaged per
// G -- the small classes ran alone, latency- and VALU-bound, for ~100 us of
// C2's 1.2 ms.)
#ifndef LVK_CLASS_STAGGER
#define LVK_CLASS_STAGGER 1
#endif
template <bool SEEDED>
__global__ __launch_bounds__(kThreads) void crc32c_classes_kernel(Params P, const uint4 *__restrict__ image,
                                                                  const uint32_t *ws) {
    const uint32_t *cls = ws + kWsCls;
    const bool ident = ws[kWsIdent] != 0u;  // sort_scatter skipped a one-key batch
    stage_tables(image);
    if (threadIdx.x == 0) g_lds[kPoolWord] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const Lut L = make_lut(lane);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t grid = gridDim.x;
    const uint32_t n23 = cls[6] + cls[7];
    // pieces of split long buffers (walked after classes 2+3; a split buffer
    // is longer than 16 KiB, so class 2 or 3, and n23 > 0 whenever there are
    // pieces)
    const uint32_t np = P.part ? min(ws[kWsPieces], kPieceBudget) : 0u;
    // With no large buffers at all, every wave walks the small classes.
#if LVK_SMALL_ALL
    const uint32_t nsmall = n23 ? kSmallWaves : kWaves;
#else
    constexpr uint32_t nsmall = kSmallWaves;
#endif
    if (wave < nsmall) {
        const uint64_t sw = blockIdx.x * nsmall + wave, nsw = grid * nsmall;
        uint64_t k = 0;
        auto stride = [&]() { return sw + (++k) * nsw; };
        if (cls[4]) {
            sorted_stream<1>(sub_list(P, cls[0], cls[4]), SortedList<SEEDED>{ident}, lane, L, sw, stride);
            k = 0;
        }
        if (cls[5]) sorted_stream<4>(sub_list(P, cls[1], cls[5]), SortedList<SEEDED>{ident}, lane, L, sw, stride);
    }
    if (n23) {
#if LVK_CLASS_STAGGER
        // A list of mostly long-buffer pieces (>= 3/4 of the entries), with
        // >= 64 KiB per wave, is the blocks kernel's long-block regime: waves
        // that start together stream their pieces in lockstep, which reads
        // slower; stagger them as crc32c_blocks_kernel does (64 x 16 MiB:
        // 223 -> 201 us per call).
        const uint64_t bytes = (static_cast<uint64_t>(ws[kWsBytes + 1]) << 32) | ws[kWsBytes];
        if (4ull * np >= 3ull * (n23 + np) && bytes >= (64ull << 10) * grid * kWaves)
            for (uint32_t k = 0; k < wave * LVK_STAGGER; ++k) __builtin_amdgcn_s_sleep(32);
#endif
        auto pool = [&]() -> uint64_t {
            uint32_t k = 0;
            if (lane == 0) k = atomicAdd(&g_lds[kPoolWord], 1u);
            return blockIdx.x + grid * static_cast<uint64_t>(__shfl(k, 0));
        };
        sorted_stream<16>(sub_list(P, cls[6] ? cls[2] : cls[3], n23, np), SortedList<SEEDED>{ident}, lane, L, pool(),
                          pool);
    }
}

// ---------------------------------------------------------------------------
// SSTable block trailers in ONE launch (include/lvgpu/table.h).
// The table's blocks are walked in file order, four per wave round, by the
// G = 16 aligned-row walk: blocks of one table have similar sizes (block_size
// plus at most one entry), so consecutive blocks give a near-uniform round
// with no length sort.  The handles (BlockHandle extents, table/format.rs:
// 29-50) are read directly, and the trailer work is the epilogue:
//  * verify: unit = contents || type (size + 1 bytes); the stored LE32 after
//    it is loaded with the tail and compared after unmask;
//  * seal: unit = contents; the type byte enters the register by one table
//    step, R(s, D || t) = T0-step(R(s, D), t), so no byte is written before
//    it is read, and type + LE32(mask(crc)) are written in the flush.
// (Round 1 ran units -> 3 sort passes -> class kernel -> trailer kernel.)
__device__ __forceinline__ bool sst_in_range(uint64_t o, uint64_t sz, uint64_t file_bytes) {
    return sz < 0xffffffffull && o <= file_bytes && sz <= file_bytes - o && file_bytes - o - sz >= 5u;
}

#ifndef LVK_SEAL_FLUSH  // rounds per seal flush (<= 16: 64 two-word slots)
#define LVK_SEAL_FLUSH 16
#endif
template <bool SEAL, bool CRCOUT = false>
struct TableUnits {
    const uint2 *handles;  // {offset, size} u64 pairs per block
    const uint8_t *types;  // seal: per-block type byte (NULL: 0 = no compression)
    uint32_t *status;      // verify: LV_SST_BLOCK_* per block
    uint32_t *crc_out;     // verify: optional crc32c(contents || type)
    uint64_t file_bytes;
    // seal: 64 slots of {block, masked crc} (16 rounds of 4 blocks per flush;
    // the trailer stores are partial-line writes, and fewer, larger bursts of
    // them measured faster); verify: 64 slots of {block, status}, or with
    // crc_out 32 slots of four words
    static constexpr uint32_t kFlush = SEAL ? LVK_SEAL_FLUSH : !CRCOUT ? 16 : 8;

    __device__ __forceinline__ RGeo load(const Params &P, uint64_t e) const {
        const bool valid = e < P.n;
        const uint64_t ec = valid ? e : P.n - 1;
        const uint2 ho = handles[2 * ec], hs = handles[2 * ec + 1];  // u64 pairs: 8-B alignment is enough
        const uint64_t o = (static_cast<uint64_t>(ho.y) << 32) | ho.x, sz = (static_cast<uint64_t>(hs.y) << 32) | hs.x;
        const bool ok = sst_in_range(o, sz, file_bytes);
        RGeo q;
        q.len = ok ? static_cast<uint32_t>(SEAL ? sz : sz + 1) : 0u;
        // in range: the block's own offset even when empty (its trailer goes
        // there; its loads stay inside the file); otherwise the file start
        q.a = ok ? P.base + o : P.base;
        q.seed = 0;
        q.bid = valid ? static_cast<uint32_t>(ec) : 0xffffffffu;
        uint32_t t = 0;
        if (SEAL && types && ok) t = types[ec];
        q.aux = (ok ? 1u : 0u) | (t << 8);
        return q;
    }
    // verify: the stored masked crc at the unit's end (two aligned dwords)
    __device__ __forceinline__ uint2 trailer(const RGeo &q, uint32_t gl) const {
        if (SEAL || gl != 0 || !(q.aux & 1u)) return make_uint2(0, 0);
        const uint64_t end = q.a + q.len;
        const uint32_t *w = reinterpret_cast<const uint32_t *>(end & ~static_cast<uint64_t>(3));
        return make_uint2(w[0], (end & 3u) ? w[1] : 0u);
    }
    __device__ __forceinline__ void stage(const Params &, uint32_t wave, uint32_t slot, const RGeo &q, uint32_t X,
                                          uint2 tr) const {
        const bool ok = q.aux & 1u;
        if constexpr (SEAL) {
            const uint32_t t = (q.aux >> 8) & 0xffu;
            const uint32_t crc = ~byte_step(X, t);
            g_oidx[wave][slot] = ok ? q.bid : 0xffffffffu;  // the flush re-reads the handle and type
            g_ocrc[wave][slot] = mask_crc(crc);
        } else {
            const uint32_t crc = ~X;
            const uint32_t k = static_cast<uint32_t>(q.a + q.len) & 3u;
            const uint32_t stored = k ? (tr.x >> (8 * k)) | (tr.y << (32 - 8 * k)) : tr.x;
            const uint32_t r = stored - 0xa282ead8u;  // unmask, crc32c.rs:59-63
            const uint32_t st = !ok ? LV_SST_BLOCK_OUT_OF_RANGE
                                    : (((r >> 17) | (r << 15)) == crc ? LV_SST_BLOCK_OK : LV_SST_BLOCK_CHECKSUM_MISMATCH);
            g_oidx[wave][slot] = q.bid;
            g_ocrc[wave][slot] = st;
            if (CRCOUT) g_ocrc[wave][32 + slot] = ok ? crc : 0u;
        }
    }
    __device__ __forceinline__ void flush(const Params &P, uint32_t wave, uint32_t lane, uint32_t nslots) const {
        if constexpr (SEAL) {
            if (lane >= nslots) return;
            const uint32_t bi = g_oidx[wave][lane];
            if (bi == 0xffffffffu || LVK_EXP_NOSEALWRITE) return;
            const uint2 ho = handles[2 * bi], hs = handles[2 * bi + 1];
            const uint64_t o = (static_cast<uint64_t>(ho.y) << 32) | ho.x, sz = (static_cast<uint64_t>(hs.y) << 32) | hs.x;
            uint8_t *p = reinterpret_cast<uint8_t *>(P.base + o + sz);  // type byte, then LE32(mask(crc))
            const uint32_t f = types ? types[bi] : 0u;
            const uint32_t m = g_ocrc[wave][lane];
            p[0] = static_cast<uint8_t>(f);
            p[1] = static_cast<uint8_t>(m);
            p[2] = static_cast<uint8_t>(m >> 8);
            p[3] = static_cast<uint8_t>(m >> 16);
            p[4] = static_cast<uint8_t>(m >> 24);
        } else if constexpr (!CRCOUT) {
            if (lane >= nslots) return;
            const uint32_t bi = g_oidx[wave][lane];
            if (bi != 0xffffffffu) status[bi] = g_ocrc[wave][lane];
        } else {
            const uint32_t sl = lane & 31u;
            if (sl >= nslots) return;
            const uint32_t bi = g_oidx[wave][sl];
            if (bi == 0xffffffffu) return;
            if (lane < 32)
                status[bi] = g_ocrc[wave][sl];
            else if (crc_out)
                crc_out[bi] = g_ocrc[wave][32 + sl];
        }
    }
};

// Rows per batch of the table walk.  A 4,097-4,352-B unit at a byte-packed
// start spans 17-19 rows of the 256-B grid: 5 four-row batches (20 rows) or
// 6 three-row batches (18 rows, with Shift_768 as the batch shift: the table
// image, host_image(kTableImage)).
#ifndef LVK_SST_ROWS
#define LVK_SST_ROWS 3
#endif
constexpr uint32_t kSstRows = LVK_SST_ROWS;
static_assert(kSstRows == 3 || kSstRows == 4, "table walk: 3 or 4 rows per batch");

template <bool SEAL, bool CRCOUT>
__global__ __launch_bounds__(kThreads) void sst_blocks_kernel(Params P, const uint4 *__restrict__ image,
                                                              TableUnits<SEAL, CRCOUT> src) {
    stage_tables(image);
    if (threadIdx.x == 0) g_lds[kPoolWord] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const Lut L = make_lut(lane);
    const uint64_t grid = gridDim.x;
    auto pool = [&]() -> uint64_t {
        uint32_t k = 0;
        if (lane == 0) k = atomicAdd(&g_lds[kPoolWord], 1u);
        return blockIdx.x + grid * static_cast<uint64_t>(__shfl(k, 0));
    };
    sorted_stream<16, TableUnits<SEAL, CRCOUT>, decltype(pool), kSstRows>(P, src, lane, L, pool(), pool);
}

// Joins the raw piece registers of the long-block split: block b's pieces
// R_k = raw[b*s + k], k < s (s a power of two <= 4,096), give
//   R(~seed, block) = XOR_k Shift_{(s-1-k) plen}(R_k)
// (linearity, DESIGN "CRC algebra").
constexpr uint32_t kPow2Tabs = 13;  // Shift_{2^v plen}, v <= 12 (s <= 4,096)

__device__ __forceinline__ uint32_t tab_shift(const uint32_t *t, uint32_t a) {
    return t[a & 0xffu] ^ t[256 + ((a >> 8) & 0xffu)] ^ t[512 + ((a >> 16) & 0xffu)] ^ t[768 + (a >> 24)];
}

// Stage n4 uint4 of `src` into LDS `dst` (16-B loads, all issued first).
__device__ __forceinline__ void stage_words(uint32_t *dst, const uint32_t *src, uint32_t n4) {
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
    uint4 *d4 = reinterpret_cast<uint4 *>(dst);
    for (uint32_t i = threadIdx.x; i < n4; i += blockDim.x) d4[i] = s4[i];
}

// s <= 1,024: one wave per block (GF(2) matrices Shift_{j plen}, j <= 64, at a
// stride of 33 words so that lanes applying different matrices read distinct
// banks): lane l < min(s, 64) runs Horner over its pieces k = l + 64 m with
// Shift_{64 plen}, then shifts by (min(s, 64) - 1 - l) plen; an xor over the
// wave.  (Byte tables here -- a tree of Shift_{2^u plen} lookups -- staged
// 28 KiB per workgroup against 8 KiB of matrices: 16 x 1 MiB 16.9 -> 19.5 us.)
__global__ __launch_bounds__(256) void combine_pieces_kernel(const uint32_t *__restrict__ raw, uint64_t n, uint32_t s,
                                                             const uint32_t *__restrict__ mats,
                                                             uint32_t *__restrict__ out, uint32_t flags) {
    __shared__ uint32_t M[65 * 33];
    for (uint32_t i = threadIdx.x; i < 65 * 32; i += blockDim.x) M[(i >> 5) * 33 + (i & 31u)] = mats[i];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = s < 64 ? s : 64, reps = s <= 64 ? 1 : s / 64;
    const uint64_t nw = static_cast<uint64_t>(gridDim.x) * (blockDim.x / 64);
    for (uint64_t b = static_cast<uint64_t>(blockIdx.x) * (blockDim.x / 64) + (threadIdx.x >> 6); b < n; b += nw) {
        uint32_t acc = 0;
        if (lane < w) {
            uint32_t nx = raw[b * s + lane];
            for (uint32_t m = 0; m < reps; ++m) {  // wave-uniform count (an unrolled 16 ran dead shift bodies)
                const uint32_t cur = nx;
                if (m + 1 < reps) nx = raw[b * s + lane + 64 * (m + 1)];
                acc = (m ? gf2_apply(M + 64 * 33, acc) : 0u) ^ cur;
            }
            acc = gf2_apply(M + (w - 1 - lane) * 33, acc);
        }
#pragma unroll
        for (int k = 32; k >= 1; k >>= 1) acc ^= __shfl_xor(acc, k);
        if (lane == 0) {
            const uint32_t crc = ~acc;
            out[b] = (flags & LV_CRC_MASK) ? mask_crc(crc) : crc;
        }
    }
}

// Blocks of many pieces (s = 2,048 or 4,096): one 1024-thread workgroup per
// block.  Thread t runs Horner with Shift_plen over its c = s / 1024
// consecutive pieces; a 6-level tree joins the lanes of each wave with
// Shift_{c 2^u plen}, and a 4-level tree over the 16 wave partials (lanes of
// wave 0) with Shift_{64 c 2^u plen}.  Every shift is a byte-table lookup
// (Shift_n(v) = S0[v.b0] ^ S1[v.b1] ^ S2[v.b2] ^ S3[v.b3], 4 KiB per n, from
// the per-plen set Shift_{2^v plen}, piece_tabs): four LDS reads where a
// GF(2) matrix product took ~100 VALU instructions, so the 14 dependent steps
// cost what 25 matrix products on 256 threads did not (1 x 16 MiB: join 12.7
// -> ~4 us, call 25.7 -> 16.8 us).
__global__ __launch_bounds__(1024) void combine_pieces_wg_kernel(const uint32_t *__restrict__ raw, uint32_t s,
                                                                 const uint32_t *__restrict__ tabs,
                                                                 uint32_t *__restrict__ out, uint32_t flags) {
    __shared__ __attribute__((aligned(16))) uint32_t T[11 * 1024];  // slot 0: Shift_plen; 1 + u: Shift_{c 2^u plen}
    __shared__ uint32_t part[16];
    const uint32_t c = s / 1024u;
    const uint32_t lc = c >= 4u ? 2u : 1u;  // log2 c (s >= 2,048)
    stage_words(T, tabs, 256u);
    stage_words(T + 1024, tabs + lc * 1024u, 10u * 256u);
    __syncthreads();
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint64_t b = blockIdx.x;
    uint32_t acc = 0;
    for (uint32_t i = 0; i < c; ++i) acc = (i ? tab_shift(T, acc) : 0u) ^ raw[b * s + t * c + i];
#pragma unroll
    for (uint32_t u = 0; u < 6; ++u) {  // lane l joins lane l + 2^u
        const uint32_t right = __shfl_down(acc, 1u << u);
        const uint32_t sh = tab_shift(T + (1u + u) * 1024u, acc);
        if ((lane & ((2u << u) - 1u)) == 0) acc = sh ^ right;
    }
    if (lane == 0) part[w] = acc;
    __syncthreads();
    if (w == 0) {
        acc = lane < 16u ? part[lane] : 0u;
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u) {
            const uint32_t right = __shfl_down(acc, 1u << u);
            const uint32_t sh = tab_shift(T + (7u + u) * 1024u, acc);
            if ((lane & ((2u << u) - 1u)) == 0) acc = sh ^ right;
        }
        if (lane == 0) {
            const uint32_t crc = ~acc;
            out[b] = (flags & LV_CRC_MASK) ? mask_crc(crc) : crc;
        }
    }
}

// Joins the pieces of the offsets API's split long buffers (sort_scatter,
// split_wave): long record {buffer, first piece slot, m, p}, pieces of
// P = 2^p bytes aligned to the buffer end; piece 0's register is
// R_0 = R(~seed, piece 0) and piece k > 0 was walked as a seed-0 buffer,
// part = R(~0, piece k) = R(0, piece k) ^ Shift_P(~0) (the seed trick), so
// R_k = part ^ Shift_P(~0) and R(~seed, buffer) = XOR_k Shift_{(m-1-k) P}(R_k).  One wave
// per buffer, Horner within lanes and a tree across them, every shift a
// wave-uniform base matrix (round 2 before: per-lane shifts by the set bits
// of m - 1 - k, 9.9 us for 64 x 16 MiB).  A lane's run of c pieces is up to
// 8 independent Horner chains joined by an in-lane tree: each Horner step is
// a dependent L2 round trip (~0.18 us), and 4,096 pieces are c = 64.
// base: Shift_{2^i} bytes, i < kBaseMats, as GF(2) matrices (32 columns).
constexpr uint32_t kBaseMats = 48;
#ifndef LVK_LONG_TABS
#define LVK_LONG_TABS 1
#endif
#ifndef LVK_LONG_LDSP  // Shift_P staged per wave for the Horner steps (d >= 2)
#define LVK_LONG_LDSP 1
#endif
__global__ __launch_bounds__(256) void combine_long_kernel(const uint32_t *__restrict__ ws,
                                                           const uint4 *__restrict__ longs,
                                                           const uint32_t *__restrict__ part,
                                                           const uint32_t *__restrict__ base,
                                                           const uint32_t *__restrict__ tabs,
                                                           uint32_t *__restrict__ out, uint32_t flags) {
    // the counter counts every claim; records exist only below the budget
    const uint32_t nl = min(ws[kWsLongs], kPieceBudget / 2);
    if (static_cast<uint64_t>(blockIdx.x) * (blockDim.x / 64) >= nl) return;  // block-uniform
#if !LVK_LONG_TABS
    __shared__ uint32_t M[kBaseMats * 32];
    for (uint32_t i = threadIdx.x; i < kBaseMats * 32; i += blockDim.x) M[i] = base[i];
    __syncthreads();
    auto shift = [&](uint32_t i, uint32_t v) { return gf2_apply(M + i * 32, v); };
#else
    // Shift_{2^i}(v) by four byte-table lookups (tables in HBM, L2-resident:
    // 192 KiB for every i) instead of a staged 32-column matrix product
    auto shift = [&](uint32_t i, uint32_t v) { return tab_shift(tabs + i * 1024u, v); };
#endif
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * (blockDim.x / 64);
#if LVK_LONG_TABS && LVK_LONG_LDSP
    __shared__ uint32_t TP[4][1024];  // per wave: Shift_P of its record
    uint32_t *const tp = TP[threadIdx.x >> 6];
#endif
    for (uint32_t w = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); w < nl; w += nw) {
        const uint4 r = longs[w];  // {buffer, first, m, p}
        const uint32_t m = r.z, p = r.w;
        if (m == 0) continue;  // a claim past the piece budget: the buffer was walked whole
        // pad the m pieces at the FRONT to 64 c (c = the power of two >= m / 64;
        // leading zero pieces add nothing): lane l runs Horner with Shift_P over
        // its c consecutive pieces, then a 6-level tree joins lane pairs with
        // Shift_{c 2^t P}.  Every matrix is wave-uniform (LDS broadcasts).
        uint32_t c = 1, lc = 0;
        while (64u * c < m) {
            c <<= 1;
            ++lc;
        }
        const uint32_t corr = shift(p, 0xffffffffu);  // Shift_P(~0)
        const int32_t pad = static_cast<int32_t>(64u * c - m);
        // chains q < Q of d = c / Q consecutive pieces each (wave-uniform)
        const uint32_t lq = lc < 3u ? lc : 3u, Q = 1u << lq, ld = lc - lq, d = 1u << ld;
        // Branch-free body (every chain's loads issued before any wait; a
        // guarded load per chain serialized them): chains q >= Q and front
        // padding read slot 0 and add 0.
        uint32_t ch[8];
        auto piece = [&](uint32_t q, uint32_t i) {
            const uint32_t j = lane * c + q * d + i;
            const bool ok = q < Q && j >= static_cast<uint32_t>(pad);
            const uint32_t k = ok ? j - static_cast<uint32_t>(pad) : 0u;
            const uint32_t v = part[r.y + k];
            return ok ? v ^ (k ? corr : 0u) : 0u;
        };
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q) ch[q] = piece(q, 0);
#if LVK_LONG_TABS && LVK_LONG_LDSP
        // d - 1 dependent Shift_P steps: from an LDS copy (one HBM round trip
        // to stage 4 KiB) instead of an L2 / HBM round trip each
        if (d > 1) {  // wave-uniform
            const uint4 *src = reinterpret_cast<const uint4 *>(tabs + p * 1024u);
            uint4 *dst = reinterpret_cast<uint4 *>(tp);
            const uint4 v0 = src[lane], v1 = src[64u + lane], v2 = src[128u + lane], v3 = src[192u + lane];
            __builtin_amdgcn_wave_barrier();  // the previous record's reads of tp are done
            dst[lane] = v0;
            dst[64u + lane] = v1;
            dst[128u + lane] = v2;
            dst[192u + lane] = v3;
            __builtin_amdgcn_wave_barrier();
        }
        for (uint32_t i = 1; i < d; ++i) {  // wave-uniform trip count
            uint32_t rk[8];
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q) rk[q] = piece(q, i);
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q) ch[q] = tab_shift(tp, ch[q]) ^ rk[q];
        }
#else
        for (uint32_t i = 1; i < d; ++i) {  // wave-uniform trip count
            uint32_t rk[8];
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q) rk[q] = piece(q, i);
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q) ch[q] = shift(p, ch[q]) ^ rk[q];
        }
#endif
#pragma unroll
        for (uint32_t t = 0; t < 3; ++t) {  // chain q joins chain q + 2^t: Shift_{d 2^t P}(left) ^ right
            if (t < lq) {
#pragma unroll
                for (uint32_t q = 0; q < 8; q += 2u << t) ch[q] = shift(p + ld + t, ch[q]) ^ ch[q + (1u << t)];
            }
        }
        uint32_t acc = ch[0];
#pragma unroll
        for (uint32_t t = 0; t < 6; ++t) {  // lane l joins lane l + 2^t: Shift_{c 2^t P}(left) ^ right
            const uint32_t right = __shfl_down(acc, 1u << t);
            const uint32_t sh = shift(p + lc + t, acc);
            if ((lane & ((2u << t) - 1u)) == 0) acc = sh ^ right;
        }
        if (lane == 0) {
            const uint32_t crc = ~acc;
            out[r.x] = (flags & LV_CRC_MASK) ? mask_crc(crc) : crc;
        }
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
// Kernel the calling thread's last batch call launched (lv_crc32c_last_kernel).
thread_local const char *g_kernel = "";

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
// The table walk's image: the G = 16 one with region A's row shift
// Shift_{256 kSstRows} (Shift_768 for three-row batches).
constexpr int kTableImage = 4;
constexpr int kImages = 5;

// Host copy of the LDS image for each G (index into kGs), and the table
// image; layout in lvk.
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

// Library-owned sort workspace of one (device, stream).  Calls on one stream
// are stream-ordered on the GPU, but two host threads enqueueing on the same
// stream would interleave their four kernels: `m` is held from the workspace
// lookup through the last launch of a call, so one call's sort passes are
// enqueued back to back and a growing hipFree never frees a buffer another
// thread has been handed but not yet launched on.
struct StreamWs {
    std::mutex m;
    uint8_t *p = nullptr;
    size_t cap = 0;
};

struct DevCtx {
    std::mutex m;  // one-time init
    bool ready = false;
    int cus = 0;
    uint4 *image[kImages] = {};  // per G (kGs), then the table image
    uint32_t *base_mats = nullptr;  // Shift_{2^i}, i < lvk::kBaseMats (combine_long_kernel)
    uint32_t *base_tabs = nullptr;  // the same shifts as byte tables (4 x 256 words each)
    std::mutex ws_m;  // guards the map (entries are never erased)
    std::map<hipStream_t, std::unique_ptr<StreamWs>> ws;
    // long-block split: Shift matrices per piece length (immutable once built)
    std::mutex mats_m;
    std::map<uint64_t, uint32_t *> piece_mats;
    std::map<uint64_t, uint32_t *> piece_tabs;
    // host-path staging (grown on demand), serialised by host_m
    std::mutex host_m;
    uint8_t *d_arena = nullptr;
    size_t d_arena_cap = 0;
    uint8_t *d_meta = nullptr;
    size_t d_meta_cap = 0;
    uint8_t *h_meta = nullptr;
    size_t h_meta_cap = 0;
    uint8_t *h_stage[2] = {nullptr, nullptr};
    size_t h_stage_cap[2] = {0, 0};
    hipEvent_t ev[2] = {nullptr, nullptr};
    hipStream_t stream = nullptr;
    uint8_t *d_scr[2] = {nullptr, nullptr};  // scratch for other host paths (WAL scan)
    size_t d_scr_cap[2] = {0, 0};
    int dev = 0;
};

constexpr size_t kStageBytes = 64ull << 20;  // pinned staging slot for pageable input

// lv_device_counters: per-device host-path traffic and allocations
struct DevCounters {
    std::atomic<uint64_t> h2d{0}, d2h{0}, allocs{0};
};
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
void par_memcpy(uint8_t *dst, const uint8_t *src, size_t bytes) {
    unsigned nt = std::thread::hardware_concurrency();
    nt = nt == 0 ? 1 : (nt > 8 ? 8 : nt);
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
            std::vector<uint32_t> bm(lvk::kBaseMats * 32);
            lvgpu::Gf2Mat m = lvgpu::shift_matrix(1);
            for (uint32_t i = 0; i < lvk::kBaseMats; ++i) {
                for (int j = 0; j < 32; ++j) bm[i * 32 + j] = m.col[j];
                m = m.then(m);  // Shift_{2^(i+1)}
            }
            LV_HIP(hipMalloc(&c.base_mats, bm.size() * 4));
            counters().allocs++;
            LV_HIP(hipMemcpy(c.base_mats, bm.data(), bm.size() * 4, hipMemcpyHostToDevice));
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
    lvk::Params P{};
    P.base = reinterpret_cast<uint64_t>(arena);
    P.off = off;
    P.len = len;
    P.seed = seed;
    P.out = out;
    P.n = n;
    P.stride = stride;
    P.blen = blen;
    P.flags = flags;
    P.ent = nullptr;
    P.sseed = nullptr;
    static const std::string name = std::string("crc32c_batch_kernel<") + std::to_string(G) +
                                    (STRIDED ? ",strided>" : ",offsets>");
    g_kernel = name.c_str();
    hipLaunchKernelGGL((lvk::crc32c_batch_kernel<G, STRIDED>), dim3(static_cast<uint32_t>(grid)),
                       dim3(lvk::kThreads), 0, s, P, c.image[gi]);
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

// Sorting workgroups and elements per workgroup for n buffers.
// At 4,096 buffers per workgroup a batch under 1M buffers leaves most CUs
// idle in the sort passes: batches under 4M split into up to kSortMinWgs
// workgroups of >= 1,024 (262,144 buffers: 64 -> 256 workgroups, +2 % for
// the whole call; 1M buffers: 256 -> 1,024, +0.1 %).
#ifndef LVK_SORT_MIN_WGS
#define LVK_SORT_MIN_WGS 1024
#endif
uint64_t sort_wgs(uint64_t n, uint64_t *chunk) {
    constexpr uint64_t kSortMinWgs = LVK_SORT_MIN_WGS;
    // small batches: >= 1 workgroup per 64 buffers (one wave each), so the
    // long-buffer split's piece writes spread over the grid (1,024 x 64 KiB:
    // one sorting workgroup wrote all 16,384 pieces, 33 us); the fewest
    // buffers go one (<= 256) or 16 (<= 4,096) per workgroup (64 x 16 MiB:
    // one wave wrote 64 x 256 pieces, 42 us)
    const uint64_t kSortMinChunk = n <= 256 ? 1 : n <= 4096 ? 16 : n < 65536 ? 64 : 1024;
    uint64_t wgs = (n + lvk::kSortChunk - 1) / lvk::kSortChunk;
    const uint64_t small = std::min(kSortMinWgs, (n + kSortMinChunk - 1) / kSortMinChunk);
    if (wgs < small) wgs = small;
    if (wgs > lvk::kSortMaxWgs) wgs = lvk::kSortMaxWgs;
    if (wgs == 0) wgs = 1;
    *chunk = (n + wgs - 1) / wgs;
    return wgs;
}

// Bytes of sort workspace the offsets API needs for n buffers: header,
// histogram matrix, n sorted 16-B entries, then n seeds in entry order.
// Byte offsets of the workspace regions (layout in lvk, "Sort workspace").
struct WsLayout {
    size_t m, wgb, ent, sseed, part, longs, total;
};

constexpr size_t al16(size_t x) { return (x + 15) & ~static_cast<size_t>(15); }

WsLayout ws_layout(uint64_t n) {
    uint64_t chunk = 0;
    const uint64_t wgs = sort_wgs(n, &chunk);
    const uint64_t ne = n + lvk::kPieceBudget;
    WsLayout w;
    w.m = lvk::kWsHeader * sizeof(uint32_t);
    w.wgb = w.m + al16(wgs * lvk::kKeys * sizeof(uint32_t));
    w.ent = w.wgb + al16(wgs * sizeof(uint64_t));
    w.sseed = w.ent + ne * sizeof(uint4);
    w.part = w.sseed + al16(ne * sizeof(uint32_t));
    w.longs = w.part + al16(lvk::kPieceBudget * sizeof(uint32_t));
    w.total = w.longs + (lvk::kPieceBudget / 2) * sizeof(uint4);
    return w;
}

size_t sort_ws_bytes(uint64_t n) { return ws_layout(n).total; }

// The library-owned workspace of (device, stream), grown on demand (the sort
// needs no initialised state).  Returns with the workspace's lock held in
// `lk`; the caller keeps it until its last launch has been enqueued.
int stream_ws_bytes(DevCtx &c, hipStream_t s, size_t need, uint8_t **out, std::unique_lock<std::mutex> *lk) {
    StreamWs *w = nullptr;
    {
        std::lock_guard<std::mutex> mk(c.ws_m);
        auto &slot = c.ws[s];
        if (!slot) slot.reset(new StreamWs);
        w = slot.get();
    }
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

// Long-block split of the strided API: log2 of the pieces per block, or 0.
// A batch of few long blocks keeps only n of the grid's 16-lane groups busy
// (one group walks a block), so blocks of >= 8 KiB are cut into 2^k pieces
// of >= 4 KiB (whole 1 KiB batches of the G = 16 blocks kernel) until the
// pieces fill one pass of the grid; combine_pieces_kernel joins them.
uint32_t pick_split(uint64_t base, uint64_t stride, uint64_t blen, uint64_t n, int forced, int cus) {
    if (forced >= 0 || base % 16 || stride % 16) return 0;
    const uint64_t want = 4ull * static_cast<uint64_t>(cus) * lvk::kWaves;
    uint32_t ps = 0;
    while ((n << ps) < want && ps < 12) {
        const uint64_t s2 = 2ull << ps;
        if (blen % s2 || (blen / s2) % 1024 || blen / s2 < 4096) break;
        ++ps;
    }
    return ps;
}
// Length-sorted launch of the offsets API, four kernels and no host sync:
// per-workgroup histograms, their column scan (+ key starts), the scatter
// into sorted entries, then the persistent class kernel.
int launch_binned(DevCtx &c, uint8_t *ws_bytes, const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                  const uint32_t *seed, uint32_t *out, uint64_t n, uint32_t flags, hipStream_t s) {
    uint32_t *ws = reinterpret_cast<uint32_t *>(ws_bytes);
    uint64_t chunk = 0;
    const uint64_t wgs = sort_wgs(n, &chunk);
    const WsLayout lay = ws_layout(n);
    uint32_t *M = reinterpret_cast<uint32_t *>(ws_bytes + lay.m);
    uint64_t *wgb = reinterpret_cast<uint64_t *>(ws_bytes + lay.wgb);
    uint4 *ent = reinterpret_cast<uint4 *>(ws_bytes + lay.ent);
    uint32_t *sseed = reinterpret_cast<uint32_t *>(ws_bytes + lay.sseed);
    uint32_t *part = reinterpret_cast<uint32_t *>(ws_bytes + lay.part);
    // long-buffer split (sort_scatter / combine_long_kernel); off for batches
    // whose buffer indices reach the piece flag bit
    uint4 *longs = n < lvk::kPieceFlag ? reinterpret_cast<uint4 *>(ws_bytes + lay.longs) : nullptr;
    const dim3 g(static_cast<uint32_t>(wgs)), b(lvk::kSortThreads);
    if (n <= lvk::kSmallSort && LVK_SMALL_SORT) {  // one launch (sort_small)
        const dim3 gs(static_cast<uint32_t>(std::max<uint64_t>(wgs, lvk::kSmallSortWgs)));
        hipLaunchKernelGGL(lvk::sort_small, gs, b, 0, s, off, len, n, chunk, ws, ent, seed, sseed, longs);
    } else {
        hipLaunchKernelGGL(lvk::sort_hist, g, b, 0, s, len, n, chunk, M, ws, wgb);
        hipLaunchKernelGGL(lvk::sort_scan, dim3(lvk::kScanWgs), dim3(lvk::kScanThreads), 0, s, M,
                           static_cast<uint32_t>(wgs), ws, wgb);
        hipLaunchKernelGGL(lvk::sort_scatter, g, b, 0, s, off, len, n, chunk, ws, M, ent, seed, sseed, longs);
    }
    lvk::Params P{};
    P.base = reinterpret_cast<uint64_t>(arena);
    P.off = off;
    P.len = len;
    P.seed = seed;
    P.out = out;
    P.n = n;
    P.stride = 0;
    P.blen = 0;
    P.flags = flags;
    P.ent = ent;
    P.sseed = seed ? sseed : nullptr;
    P.nplain = n;
    P.part = longs ? part : nullptr;
    g_kernel = "sort+crc32c_classes_kernel";
    if (seed)
        hipLaunchKernelGGL(lvk::crc32c_classes_kernel<true>, dim3(static_cast<uint32_t>(c.cus)), dim3(lvk::kThreads), 0,
                           s, P, c.image[2], ws);
    else
        hipLaunchKernelGGL(lvk::crc32c_classes_kernel<false>, dim3(static_cast<uint32_t>(c.cus)), dim3(lvk::kThreads),
                           0, s, P, c.image[2], ws);
    // joins split long buffers (exits at once when the sort split none).  (A
    // last-finisher join inside the class kernel -- agent-scope release and
    // acquire around a per-buffer counter -- measured 64 x 16 MiB 200 -> 345
    // us and 1,024 x 64 KiB 41 -> 177 us: every fence writes back or
    // invalidates the XCD's whole L2; and C3 via offsets -2 % from spills.)
    if (longs)
        hipLaunchKernelGGL(lvk::combine_long_kernel, dim3(static_cast<uint32_t>(c.cus)), dim3(256), 0, s, ws, longs,
                           part, c.base_mats, c.base_tabs, out, flags);
    return 0;
}

// Group size for the uniform-block kernel, or -1 when the blocks are not
// 16-B aligned whole batches for any supported G.
int pick_block_gi(uint64_t base, uint64_t stride, uint64_t blen, int forced, uint64_t n, int cus) {
    if (blen == 0 || base % 16 || stride % 16) return -1;
    auto fits = [&](int gi) { return blen % (16ull * kGs[gi] * lvk::U) == 0; };
    if (forced >= 0) return fits(forced) ? forced : -1;
    // Few blocks: 16-lane groups would keep only n/4 of the grid's waves
    // busy, each walking its blocks alone; 64-lane groups put n waves on them.
    if (n < 4ull * static_cast<uint64_t>(cus) * lvk::kWaves && fits(3)) return 3;
    for (int gi : {2, 1, 0})
        if (fits(gi)) return gi;
    return -1;
}

template <int G>
void launch_blocks_g(const DevCtx &c, int gi, const uint8_t *base, uint64_t stride, uint32_t blen,
                     uint64_t n, const uint32_t *seed, uint32_t *out, uint32_t flags, hipStream_t s) {
    const uint64_t groups_per_wg = static_cast<uint64_t>(lvk::kWaves) * (64 / G);
    uint64_t grid = (n + groups_per_wg - 1) / groups_per_wg;
    if (grid > static_cast<uint64_t>(c.cus)) grid = c.cus;
    if (grid == 0) grid = 1;
    lvk::Params P{};
    P.base = reinterpret_cast<uint64_t>(base);
    P.off = nullptr;
    P.len = nullptr;
    P.seed = seed;
    P.out = out;
    P.n = n;
    P.stride = stride;
    P.blen = blen;
    P.flags = flags;
    P.ent = nullptr;
    P.sseed = nullptr;
    const uint32_t nb = static_cast<uint32_t>(blen / (16ull * G * lvk::U));
    static const std::string name = "crc32c_blocks_kernel<" + std::to_string(G) + ">";
    g_kernel = name.c_str();
    if (seed)
        hipLaunchKernelGGL((lvk::crc32c_blocks_kernel<G, true>), dim3(static_cast<uint32_t>(grid)),
                           dim3(lvk::kThreads), 0, s, P, nb, c.image[gi]);
    else
        hipLaunchKernelGGL((lvk::crc32c_blocks_kernel<G, false>), dim3(static_cast<uint32_t>(grid)),
                           dim3(lvk::kThreads), 0, s, P, nb, c.image[gi]);
}

void launch_blocks(const DevCtx &c, int gi, const uint8_t *base, uint64_t stride, uint32_t blen,
                   uint64_t n, const uint32_t *seed, uint32_t *out, uint32_t flags, hipStream_t s) {
    switch (gi) {
        case 0: launch_blocks_g<1>(c, gi, base, stride, blen, n, seed, out, flags, s); break;
        case 1: launch_blocks_g<4>(c, gi, base, stride, blen, n, seed, out, flags, s); break;
        case 2: launch_blocks_g<16>(c, gi, base, stride, blen, n, seed, out, flags, s); break;
        default: launch_blocks_g<64>(c, gi, base, stride, blen, n, seed, out, flags, s); break;
    }
}

int check_launch() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return set_err(static_cast<int>(e), std::string("kernel launch: ") + hipGetErrorString(e));
    return 0;
}

}  // namespace

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

int lv_device_init(void) {
    DevCtx *c = nullptr;
    return current_ctx(&c);
}

static int batch_device_impl(const uint8_t *d_arena, const uint64_t *d_off, const uint32_t *d_len,
                             const uint32_t *d_seed, uint32_t *d_out, size_t n, uint32_t flags,
                             void *stream, uint8_t *d_ws, size_t ws_bytes) {
    g_err.clear();
    if (n == 0) return LV_OK;
    if (!d_arena || !d_off || !d_len || !d_out) return set_err(LV_ERR_INVALID, "null device pointer");
    if (n > 0xffffffffull) return set_err(LV_ERR_INVALID, "more than 2^32-1 buffers per call");
    DevCtx *c = nullptr;
    if (int rc = current_ctx(&c)) return rc;
    const int gi = forced_gi(flags);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (gi >= 0) {
        launch_g<false>(*c, gi, d_arena, d_off, d_len, 0, 0, d_seed, d_out, n, flags, s);
        return check_launch();
    }
    std::unique_lock<std::mutex> ws_lk;  // held through the last launch (library workspace)
    if (d_ws) {
        if (ws_bytes < sort_ws_bytes(n)) return set_err(LV_ERR_INVALID, "workspace too small");
        if (reinterpret_cast<uintptr_t>(d_ws) % 16) return set_err(LV_ERR_INVALID, "workspace must be 16-byte aligned");
        // no initialisation: every workspace word the sort reads, it wrote first
    } else if (int rc = stream_ws(*c, s, n, &d_ws, &ws_lk)) {
        return rc;
    }
    if (int rc = launch_binned(*c, d_ws, d_arena, d_off, d_len, d_seed, d_out, n, flags, s)) return rc;
    return check_launch();
}

int lv_crc32c_batch_device(const uint8_t *d_arena, const uint64_t *d_off, const uint32_t *d_len,
                           const uint32_t *d_seed, uint32_t *d_out, size_t n, uint32_t flags,
                           void *stream) {
    return batch_device_impl(d_arena, d_off, d_len, d_seed, d_out, n, flags, stream, nullptr, 0);
}

size_t lv_crc32c_workspace_bytes(size_t n) { return sort_ws_bytes(n); }

int lv_crc32c_batch_device_ws(const uint8_t *d_arena, const uint64_t *d_off, const uint32_t *d_len,
                              const uint32_t *d_seed, uint32_t *d_out, size_t n, uint32_t flags,
                              void *d_workspace, size_t workspace_bytes, void *stream) {
    if (!d_workspace) return set_err(LV_ERR_INVALID, "null workspace");
    return batch_device_impl(d_arena, d_off, d_len, d_seed, d_out, n, flags, stream,
                             static_cast<uint8_t *>(d_workspace), workspace_bytes);
}

// ---- WAL scan of a log in HBM (include/lvgpu/wal.h) ----
static uint64_t wal_wgs(uint64_t nblocks, uint64_t *chunk) {
    uint64_t wgs = (nblocks + lvk::kSortThreads - 1) / lvk::kSortThreads;
    wgs = std::max<uint64_t>(1, std::min<uint64_t>(wgs, lvk::kSortMaxWgs));
    *chunk = (nblocks + wgs - 1) / wgs;
    return wgs;
}

struct WalWs {
    size_t m, wgrec, blk, hc, ent, total;
};

static WalWs wal_ws_layout(uint64_t bytes, uint64_t cap) {
    const uint64_t nblocks = (bytes + lvk::kWalBlock - 1) / lvk::kWalBlock;
    uint64_t chunk = 0;
    const uint64_t wgs = wal_wgs(nblocks, &chunk);
    WalWs w;
    w.m = lvk::kWsHeader * sizeof(uint32_t);
    w.wgrec = w.m + al16(wgs * lvk::kKeys * sizeof(uint32_t));
    w.blk = w.wgrec + al16(wgs * sizeof(uint64_t));
    w.hc = w.blk + al16(nblocks * sizeof(uint32_t));
    w.ent = w.hc + nblocks * lvk::kHdrCache * sizeof(uint64_t);
    w.total = w.ent + cap * sizeof(uint4);
    return w;
}

size_t lv_wal_scan_workspace_bytes(size_t bytes, size_t cap) { return wal_ws_layout(bytes, cap).total; }

int lv_wal_scan_device(const uint8_t *d_log, size_t bytes, uint64_t *d_hdr_off, uint32_t *d_crc, uint32_t *d_info,
                       size_t cap, uint64_t *d_count, void *d_workspace, size_t workspace_bytes, void *stream) {
    g_err.clear();
    if (!d_count) return set_err(LV_ERR_INVALID, "null count pointer");
    if ((!d_log && bytes) || (cap && (!d_hdr_off || !d_crc || !d_info)) || !d_workspace)
        return set_err(LV_ERR_INVALID, "null device pointer");
    if (reinterpret_cast<uintptr_t>(d_log) % 8) return set_err(LV_ERR_INVALID, "log must be 8-byte aligned");
    if (reinterpret_cast<uintptr_t>(d_workspace) % 16) return set_err(LV_ERR_INVALID, "workspace must be 16-byte aligned");
    if (bytes / lvk::kWalHeader >= 0xffffffffull || cap > 0xffffffffull)
        return set_err(LV_ERR_INVALID, "log too large for one scan");
    const WalWs lay = wal_ws_layout(bytes, cap);
    if (workspace_bytes < lay.total) return set_err(LV_ERR_INVALID, "workspace too small");
    DevCtx *c = nullptr;
    if (int rc = current_ctx(&c)) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint64_t nblocks = (bytes + lvk::kWalBlock - 1) / lvk::kWalBlock;
    if (nblocks == 0) {
        LV_HIP(hipMemsetAsync(d_count, 0, sizeof(uint64_t), s));
        return LV_OK;
    }
    uint8_t *wb = static_cast<uint8_t *>(d_workspace);
    uint32_t *ws = reinterpret_cast<uint32_t *>(wb);
    uint32_t *M = reinterpret_cast<uint32_t *>(wb + lay.m);
    uint64_t *wgrec = reinterpret_cast<uint64_t *>(wb + lay.wgrec);
    uint32_t *blk = reinterpret_cast<uint32_t *>(wb + lay.blk);
    uint64_t *hc = reinterpret_cast<uint64_t *>(wb + lay.hc);
    uint4 *ent = reinterpret_cast<uint4 *>(wb + lay.ent);
    uint64_t chunk = 0;
    const uint64_t wgs = wal_wgs(nblocks, &chunk);
    const dim3 g(static_cast<uint32_t>(wgs)), b(lvk::kSortThreads);
    hipLaunchKernelGGL(lvk::wal_hist, g, b, 0, s, d_log, static_cast<uint64_t>(bytes), nblocks, chunk, M, wgrec, blk,
                       hc);
    hipLaunchKernelGGL(lvk::sort_scan, dim3(lvk::kScanWgs), dim3(lvk::kScanThreads), 0, s, M,
                       static_cast<uint32_t>(wgs), ws, wgrec);
    lvk::WalOut o{d_hdr_off, d_info, d_count, cap};
    hipLaunchKernelGGL(lvk::wal_scatter, g, b, 0, s, d_log, static_cast<uint64_t>(bytes), nblocks, chunk, ws, M, wgrec,
                       blk, hc, ent, o);
    lvk::Params P{};
    P.base = reinterpret_cast<uint64_t>(d_log);
    P.out = d_crc;
    P.n = cap;
    P.nplain = cap;
    P.ent = ent;
    hipLaunchKernelGGL(lvk::crc32c_classes_kernel<false>, dim3(static_cast<uint32_t>(c->cus)), dim3(lvk::kThreads), 0,
                       s, P, c->image[2], ws);
    g_kernel = "wal_hist+sort_scan+wal_scatter+crc32c_classes_kernel";
    return check_launch();
}

int lv_crc32c_batch_strided(const uint8_t *d_base, uint64_t stride, uint32_t block_len, size_t n,
                            const uint32_t *d_seed, uint32_t *d_out, uint32_t flags, void *stream) {
    g_err.clear();
    if (n == 0) return LV_OK;
    if (!d_base || !d_out) return set_err(LV_ERR_INVALID, "null device pointer");
    if (n > 0xffffffffull) return set_err(LV_ERR_INVALID, "more than 2^32-1 buffers per call");
    DevCtx *c = nullptr;
    if (int rc = current_ctx(&c)) return rc;
    const int gi = forced_gi(flags);
    hipStream_t hs = static_cast<hipStream_t>(stream);
    const uint32_t ps = pick_split(reinterpret_cast<uint64_t>(d_base), stride, block_len, n, gi, c->cus);
    if (ps > 0) {
        const uint64_t nv = static_cast<uint64_t>(n) << ps, plen = block_len >> ps;
        const uint32_t *mats = nullptr;
        if (int rc = piece_mats(*c, plen, &mats)) return rc;
        const uint32_t nb = static_cast<uint32_t>(plen / (16ull * 16 * lvk::U));
        if ((1u << ps) <= lvk::kFuseMax && nv <= 64ull * static_cast<uint64_t>(c->cus)) {
            // one round of the grid: each workgroup joins its own blocks' pieces
            lvk::Params P{};
            P.base = reinterpret_cast<uint64_t>(d_base);
            P.seed = d_seed;
            P.out = d_out;
            P.n = nv;
            P.stride = stride;
            P.blen = static_cast<uint32_t>(plen);
            P.flags = flags;
            P.plen = plen;
            P.pshift = ps;
            P.mats = mats;
            const dim3 grid(static_cast<uint32_t>((nv + 63) / 64));
            if (d_seed)
                hipLaunchKernelGGL((lvk::crc32c_blocks_kernel<16, true, true, true>), grid, dim3(lvk::kThreads), 0, hs,
                                   P, nb, c->image[2]);
            else
                hipLaunchKernelGGL((lvk::crc32c_blocks_kernel<16, false, true, true>), grid, dim3(lvk::kThreads), 0,
                                   hs, P, nb, c->image[2]);
            g_kernel = "crc32c_blocks_kernel<16,pieces,fused>";
            return check_launch();
        }
        uint8_t *scr = nullptr;
        std::unique_lock<std::mutex> ws_lk;  // held through both launches
        if (int rc = stream_ws_bytes(*c, hs, nv * 4, &scr, &ws_lk)) return rc;
        lvk::Params P{};
        P.base = reinterpret_cast<uint64_t>(d_base);
        P.seed = d_seed;
        P.out = reinterpret_cast<uint32_t *>(scr);
        P.n = nv;
        P.stride = stride;
        P.blen = static_cast<uint32_t>(plen);
        P.plen = plen;
        P.pshift = ps;
        const uint64_t grid = std::min<uint64_t>(c->cus, (nv + 63) / 64);
        if (d_seed)
            hipLaunchKernelGGL((lvk::crc32c_blocks_kernel<16, true, true>), dim3(static_cast<uint32_t>(grid)),
                               dim3(lvk::kThreads), 0, hs, P, nb, c->image[2]);
        else
            hipLaunchKernelGGL((lvk::crc32c_blocks_kernel<16, false, true>), dim3(static_cast<uint32_t>(grid)),
                               dim3(lvk::kThreads), 0, hs, P, nb, c->image[2]);
        const uint32_t *tabs = nullptr;
        if (int rc = piece_tabs(*c, plen, &tabs)) return rc;
        if (ps >= 11) {  // > 1,024 pieces per block: a workgroup per block
            hipLaunchKernelGGL(lvk::combine_pieces_wg_kernel, dim3(static_cast<uint32_t>(n)), dim3(1024), 0, hs, P.out,
                               1u << ps, tabs, d_out, flags);
            g_kernel = "crc32c_blocks_kernel<16,pieces>+combine_pieces_wg_kernel";
        } else {
            hipLaunchKernelGGL(lvk::combine_pieces_kernel,
                               dim3(static_cast<uint32_t>(std::min<uint64_t>(1024, (n + 3) / 4))), dim3(256), 0, hs,
                               P.out, static_cast<uint64_t>(n), 1u << ps, mats, d_out, flags);
            g_kernel = "crc32c_blocks_kernel<16,pieces>+combine_pieces_kernel";
        }
        return check_launch();
    }
    // Aligned whole-batch blocks take the uniform-block kernel.
    const int bgi = pick_block_gi(reinterpret_cast<uint64_t>(d_base), stride, block_len, gi, n, c->cus);
    if (bgi >= 0) {
        launch_blocks(*c, bgi, d_base, stride, block_len, n, d_seed, d_out, flags,
                      static_cast<hipStream_t>(stream));
        return check_launch();
    }
    launch_g<true>(*c, gi >= 0 ? gi : pick_gi(block_len), d_base, nullptr, nullptr, stride, block_len, d_seed,
                   d_out, n, flags, static_cast<hipStream_t>(stream));
    return check_launch();
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

// SSTable trailers (csrc/sst.hip): one sst_blocks_kernel launch.
#ifndef LVK_VERIFY_WIDE  // experiment: the four-word verify staging even without crc_out
#define LVK_VERIFY_WIDE 0
#endif
int launch_sst_blocks(bool seal, const uint8_t *d_file, uint64_t file_bytes, const uint64_t *d_handles,
                      const uint8_t *d_types, size_t n, uint32_t *d_status, uint32_t *d_crc, void *stream) {
    DevCtx *c = nullptr;
    if (int rc = current_ctx(&c)) return rc;
    lvk::Params P{};
    P.base = reinterpret_cast<uint64_t>(d_file);
    P.n = n;
    P.flags = 0;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 grid(static_cast<uint32_t>(std::min<uint64_t>(c->cus, (n + 3) / 4))), block(lvk::kThreads);
    if (seal) {
        lvk::TableUnits<true> u{reinterpret_cast<const uint2 *>(d_handles), d_types, nullptr, nullptr, file_bytes};
        g_kernel = "sst_blocks_kernel<seal>";
        hipLaunchKernelGGL((lvk::sst_blocks_kernel<true, false>), grid, block, 0, s, P, c->image[kTableImage], u);
    } else if (d_crc || LVK_VERIFY_WIDE) {
        lvk::TableUnits<false, true> u{reinterpret_cast<const uint2 *>(d_handles), nullptr, d_status, d_crc, file_bytes};
        g_kernel = "sst_blocks_kernel<verify,crc>";
        hipLaunchKernelGGL((lvk::sst_blocks_kernel<false, true>), grid, block, 0, s, P, c->image[kTableImage], u);
    } else {
        lvk::TableUnits<false, false> u{reinterpret_cast<const uint2 *>(d_handles), nullptr, d_status, nullptr,
                                        file_bytes};
        g_kernel = "sst_blocks_kernel<verify>";
        hipLaunchKernelGGL((lvk::sst_blocks_kernel<false, false>), grid, block, 0, s, P, c->image[kTableImage], u);
    }
    return check_launch();
}

void count_h2d(uint64_t bytes) { counters().h2d += bytes; }
void count_d2h(uint64_t bytes) { counters().d2h += bytes; }

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
    if (int rc = launch_binned(*c, ws, c->d_arena, d_off, d_len, h_seed ? d_seed : nullptr, d_out, n, flags, s))
        return rc;
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
