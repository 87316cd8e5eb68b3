// MI355X (gfx950 / CDNA4) batched CRC32C: device building blocks shared by
// every kernel (lvk/core.h).
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
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../../include/lvgpu/crc32c.h"
#include "knobs.h"

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

static __shared__ __attribute__((aligned(16))) uint32_t g_lds[kImageWords];

// Per-wave output staging (8 KiB; with the image, exactly the 160 KiB of a
// CU).  Results go to LDS and leave in one global store per wave every few
// rounds.  A global store in the batch loop costs a pipeline drain: on gfx9
// stores count in vmcnt, the register allocator soon reuses the store's
// registers, and waiting for the store waits (in order) for every prefetch
// load issued before it.
static __shared__ uint32_t g_oidx[kWaves][64];
static __shared__ uint32_t g_ocrc[kWaves][64];
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
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // (round 1: 78.6 % with plain xors -> 80.5 %)
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
// NU rows per batch; W4OFF = LDS offset of the Latin row-shift table (the
// image's W4 = Shift_{64G}, or region B's W2 = Shift_{32G} for NU = 2).
// SKIP (FIRST batches only): the leading rows that hold no buffer byte for
// any group of the wave are not folded (their accumulators start at 0, as a
// fold of zero granules would leave them).
template <bool FIRST, int W4K = -1, uint32_t NU = U, uint32_t W4OFF = kRegionA + kHalf, uint32_t SKIP = 0>
__device__ __forceinline__ void fold_batch(const uint4 (&v)[NU], uint32_t (&A)[NU], const Lut &L) {
    static_assert(SKIP == 0 || FIRST, "only a first batch skips rows");
    static_assert(SKIP < NU, "at least one row");
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
    uint32_t *tmp;          // class kernel, sorted list: CRCs by sorted position (combine_long_kernel unsorts), or null
    const uint32_t *mats;   // blocks kernel, FUSE: Shift_{j plen}, j < 2^pshift (32 column words each)
    const uint32_t *tabs;   // fused small-batch kernel: the byte tables Shift_{2^i}, 1,024 words each
    // class kernel, lv_crc32c_batch_device_hint: a uniform batch none of whose
    // buffers can split is one sort key in index order, known on the host --
    // no sort runs; hident = 1 + its length class (0: the sort's ranges)
    uint32_t hident;
    // The hint's facts, checked where a kernel reads what they describe
    // (lv_crc32c_batch_check): violations are or-ed into *herr as
    // LV_HINT_ERR_* bits.  herr null: no hint to check (hlen / htotal unused).
    uint32_t *herr;
    uint64_t htotal;  // the hint's total_bytes
    uint32_t hlen;    // the hint's max_len
    uint32_t huni;    // the hint's uniform word
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

// R = sum of the columns of m selected by the bits of v (a GF(2) matrix-vector product).
__device__ __forceinline__ uint32_t gf2_apply(const uint32_t *m, uint32_t v) {
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) r ^= (v >> j & 1u) ? m[j] : 0u;
    return r;
}

constexpr uint32_t kPow2Tabs = 13;  // Shift_{2^v plen}, v <= 12 (s <= 4,096)

__device__ __forceinline__ uint32_t tab_shift(const uint32_t *t, uint32_t a) {
    return t[a & 0xffu] ^ t[256 + ((a >> 8) & 0xffu)] ^ t[512 + ((a >> 16) & 0xffu)] ^ t[768 + (a >> 24)];
}

// Stage n4 uint4 of `src` into LDS `dst`: 16-B loads in batches of four per
// thread, each batch issued before its first LDS store (a plain copy loop
// waits for every load before the next: one L2 round trip per 16 B per
// thread).
__device__ __forceinline__ void stage_words(uint32_t *dst, const uint32_t *src, uint32_t n4) {
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
    uint4 *d4 = reinterpret_cast<uint4 *>(dst);
    const uint32_t b = blockDim.x;
    uint32_t i = threadIdx.x;
    for (; i + 3u * b < n4; i += 4u * b) {  // named registers: an array here went to LDS
        const uint4 v0 = s4[i], v1 = s4[i + b], v2 = s4[i + 2u * b], v3 = s4[i + 3u * b];
        d4[i] = v0;
        d4[i + b] = v1;
        d4[i + 2u * b] = v2;
        d4[i + 3u * b] = v3;
    }
    for (; i < n4; i += b) d4[i] = s4[i];
}

// The base shifts Shift_{2^i} bytes, i < kBaseMats, as byte tables (DevCtx::base_tabs).
constexpr uint32_t kBaseMats = 48;

// Rows per batch of the table walk.  A 4,097-4,352-B unit at a byte-packed
// start spans 17-19 rows of the 256-B grid: 5 four-row batches (20 rows) or
// 6 three-row batches (18 rows, with Shift_768 as the batch shift: the table
// image, host_image(kTableImage)).
constexpr uint32_t kSstRows = LVK_SST_ROWS;
static_assert(kSstRows == 3 || kSstRows == 4, "table walk: 3 or 4 rows per batch");
constexpr uint32_t kSealRows = LVK_SEAL_ROWS;  // the seal's rows per batch (4: on the G = 16 image)
static_assert(kSealRows == kSstRows || kSealRows == 4, "seal: the table image's rows, or 4 on the G = 16 image");

}  // namespace lvk
