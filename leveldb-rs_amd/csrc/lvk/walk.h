// The wave-uniform walk of length-sorted entries (offsets API, WAL units)
// and of file-ordered units (SST blocks): geometry, the 256-B-aligned row
// batches, fix-ups, merge and the sorted_stream loop with its Src policies.
#pragma once
#include "sort.h"

namespace lvk {

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
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v, int from) {
    for (int m = from; m < 64; m <<= 1) {
        uint32_t o;
        if (m == 16) {
            const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
            o = r[0] > r[1] ? r[0] : r[1];
        } else if (m == 32) {
            const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
            o = r[0] > r[1] ? r[0] : r[1];
        } else {
            o = __shfl_xor(v, m);
        }
        v = o > v ? o : v;
    }
    return __builtin_amdgcn_readfirstlane(v);
}

// Geometry of sorted entry e (clamped to the last entry for lanes past the
// end, so every address stays valid).  Seeds come pre-sorted (sort_scatter),
// so no load depends on another.
// bid: the entry's output slot -- its buffer index (v.w), a piece slot
// (kPieceFlag), ~0u for a split buffer's own entry; with P.tmp the sorted
// position instead of the buffer index, so a wave's results land in runs of
// K consecutive words (combine_long_kernel moves them to out[]; scattered
// single-word stores into out[] cost C2 ~35 us, profiles/r04/outstore/).
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
    const bool piece = P.nplain < P.n && (v.w & kPieceFlag) && v.w != 0xffffffffu;
    const uint32_t slot = P.tmp && !piece && v.w != 0xffffffffu ? static_cast<uint32_t>(ec) : v.w;
    q.bid = valid ? slot : 0xffffffffu;
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

// Granules outside a buffer load from this zero block (load_rbatch_al, and
// in the exact wait-count mode every lane's tail).
static __device__ __attribute__((aligned(256))) uint4 g_zero_granules[16];  // zero-initialised

// The granule after the last whole granule (k = (alow+len) & 15 bytes of it
// belong to the buffer).
template <bool EXACT = false>
__device__ __forceinline__ uint4 load_rtail(const RGeo &q, uint32_t gl) {
    if constexpr (EXACT) {  // every lane loads (others: the zero block): no exec-masked load
        const bool on = gl == 0 && ((q.alow() + q.len) & 15u);
        return load16_rt(on ? q.abase() + (static_cast<uint64_t>(q.ng()) << 4)
                            : reinterpret_cast<uint64_t>(&g_zero_granules[gl & 15u]));
    }
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

// jfix: the round's last head batch (round_jfix_al).  Past it and before the
// last batch every group's granules lie inside its buffer (a group's rows end
// at its last whole granule's row, and only that row holds granules past the
// end), so those batches take plain addresses, no range selects (C2 / C4 /
// WAL +0.3-1 %; the table walk, 6 batches of 3 rows per unit, measured
// -0.7 % and passes no jfix: Src::kAlMid, profiles/r03/walk/ab_al_mid.txt).
template <uint32_t NU>
__device__ __forceinline__ void load_rbatch_al(const RGeo &q, uint32_t nbw, uint32_t j, uint32_t gl,
                                               uint4 (&v)[NU], uint32_t jfix = 0xffffffffu) {
    const AGeo g = al_geo(q);
    const uint64_t ab = q.abase();
    if (jfix != 0xffffffffu && j > jfix && j + 1u < nbw) {  // wave-uniform
        const uint64_t a0 = ab + (static_cast<uint64_t>(static_cast<uint32_t>(
                                      16 * al_row<NU>(g, nbw, j, 0) + static_cast<int32_t>(gl) - g.ph)) << 4);
#pragma unroll
        for (uint32_t i = 0; i < NU; ++i) v[i] = load16(a0 + 256u * i);
        return;
    }
    const int32_t dmax = static_cast<int32_t>(q.ng()) - 1;
#pragma unroll
    for (uint32_t i = 0; i < NU; ++i) {
        const int32_t d = 16 * al_row<NU>(g, nbw, j, i) + static_cast<int32_t>(gl) - g.ph;
        const uint64_t ad = (d < 0 || d > dmax) ? reinterpret_cast<uint64_t>(&g_zero_granules[gl])
                                                : ab + (static_cast<uint32_t>(d) << 4);
        v[i] = load16(ad);
    }
}

// Head fix-up (as fix_rbatch); granules outside [0, dmax] were loaded from
// the zero block.
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
        if ((d == 0 || (d == 1 && alow > 12)) && d <= dmax) {
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
    if constexpr (NU == 4) {
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
template <int G, uint32_t NU>
__device__ __forceinline__ uint32_t round_pad(const RGeo &q, uint32_t nbw) {
    uint32_t padg;
    if constexpr (G == 16) {
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
    fold_batch<true, W4K, NU, W4OFF>(v, A, L);
}

// The raw register R(~seed, buffer) (lane 0 of the group), before the final
// xor and mask: the tail bytes, then the short-buffer seed.
__device__ __forceinline__ uint32_t finish_raw(const RGeo &q, uint32_t X, const uint4 &tail, uint32_t gl,
                                               const Lut &L) {
    X = fold_tail(X, tail, q, L);
    if (gl == 0 && q.len < 4) {  // R(s, D) = R(0, D) ^ Shift_|D|(s) for short buffers
        uint32_t s = ~q.seed;
        for (uint32_t i = 0; i < q.len; ++i) s = byte_step(s, 0u);
        X ^= s;
    }
    return X;
}

// s_waitcnt immediate that waits for vmcnt <= n only (gfx9 encoding:
// vmcnt bits 3:0 and 15:14, expcnt 6:4 and lgkmcnt 11:8 at their maxima).
constexpr int vmcnt_only(uint32_t n) {
    return static_cast<int>((n & 15u) | ((n >> 4) << 14) | (7u << 4) | (15u << 8));
}

// Entry source and result sink of the sorted walk: the offsets API's
// length-sorted list.  load() reads entry e; trailer() issues any extra
// per-unit loads with the tail load; stage() parks a unit's result in the
// wave's LDS slots (lane 0 of the group); flush() stores the parked results
// of the last rounds, one global store per lane, every kFlush rounds.
template <bool SEEDED>
struct SortedList {
    static constexpr uint32_t kFlush = 16;  // 64 slots of one word pair
    static constexpr bool kAlMid = true;    // plain addresses in middle batches (load_rbatch_al)
    static constexpr bool kOneRound = false;  // sorted_stream's one-round path (FusedUnits)
    static constexpr uint32_t kExact = 0;  // sorted_stream: wait-count mode (below)
    // sorted_stream: explicit wait for the batch it folds (with kExact 2:
    // C2 flat, C4 -0.4 %, C3 via offsets -2.5 %, the WAL scan flat,
    // profiles/r06/curwait/; the seal keeps it)
    static constexpr bool kCurWait = false;
    static constexpr uint32_t kTrailerLoads = 0;
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
            (P.tmp && !ident ? P.tmp : P.out)[bi] = cv;  // (an identity list is in buffer order already)
    }
};

// One wave walks rounds of the sorted list: round rho holds entries
// rho*K + group (K = 64/G groups).  The rounds come from `next()` (a static
// stride, or a workgroup's shared pool) until it returns rho >= nr.  Batches
// are prefetched one ahead, across rounds, in two ping-pong register slots;
// all control is wave-uniform.  Results are staged in LDS (g_oidx/g_ocrc)
// and stored every G rounds.
// Wait counts (round 4): the compiler counts loads in flight per path and
// merges paths by their minimum, so a load that only some paths issue (an
// exec-masked tail load, the next round's loads under `more`) makes the
// fold of a batch wait with vmcnt(0..3) -- also for the prefetch issued
// just before it.  Src::kExact selects the load form: 0 = masked loads;
// 2 = unconditional loads within each path (the next round's entries and
// first batch always, clamped).  (Mode 1, the same loads every step with the
// tail and trailer re-read, was measured and removed.)  Exact waits (vmcnt(8..5) in the
// fold) measured, against mode 0 on one box (profiles/r04/walk_modes/,
// mode2_ab/): class kernel mode 1 / 2 -- C3 via offsets -2.5 / -3 %, C2 0,
// C4 -0.6 %, WAL scan +0.6 / -0.3 % -- so it keeps mode 0 (16 waves per CU
// hide the exposed round trip); SST verify mode 2 +2.8 % (0.703 -> 0.723,
// final_ab/), the seal -4 % (it kept mode 0 until round 6, when mode 2 with
// Src::kCurWait -- one explicit s_waitcnt for the folded batch after this
// step's loads -- took it 0.665-0.669 -> 0.683-0.688: the compiler's own
// merge had still waited vmcnt(0) in the head batches' fix-up, i.e. for the
// prefetch too); the fused small-batch kernel +0.5-1.3 us (mode 0).
// (Round 2 issued the same loads in every step by re-reading the entries
// each batch as well: 4-5 % slower from extra loads and spills.)
template <int G, class Src, class Next, uint32_t ALR = kAlRows>
__device__ __forceinline__ void sorted_stream(const Params &P, const Src &src, uint32_t lane, const Lut &L,
                                              uint64_t rho, Next next) {
    constexpr bool AL = G == 16;  // 256-B-aligned rows (merge_al)
    // exact wait counts (below): Src::kExact 0 = masked loads, 2 =
    // unconditional loads within each path
    static_assert(Src::kExact == 0 || Src::kExact == 2, "wait-count mode 0 or 2");
    constexpr bool EX = Src::kExact != 0;
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
    if (EX || rhon < nr) qn = src.load(P, rhon * K + grp);
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
    if constexpr (AL && Src::kOneRound && NU == 4) {
        // The wave's only round, <= 4 batches (a batch of <= 1,024 one-round
        // units: the pieces of a few long buffers): every batch's loads are
        // requested at once -- one memory round trip for the walk instead of
        // one per batch (the strided API's FUSE path does the same).  Missing
        // batches reload batch 0 (branch-free: guarded loads made the
        // compiler wait for each).
        if (rhon >= nr && nbw <= 4u) {  // wave-uniform
            uint4 v1[NU], v2[NU], v3[NU];
            load_rbatch_al<NU>(q, nbw, nbw > 1u ? 1u : 0u, gl, v1, jfix);
            load_rbatch_al<NU>(q, nbw, nbw > 2u ? 2u : 0u, gl, v2, jfix);
            load_rbatch_al<NU>(q, nbw, nbw > 3u ? 3u : 0u, gl, v3, jfix);
            tail = load_rtail<EX>(q, gl);
            tr = src.trailer(q, gl);
            auto fold_j = [&](uint4(&v)[NU], uint32_t jj) {
                if (jj <= jfix) fix_rbatch_al<NU>(q, nbw, jj, gl, v);
                if (jj + 1u == nbw) a3p = jj == 0 ? 0u : A[NU - 1];
                if (jj == 0)
                    fold_first<W4K, NU, W4OFF>(v, A, L, pad);
                else
                    fold_batch<false, W4K, NU, W4OFF>(v, A, L);
            };
            fold_j(slot0, 0);
            if (nbw > 1u) fold_j(v1, 1);
            if (nbw > 2u) fold_j(v2, 2);
            if (nbw > 3u) fold_j(v3, 3);
            uint32_t X = merge_al<NU>(A, a3p, L, q, gl, lane, rot);
            X = finish_raw(q, X, tail, gl, L);
            if (gl == 0) src.stage(P, wave, grp, q, X, tr);
            __builtin_amdgcn_wave_barrier();
            src.flush(P, wave, lane, K);
            return;
        }
    }

    auto step = [&](uint4(&cur)[NU], uint4(&nxt)[NU]) -> bool {
        const bool lastj = j + 1 == nbw;
        const bool more = rhon < nr;
        if (!lastj) {
            if constexpr (AL)
                load_rbatch_al<NU>(q, nbw, j + 1, gl, nxt, Src::kAlMid ? jfix : 0xffffffffu);
            else
                load_rbatch<G>(q, nbw, j + 1, gl, nxt);
        } else {
            tail = load_rtail<EX>(q, gl);  // consumed after this batch's fold
            tr = src.trailer(q, gl);
            if (EX || more) {  // (exact: past the list, qn is the clamped last entry)
                if constexpr (AL) {
                    nbwn = round_nbw_al<NU>(al_geo(qn));
                    load_rbatch_al<NU>(qn, nbwn, 0, gl, nxt);
                } else {
                    nbwn = round_nbw<G>(qn);
                    load_rbatch<G>(qn, nbwn, 0, gl, nxt);
                }
            }
        }
        if constexpr (Src::kCurWait) {
            // (exact loads only) every memory operation but this step's own
            // -- the batch after this one, and on the last step the tail and
            // trailer before it -- is done, so `cur` has landed: an explicit
            // wait the compiler's counters then trust, where its own merge
            // over the loop's paths waited for the new batch too
            // (one immediate for both paths: on the last step it also waits
            // for the tail, as the verify walk's own counts do)
            static_assert(Src::kExact != 0, "the explicit wait needs exact load counts");
            __builtin_amdgcn_s_waitcnt(vmcnt_only(NU));
        }
        if constexpr (AL) {
            if (j <= jfix) fix_rbatch_al<NU>(q, nbw, j, gl, cur);
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
        if (EX || rhon < nr) qn = src.load(P, rhon * K + grp);  // (src.load clamps)
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
    P.tmp = P0.tmp ? P0.tmp + start : nullptr;
    P.n = static_cast<uint64_t>(count) + pieces;
    P.nplain = count;
    return P;
}

// Next round of the workgroup's large-buffer share: a word of combine table
// k = 5 (Shift_512), which no group of the class kernel uses, since the LDS
// is full (image + output staging = 160 KiB).
constexpr uint32_t kPoolWord = (kComb + 5 * 4096) / 4;

}  // namespace lvk
