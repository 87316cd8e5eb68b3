// The offsets API (lv_crc32c_batch_device, lv_crc32c_batch_device_ws): the
// length sort (sort.hip), then ONE persistent class kernel over the sorted
// list -- small classes on a few waves per workgroup, the large ones and the
// pieces of split long buffers from a per-workgroup pool -- and the join of
// split long buffers (combine_long_kernel).  The walk: lvk/walk.h.
#include <hip/hip_runtime.h>

#include <mutex>

#include "lvh.h"
#include "lvk/walk.h"

namespace lvk {

// Waves per workgroup that walk the small classes (<= 2 KiB) before joining
// the large-buffer pool.  Measured on C2/C4: class 0 runs as fast on 4 waves
// per CU as on 16 (it is bound by per-buffer VALU work and random line
// reads, not latency), and classes 2+3 run FASTER on 12 waves than on 16.
constexpr uint32_t kSmallWaves = LVK_SMALL_WAVES;
constexpr uint32_t kSmallRounds = LVK_SMALL_ROUNDS;  // small-class rounds per wave

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
template <bool SEEDED>
__global__ __launch_bounds__(kThreads) void crc32c_classes_kernel(Params P, const uint4 *__restrict__ image,
                                                                  const uint32_t *ws) {
    // The class ranges [start k, count 4 + k): the sort's workspace header,
    // or -- a hinted uniform batch that no sort ran for (P.hident = its
    // class + 1) -- every buffer in that one class.  Read or computed where
    // used (an array of the eight selected values cost the kernel 24 VGPRs
    // of spills and C3 via offsets 0.75 -> 0.67).
    const uint32_t hc = P.hident;
    const bool hostid = hc != 0u;
    auto cls = [&](uint32_t k) -> uint32_t {
        if (!hostid) return ws[kWsCls + k];
        const uint32_t c = hc - 1u, nn = static_cast<uint32_t>(P.n);
        return k < 4u ? (k <= c ? 0u : nn) : (k - 4u == c ? nn : 0u);
    };
    const bool ident = hostid || ws[kWsIdent] != 0u;  // sort_scatter skipped a one-key batch
    stage_tables(image);
    if (threadIdx.x == 0) g_lds[kPoolWord] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const Lut L = make_lut(lane);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t grid = gridDim.x;
    const uint32_t n23 = cls(6) + cls(7);
    // pieces of split long buffers (walked after classes 2+3; a split buffer
    // is longer than 16 KiB, so class 2 or 3, and n23 > 0 whenever there are
    // pieces)
    const uint32_t np = P.part ? min(ws[kWsPieces], kPieceBudget) : 0u;
    // With no large buffers at all, every wave walks the small classes.
    // Otherwise (round 3) as few waves per workgroup as keep each one at <=
    // kSmallRounds rounds of the small classes (64 class-0 or 16 class-1
    // buffers a round), at most kSmallWaves: a small-class round is latency-
    // bound, a wave taken from the large pool costs bandwidth.  Measured
    // (profiles/r03/small_waves/): the 1 GiB WAL scan (12 rounds on one wave)
    // 61.0 -> 63.2 % with 1 wave instead of 4, C2 (24 rounds on 3) 73.8 ->
    // 74.2-75.4 %, C4 (23 on 4) best with 4 (-1.2 % with 2, -1.8 % with 1).
    // Round 4, with the CRCs stored by sorted position: kSmallRounds 52
    // (fewer small-class waves) over 26, C2 0.770 -> 0.773, C4 0.755 ->
    // 0.761, WAL unchanged; 13 and 104 lower (profiles/r04/small_rounds*/).
    uint32_t nsmall = n23 ? kSmallWaves : kWaves;
    if (n23) {
        const uint64_t rounds = (cls(4) + 63ull) / 64u + (cls(5) + 15ull) / 16u;
        const uint64_t per = static_cast<uint64_t>(kSmallRounds) * gridDim.x;
        const uint64_t ns = (rounds + per - 1) / per;
        nsmall = static_cast<uint32_t>(ns < 1 ? 1 : (ns > kSmallWaves ? kSmallWaves : ns));
    }
    if (wave < nsmall) {
        const uint64_t sw = blockIdx.x * nsmall + wave, nsw = grid * nsmall;
        uint64_t k = 0;
        auto stride = [&]() { return sw + (++k) * nsw; };
        if (cls(4)) {
            sorted_stream<1>(sub_list(P, cls(0), cls(4)), SortedList<SEEDED>{ident}, lane, L, sw, stride);
            k = 0;
        }
        if (cls(5)) sorted_stream<4>(sub_list(P, cls(1), cls(5)), SortedList<SEEDED>{ident}, lane, L, sw, stride);
    }
    if (n23) {
        // A list of mostly long-buffer pieces (>= 3/4 of the entries), with
        // >= 64 KiB per wave, is the blocks kernel's long-block regime: waves
        // that start together stream their pieces in lockstep, which reads
        // slower; stagger them as crc32c_blocks_kernel does (64 x 16 MiB:
        // 223 -> 201 us per call).
        const uint64_t bytes = hostid ? 0u : (static_cast<uint64_t>(ws[kWsBytes + 1]) << 32) | ws[kWsBytes];
        if (4ull * np >= 3ull * (n23 + np) && bytes >= (64ull << 10) * grid * kWaves)
            for (uint32_t k = 0; k < wave * LVK_STAGGER; ++k) __builtin_amdgcn_s_sleep(32);
        // Walk order of classes 2 + 3 (each sorted longest first): with both
        // present, the full rounds are rotated to start at class 3's first
        // round, so the pool ends on class 2's shortest buffers instead of a
        // round of 32-64 KiB buffers (the persistent grid's ragged end).  The
        // rotation is on the wave-uniform round index (scalar registers: an
        // entry remap in SortedList::load cost the class kernel 5 VGPRs of
        // spills and C3 via offsets 5 %).
        const uint64_t rrot = (cls(6) && cls(7)) ? n23 / 4u : 0u;  // K = 4 entries per round
        const uint64_t s3 = cls(6) / 4u;
        auto pool = [&]() -> uint64_t {
            uint32_t k = 0;
            if (lane == 0) k = atomicAdd(&g_lds[kPoolWord], 1u);
            uint64_t rho = blockIdx.x + grid * static_cast<uint64_t>(__shfl(k, 0));
            if (rho < rrot) {
                rho += s3;
                if (rho >= rrot) rho -= rrot;
            }
            return rho;
        };
        sorted_stream<16>(sub_list(P, cls(6) ? cls(2) : cls(3), n23, np), SortedList<SEEDED>{ident}, lane, L, pool(),
                          pool);
    }
}

// The hinted identity path's check (lv_crc32c_batch_device_hint, a uniform
// batch walked in index order with no sort): every length must be the
// hint's.  A launch of its own: the same check inside the class kernel, at
// its start or its end, moved the seeded walk's register allocation into
// spills with reloads in the round loops.
__global__ __launch_bounds__(256) void hint_len_kernel(const uint32_t *__restrict__ len, uint64_t n, uint32_t hlen,
                                                       uint32_t *__restrict__ err) {
    const uint64_t str = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    uint32_t bad = 0;
    uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    for (; i + 3 * str < n; i += 4 * str)  // four loads in flight per thread
        bad |= (len[i] ^ hlen) | (len[i + str] ^ hlen) | (len[i + 2 * str] ^ hlen) | (len[i + 3 * str] ^ hlen);
    for (; i < n; i += str) bad |= len[i] ^ hlen;
    if (bad) atomicOr(err, LV_HINT_ERR_NOT_UNIFORM);
}

// Joins the pieces of the offsets API's split long buffers (sort_scatter,
// split_wave): long record {buffer, first piece slot, m, p}, pieces of
// P = 2^p bytes aligned to the buffer end; piece 0's register is
// R_0 = R(~seed, piece 0) and piece k > 0 was walked as a seed-0 buffer,
// part = R(~0, piece k) = R(0, piece k) ^ Shift_P(~0) (the seed trick), so
// R_k = part ^ Shift_P(~0) and R(~seed, buffer) = XOR_k Shift_{(m-1-k) P}(R_k).
// Buffers of <= 64 pieces: one wave each, Horner within lanes and a tree
// across them, every shift a wave-uniform base matrix (round 2 before:
// per-lane shifts by the set bits of m - 1 - k, 9.9 us for 64 x 16 MiB).  A
// lane's run of c pieces is up to 8 independent Horner chains joined by an
// in-lane tree: each Horner step is a dependent L2 round trip (~0.18 us).
// Buffers of more pieces: one workgroup each (round 3), with every table it
// needs staged in LDS once -- a lone 16 MiB buffer (4,096 pieces) took 7.1 us
// on one wave, 8 + 3 + 6 dependent L2 steps.
constexpr uint32_t kWgJoinMin = 65;  // pieces: one workgroup per buffer from here on
__global__ __launch_bounds__(1024) void combine_long_kernel(const uint32_t *__restrict__ ws,
                                                           const uint4 *__restrict__ longs,
                                                           const uint32_t *__restrict__ part,
                                                           const uint32_t *__restrict__ tabs,
                                                           uint32_t *__restrict__ out, uint32_t flags,
                                                           const uint32_t *__restrict__ tmp,
                                                           const uint32_t *__restrict__ spos, uint64_t nb) {
    // Unsort (the sorted path): the class kernel stored each CRC at its
    // buffer's sorted position, in runs of consecutive words; out[i] =
    // tmp[spos[i]] writes whole lines in buffer order.  Split buffers
    // (spos = ~0u) are the join's below; a one-key batch (kWsIdent) was walked
    // in buffer order straight into out[].
    if (tmp && ws[kWsIdent] == 0u) {  // grid-uniform
        const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
        for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < nb; i += stride) {
            const uint32_t sp = spos[i];
            if (sp != 0xffffffffu) out[i] = tmp[sp];
        }
    }
    // the counter counts every claim; records exist only below the budget
    const uint32_t nl = longs ? min(ws[kWsLongs], kPieceBudget / 2) : 0u;
    if (blockIdx.x >= nl) return;  // block-uniform (every workgroup below nl has a wave or a record)
    // Shift_{2^i}(v) by four byte-table lookups (tables in HBM, L2-resident:
    // 192 KiB for every i) instead of a staged 32-column matrix product
    // (round 2: 1,024 x 64 KiB 36.8 -> 32.7 us, profiles/r02/long/ab_long_tables.txt)
    auto shift = [&](uint32_t i, uint32_t v) { return tab_shift(tabs + i * 1024u, v); };
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * (blockDim.x / 64);
    for (uint32_t w = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); w < nl; w += nw) {
        const uint4 r = longs[w];  // {buffer, first, m, p}
        const uint32_t m = r.z, p = r.w;
        // m = 0: a claim past the piece budget, the buffer was walked whole;
        // m >= kWgJoinMin: the workgroup loop below
        if (m == 0 || m >= kWgJoinMin) continue;
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
        for (uint32_t i = 1; i < d; ++i) {  // wave-uniform trip count
            uint32_t rk[8];
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q) rk[q] = piece(q, i);
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q) ch[q] = shift(p, ch[q]) ^ rk[q];
        }
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
    // Buffers of >= kWgJoinMin pieces, one workgroup each: the m pieces are
    // padded at the FRONT to 1024 c (c = the power of two >= m / 1024) and
    // staged in LDS; thread j runs Q = min(c, 4) Horner chains of d = c / Q
    // pieces with Shift_P and an in-thread tree, then a 6-level lane tree
    // with Shift_{c 2^t P} and a 4-level tree over the 16 wave partials with
    // Shift_{64 c 2^t P}.  Every shift is Shift_{2^v P} for v < lc + 10 <= 12
    // (c <= 4: m <= kMaxPieces = 4,096): the base tables p .. p + lc + 9,
    // staged in LDS with the pieces in one round trip.  (LDS kept small: a
    // version of this kernel at 153 KiB ran every launch several times
    // slower.)
    static_assert(kMaxPieces <= 4096, "join: c <= 4 pieces per thread");
    __shared__ uint32_t TW[12 * 1024];
    __shared__ uint32_t PW[4 * 1024 + 64];  // + one pad word per 64
    __shared__ uint32_t wpart[kWaves];
    const uint32_t t = threadIdx.x, wv = t >> 6, nt = blockDim.x;
    for (uint32_t ri = blockIdx.x; ri < nl; ri += gridDim.x) {  // block-uniform
        const uint4 r = longs[ri];
        const uint32_t m = r.z, p = r.w;
        if (m < kWgJoinMin) continue;
        uint32_t c = 1, lc = 0;
        while (nt * c < m) {
            c <<= 1;
            ++lc;
        }
        const uint32_t lq = lc < 2u ? lc : 2u, Q = 1u << lq, ld = lc - lq, d = 1u << ld;
        const uint32_t pad = nt * c - m;
        __syncthreads();  // the previous record's readers of TW / PW are done
        // One memory round trip: the pieces' loads, then the tables' (staged
        // in LDS), then the pieces' LDS stores; Shift_P(~0) from the staged
        // table afterwards (loading it first cost a round trip of its own).
        // Padded piece x at PW[x + x / 64], raw (the seed correction is
        // applied on reading): coalesced loads, conflict-free stores, and
        // thread t's run t c + i reads 64 distinct banks for any power of two
        // c <= 64.  (Named registers, not an array: arrays in these copy
        // loops were placed in LDS by the compiler.)
        auto ldp = [&](uint32_t x) {
            const bool on = x < nt * c && x >= pad;
            const uint32_t v = part[r.y + (on ? x - pad : 0u)];
            return on ? v : 0u;
        };
        auto st = [&](uint32_t x, uint32_t v) {
            if (x < nt * c) PW[x + (x >> 6)] = v;
        };
        if (c == 4u) {  // block-uniform: m > 2,048, four pieces per thread
            const uint32_t v0 = ldp(t), v1 = ldp(t + nt), v2 = ldp(t + 2u * nt), v3 = ldp(t + 3u * nt);
            stage_words(TW, tabs + p * 1024u, (lc + 10u) * 256u);
            st(t, v0);
            st(t + nt, v1);
            st(t + 2u * nt, v2);
            st(t + 3u * nt, v3);
        } else if (c == 2u) {
            const uint32_t v0 = ldp(t), v1 = ldp(t + nt);
            stage_words(TW, tabs + p * 1024u, (lc + 10u) * 256u);
            st(t, v0);
            st(t + nt, v1);
        } else {
            const uint32_t v0 = ldp(t);
            stage_words(TW, tabs + p * 1024u, (lc + 10u) * 256u);
            st(t, v0);
        }
        __syncthreads();
        const uint32_t corr = tab_shift(TW, 0xffffffffu);  // Shift_P(~0): pieces k > 0 started from ~0
        auto sh = [&](uint32_t v, uint32_t a) { return tab_shift(TW + v * 1024u, a); };
        auto pw = [&](uint32_t i) {  // thread t's padded piece t c + i (piece x - pad > 0: remove Shift_P(~0))
            const uint32_t x = t * c + i;
            return PW[x + (x >> 6)] ^ (x > pad ? corr : 0u);
        };
        uint32_t ch[4];
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) ch[q] = q < Q ? pw(q * d) : 0u;
        for (uint32_t i = 1; i < d; ++i) {  // block-uniform trip count
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q)
                if (q < Q) ch[q] = sh(0, ch[q]) ^ pw(q * d + i);
        }
#pragma unroll
        for (uint32_t u = 0; u < 2; ++u)  // chain q joins chain q + 2^u: Shift_{d 2^u P}
            if (u < lq) {
#pragma unroll
                for (uint32_t q = 0; q < 4; q += 2u << u) ch[q] = sh(ld + u, ch[q]) ^ ch[q + (1u << u)];
            }
        uint32_t acc = ch[0];
#pragma unroll
        for (uint32_t u = 0; u < 6; ++u) {  // lane l joins lane l + 2^u: Shift_{c 2^u P}
            const uint32_t right = __shfl_down(acc, 1u << u);
            const uint32_t shv = sh(lc + u, acc);
            if ((lane & ((2u << u) - 1u)) == 0) acc = shv ^ right;
        }
        if (lane == 0) wpart[wv] = acc;
        __syncthreads();
        if (wv == 0) {  // wave w holds the w-th sixteenth: a 4-level tree over lanes 0..15
            acc = lane < kWaves ? wpart[lane] : 0u;
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u) {
                const uint32_t right = __shfl_down(acc, 1u << u);
                const uint32_t shv = sh(lc + 6u + u, acc);
                if ((lane & ((2u << u) - 1u)) == 0) acc = shv ^ right;
            }
            if (lane == 0) {
                const uint32_t crc = ~acc;
                out[r.x] = (flags & LV_CRC_MASK) ? mask_crc(crc) : crc;
            }
        }
    }
}


// ---------------------------------------------------------------------------
// Small batches (n <= kFusedMax buffers) in ONE walk launch, no sort: every
// workgroup reads all n lengths (<= 4 KiB, L2-resident), so each knows the
// batch's payload bytes, every buffer's split (split_rule) and the exclusive
// prefix of the units -- a buffer is one unit, or its m pieces -- and walks
// its share of the units with the G = 16 aligned-row walk straight from that
// prefix.  Unit u belongs to the buffer i with pre(i) <= u < pre(i + 1) (a
// binary search in LDS); a piece parks its raw register in part[u] and
// workgroup 0 writes the long records for combine_long_kernel.  This replaces
// sort_small (one launch of ~8 us that every workgroup spent reading the
// lengths anyway) for the reference bench's few long buffers
// (benches/crc32c.rs:54-60: 1 MiB and 16 MiB) and any other small batch.
// The prefix lives in combine table 4's LDS (Shift_256), which a G = 16 walk
// never reads; the LDS is otherwise full (image + output staging).
constexpr uint32_t kFusedMax = 1024;                   // buffers: one per thread
// The sort's split (4 KiB pieces, <= kMaxPieces per buffer).  Measured with
// 1 KiB pieces (up to 16,384 per buffer, so that a lone 16 MiB buffer gives
// every G = 16 group of the grid a piece): the walk gained <= 1 us and the
// join of 16,384 pieces cost 9.2 us against ~5 for 4,096.
constexpr uint32_t kFusedPieceLog2 = 12;
constexpr uint32_t kFusedMaxPieces = kMaxPieces;
static_assert(kFusedMaxPieces / 2 >= 64, "a local split buffer (<= 64 pieces) must be split at the batch's 2^pb");
constexpr uint32_t kUnitPre = (kComb + 4 * 4096) / 4;  // LDS word: unit prefix | log2 piece << 24
constexpr uint32_t kFusedScratch = kPoolWord + 1;      // LDS words: per-wave payload sums, scan totals
static_assert(kFusedMax <= 1024 && kUnitPre + kFusedMax <= kPoolWord, "prefix fits combine table 4");

template <bool SEEDED>
struct FusedUnits {
    static constexpr uint32_t kFlush = 16;
    static constexpr bool kAlMid = true;
    static constexpr bool kOneRound = true;  // sorted_stream: a one-round wave loads all batches at once
    static constexpr bool kCurWait = false;
    static constexpr uint32_t kTrailerLoads = 0;
    // wait-count modes 1 / 2 (walk.h) measured 0.7-1.3 / 0.5-0.9 us slower on
    // the few-long-buffer calls (profiles/r04/new_ab/, mode2_ab/): masked
    static constexpr uint32_t kExact = 0;
    uint32_t nbuf;  // buffers (<= kFusedMax); P.n = units
    __device__ __forceinline__ RGeo load(const Params &P, uint64_t e) const {
        const bool valid = e < P.n;
        const uint32_t u = static_cast<uint32_t>(valid ? e : P.n - 1);
        uint32_t i = 0;  // the last buffer whose first unit is <= u
#pragma unroll
        for (uint32_t step = kFusedMax / 2; step >= 1; step >>= 1)
            if (i + step < nbuf && (g_lds[kUnitPre + i + step] & 0xffffffu) <= u) i += step;
        const uint32_t w = g_lds[kUnitPre + i];
        const uint32_t p = w >> 24, k = u - (w & 0xffffffu);
        const uint32_t Lb = P.len[i];
        const uint64_t a = P.base + P.off[i];
        const uint32_t sd = SEEDED ? P.seed[i] : 0u;
        RGeo q;
        q.aux = 0;
        if (p == 0) {  // a whole buffer
            q.a = Lb ? a : P.base;  // an empty buffer reads nothing of its own
            q.len = Lb;
            q.seed = sd;
            q.bid = valid ? i : 0xffffffffu;
        } else {  // piece k of P = 2^p bytes, aligned to the buffer's end (piece 0: the rest)
            const uint64_t PB = 1ull << p;
            const uint32_t m = static_cast<uint32_t>((Lb + PB - 1) >> p);
            const uint64_t first = Lb - (static_cast<uint64_t>(m) - 1) * PB;
            q.a = a + (k ? first + (k - 1) * PB : 0u);
            q.len = static_cast<uint32_t>(k ? PB : first);
            q.seed = k ? 0u : sd;  // pieces k > 0 are walked as seed-0 buffers (combine_long_kernel)
            q.bid = valid ? (u | kPieceFlag) : 0xffffffffu;
        }
        return q;
    }
    __device__ __forceinline__ uint2 trailer(const RGeo &, uint32_t) const { return make_uint2(0, 0); }
    __device__ __forceinline__ void stage(const Params &P, uint32_t wave, uint32_t slot, const RGeo &q, uint32_t X,
                                          uint2) const {
        g_oidx[wave][slot] = q.bid;
        g_ocrc[wave][slot] = q.bid != 0xffffffffu && (q.bid & kPieceFlag) ? X : final_crc(P, X);
    }
    __device__ __forceinline__ void flush(const Params &P, uint32_t wave, uint32_t lane, uint32_t nslots) const {
        const uint32_t bi = g_oidx[wave][lane], cv = g_ocrc[wave][lane];
        if (lane >= nslots || bi == 0xffffffffu) return;
        if (bi & kPieceFlag)
            P.part[bi & ~kPieceFlag] = cv;
        else
            P.out[bi] = cv;
    }
};

// Exclusive scan of v over the workgroup's 1024 threads (wave scans, then
// the earlier waves' totals); *total gets the sum.  `sc` is 16 LDS words.
__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t *sc, uint32_t *total) {
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint32_t inc = v;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t x = __shfl_up(inc, d);
        if (lane >= d) inc += x;
    }
    if (lane == 63) sc[w] = inc;
    __syncthreads();
    uint32_t before = 0, all = 0;
    for (uint32_t k = 0; k < kWaves; ++k) {
        const uint32_t t = sc[k];
        before += k < w ? t : 0u;
        all += t;
    }
    __syncthreads();  // sc is reused by the next scan
    *total = all;
    return before + inc - v;
}

template <bool SEEDED>
__global__ __launch_bounds__(kThreads) void crc32c_fused_small_kernel(Params P, const uint4 *__restrict__ image,
                                                                      uint32_t *__restrict__ ws,
                                                                      uint4 *__restrict__ longs) {
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint32_t nbuf = static_cast<uint32_t>(P.nplain);
    const uint32_t Lt = t < nbuf ? P.len[t] : 0u;  // requested before the staging: one round trip for both
    stage_tables(image);  // ends with a barrier: combine table 4 may be overwritten now
    uint64_t sum = Lt;
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) sum += __shfl_xor(sum, k);
    uint32_t *sc = g_lds + kFusedScratch;  // 2 x 16 words of payload sums, then 16 scan words
    if (lane == 0) {
        sc[2 * w] = static_cast<uint32_t>(sum);
        sc[2 * w + 1] = static_cast<uint32_t>(sum >> 32);
    }
    __syncthreads();
    uint64_t total = 0;
    for (uint32_t k = 0; k < kWaves; ++k) total += (static_cast<uint64_t>(sc[2 * k + 1]) << 32) | sc[2 * k];
    if (P.herr && blockIdx.x == 0) {
        // the host left out the join on the hint's word: check it against
        // the lengths (one workgroup reports)
        uint32_t bad = 0;
        if (t < nbuf) bad |= P.huni ? (Lt != P.hlen ? LV_HINT_ERR_NOT_UNIFORM : 0u) : (Lt > P.hlen ? LV_HINT_ERR_LONGER : 0u);
        if (t == 0 && total != P.htotal) bad |= LV_HINT_ERR_TOTAL;
        if (bad) atomicOr(P.herr, bad);
    }
    uint32_t p = 0;
    const uint32_t m = t < nbuf ? split_rule(Lt, total, &p, kFusedPieceLog2, kFusedMaxPieces) : 0u;
    const uint32_t units = t < nbuf ? (m ? m : 1u) : 0u;
    uint32_t nunits = 0, nlong = 0;
    const uint32_t pre = block_exscan(units, sc + 32, &nunits);
    nunits = __builtin_amdgcn_readfirstlane(nunits);  // block-uniform (scalar registers)
    const uint64_t grid = gridDim.x;
    // One pass (every wave <= 1 round): workgroup b walks the contiguous units
    // [b S, (b + 1) S), S = whole rounds, as many rounds per workgroup as the
    // round-robin pool gave it; a split buffer whose pieces all fall in one
    // workgroup's units is joined there, after the walk (no long record).
    const bool onepass = nunits <= 4ull * kWaves * grid;
    const uint32_t S = onepass ? 4u * static_cast<uint32_t>((nunits + 4ull * grid - 1) / (4ull * grid)) : 1u;
    uint32_t pb = ceil_log2(total / 16384u);  // the batch's piece length (split_rule), for the join
    pb = pb > kFusedPieceLog2 ? pb : kFusedPieceLog2;
    pb = __builtin_amdgcn_readfirstlane(pb < 31u ? pb : 31u);
    // The in-workgroup join stages only Shift_{2^v 2^pb}, v < 6: a buffer is
    // local only if it was split at the batch's piece length 2^pb (split_rule's
    // L / kMaxPieces term gives a larger one only to buffers of > kMaxPieces / 2
    // pieces, which never fit one workgroup's <= 64 units; checked, not assumed).
    const bool local = onepass && m && p == pb && pre / S == (pre + m - 1u) / S;
    const uint32_t lpre = block_exscan(m && !local ? 1u : 0u, sc + 32, &nlong);
    if (t < nbuf) g_lds[kUnitPre + t] = pre | (p << 24);
    if (blockIdx.x == 0) {
        if (m && !local) longs[lpre] = make_uint4(t, pre, m, p);
        if (t == 0) {
            ws[kWsLongs] = nlong;
            ws[kWsPieces] = nunits;
        }
    }
    uint32_t *const lflag = g_lds + kFusedScratch + 48;  // a local buffer in the batch / in this workgroup
    const uint32_t b0 = static_cast<uint32_t>(blockIdx.x) * S;
    if (t == 0) {
        g_lds[kPoolWord] = 0;
        lflag[0] = 0;
        lflag[1] = 0;
    }
    __syncthreads();
    if (local) lflag[0] = 1u;
    if (local && pre >= b0 && pre < b0 + S) lflag[1] = 1u;
    __syncthreads();
    const Lut L = make_lut(lane);
    Params Q = P;
    Q.n = nunits;
    // Without a local buffer, the round-robin pool (every workgroup busy);
    // with one, workgroup b's static rounds.  (One instantiation of the walk
    // for both: two spilled 33 VGPRs.)
    const bool lmode = __builtin_amdgcn_readfirstlane(lflag[0]) != 0u;
    constexpr uint64_t kNone = ~0ull >> 2;  // a round index past any list
    const uint32_t rw = S / 4u;             // local mode: rounds of this workgroup
    auto next = [&]() -> uint64_t {
        if (lmode) return kNone;
        uint32_t k = 0;
        if (lane == 0) k = atomicAdd(&g_lds[kPoolWord], 1u);
        return blockIdx.x + grid * static_cast<uint64_t>(__shfl(k, 0));
    };
    const uint64_t rho0 = lmode ? (w < rw ? blockIdx.x * static_cast<uint64_t>(rw) + w : kNone) : next();
    sorted_stream<16, FusedUnits<SEEDED>>(Q, FusedUnits<SEEDED>{nbuf}, lane, L, rho0, next);
    if (!lmode) return;
    // ---- the in-workgroup join of this workgroup's local split buffers ----
    __syncthreads();  // the walk is done: its piece registers are in g_ocrc
    if (lflag[1] == 0) return;  // block-uniform
    // Local buffers have m <= S <= 64 pieces, so their piece length is the
    // batch's, 2^pb (a larger one comes from L > 4,096 x 2^pb, m > 2,048):
    // stage Shift_{2^v P}, v < 6, over the image's region A (no longer read).
    const uint32_t n4 = nunits;
    stage_words(g_lds, P.tabs + pb * 1024u, 6u * 256u);
    __syncthreads();
    if (w != 0 || lane >= S) return;
    // lane l: unit b0 + l (walked by wave l / 4 as group l % 4 of its one round)
    const uint32_t u = b0 + lane;
    if (u >= n4) return;
    uint32_t i = 0;  // the last buffer whose first unit is <= u
#pragma unroll
    for (uint32_t step = kFusedMax / 2; step >= 1; step >>= 1)
        if (i + step < nbuf && (g_lds[kUnitPre + i + step] & 0xffffffu) <= u) i += step;
    const uint32_t wi = g_lds[kUnitPre + i];
    const uint32_t pi = wi & 0xffffffu;
    const uint32_t mi = (i + 1 < nbuf ? g_lds[kUnitPre + i + 1] & 0xffffffu : n4) - pi;
    const bool mine = (wi >> 24) != 0 && pi / S == (pi + mi - 1u) / S;  // a local split buffer
    const uint32_t k = u - pi;
    // R_k (piece k > 0 was walked from ~0: remove Shift_P(~0)), shifted by
    // (m - 1 - k) P bit by bit, then a segmented xor over the buffer's lanes
    uint32_t R = g_ocrc[lane >> 2][lane & 3u] ^ (k ? tab_shift(g_lds, 0xffffffffu) : 0u);
    const uint32_t j = mi - 1u - k;
#pragma unroll
    for (uint32_t v = 0; v < 6; ++v) {
        const uint32_t sh = tab_shift(g_lds + v * 1024u, R);
        R = (j >> v) & 1u ? sh : R;
    }
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_down(R, d);
        if (k % (2u * d) == 0 && k + d < mi) R ^= o;
    }
    if (mine && k == 0) {
        const uint32_t crc = ~R;
        P.out[i] = (P.flags & LV_CRC_MASK) ? mask_crc(crc) : crc;
    }
}

}  // namespace lvk

namespace lvh {

void launch_classes(const DevCtx &c, bool seeded, const lvk::Params &P, const uint32_t *ws, hipStream_t s) {
    if (seeded)
        hipLaunchKernelGGL(lvk::crc32c_classes_kernel<true>, dim3(static_cast<uint32_t>(c.cus)), dim3(lvk::kThreads), 0,
                           s, P, c.image[kAlImage], ws);
    else
        hipLaunchKernelGGL(lvk::crc32c_classes_kernel<false>, dim3(static_cast<uint32_t>(c.cus)), dim3(lvk::kThreads),
                           0, s, P, c.image[kAlImage], ws);
}

// ---- the batch hint (lv_crc32c_batch_device_hint) ----
// Host replica of lvk::split_rule (lvk/sort.h) for the offsets API's split,
// pmin = 12 (4 KiB) and maxp = kMaxPieces in both the sort and the fused
// small-batch path.  Whether a buffer splits is monotone in its length L:
// with q_b = max(ceil_log2(total / 16,384), 12), L splits iff L > 16 KiB and
// L > 2^(q_b + 1) (the L / kMaxPieces term only raises q where L / 2^q is
// far above 2).
static uint32_t host_ceil_log2(uint64_t x) { return x <= 1 ? 0u : 64u - static_cast<uint32_t>(__builtin_clzll(x - 1)); }

static uint32_t host_split_rule(uint32_t L, uint64_t total, uint32_t *p) {
    *p = 0;
    if (L <= 16384u) return 0u;
    uint32_t q = host_ceil_log2(total / 16384u);
    const uint32_t pl = host_ceil_log2((static_cast<uint64_t>(L) + lvk::kMaxPieces - 1) / lvk::kMaxPieces);
    q = std::max(q, pl);
    q = std::max(q, 12u);
    q = std::min(q, 31u);
    if (L <= (2ull << q)) return 0u;
    *p = q;
    return static_cast<uint32_t>((L + (1ull << q) - 1) >> q);
}

// Does the batch need combine_long_kernel?  No when no buffer of at most
// max_len bytes can split in a batch of `total` bytes; for a uniform batch of
// <= kFusedMax buffers also when every split buffer's pieces fall in one
// workgroup's static rounds of the fused kernel, which joins those itself
// (the same unit layout crc32c_fused_small_kernel computes on the device).
bool hint_needs_join(const lv_batch_hint &h, uint64_t n, uint32_t cus) {
    if ((h.uniform & LV_HINT_ALIGNED16) && h.max_len) {
        // (an aligned arena) the strided API's kernels: a join launch
        // (combine_pieces_*) only for a split whose pieces do not join in the walk
        const UniformPlan pl = uniform_plan(static_cast<int>(cus), 0, 0, h.max_len, n, -1);
        if (pl.applies()) return pl.scratch != 0;
    }
    uint32_t p = 0;
    const bool nosplit = host_split_rule(h.max_len, h.total_bytes, &p) == 0;  // monotone: nothing splits
    // > kFusedMax buffers: the sorted path's join launch also unsorts the
    // CRCs; only a uniform batch with nothing to split (the identity list,
    // no sort) goes without it
    if (n > lvk::kFusedMax) return !(h.uniform && nosplit);
    if (nosplit) return false;
    if (!h.uniform) return true;
    const uint32_t m = host_split_rule(h.max_len, h.total_bytes, &p);
    const uint64_t nunits = n * m;
    const uint64_t grid = cus;
    if (nunits > 4ull * lvk::kWaves * grid) return true;  // not one pass: the pool, no local joins
    const uint64_t S = 4ull * ((nunits + 4ull * grid - 1) / (4ull * grid));
    uint32_t pb = host_ceil_log2(h.total_bytes / 16384u);
    pb = std::min(std::max(pb, lvk::kFusedPieceLog2), 31u);
    if (p != pb) return true;
    for (uint64_t t = 0; t < n; ++t)
        if ((t * m) / S != (t * m + m - 1) / S) return true;  // straddles two workgroups
    return false;
}

// Length-sorted launch of the offsets API, no host sync: the sort (one or
// three launches), the persistent class kernel, the long-buffer join.
int launch_binned(DevCtx &c, uint8_t *ws_bytes, const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                  const uint32_t *seed, uint32_t *out, uint64_t n, uint32_t flags, hipStream_t s, bool join,
                  const HintCheck *hc) {
    uint32_t *ws = reinterpret_cast<uint32_t *>(ws_bytes);
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
    P.nplain = n;
    uint4 *longs = nullptr;
    if (n <= lvk::kFusedMax) {
        // small batch: the split and the walk in one launch (no sort), then the join
        const WsLayout lay = ws_layout(n);
        longs = reinterpret_cast<uint4 *>(ws_bytes + lay.longs);
        P.part = reinterpret_cast<uint32_t *>(ws_bytes + lay.part);
        P.tabs = c.base_tabs;
        // the hint decided whether the join runs: the kernel checks its facts
        // against the lengths it reads (the sorted path below always joins,
        // so no fact of the hint changes what it computes)
        set_hint(P, hc, 0);
        g_kernel = join ? "crc32c_fused_small_kernel+combine_long_kernel" : "crc32c_fused_small_kernel";
        if (seed)
            hipLaunchKernelGGL(lvk::crc32c_fused_small_kernel<true>, dim3(static_cast<uint32_t>(c.cus)),
                               dim3(lvk::kThreads), 0, s, P, c.image[kAlImage], ws, longs);
        else
            hipLaunchKernelGGL(lvk::crc32c_fused_small_kernel<false>, dim3(static_cast<uint32_t>(c.cus)),
                               dim3(lvk::kThreads), 0, s, P, c.image[kAlImage], ws, longs);
    } else {
        // sorted path: the join launch also unsorts the class kernel's CRCs
        // (combine_long_kernel), so it always runs
        longs = launch_sort(ws_bytes, off, len, seed, n, s, &P);
        g_kernel = "sort+crc32c_classes_kernel+combine_long_kernel";
        launch_classes(c, seed != nullptr, P, ws, s);
        hipLaunchKernelGGL(lvk::combine_long_kernel, dim3(static_cast<uint32_t>(c.cus)), dim3(1024), 0, s, ws, longs,
                           P.part, c.base_tabs, out, flags, P.tmp,
                           reinterpret_cast<const uint32_t *>(ws_bytes + ws_layout(n).pos), n);
        return 0;
    }
    // joins split long buffers (exits at once when the sort split none).  (A
    // last-finisher join inside the class kernel -- agent-scope release and
    // acquire around a per-buffer counter -- measured 64 x 16 MiB 200 -> 345
    // us and 1,024 x 64 KiB 41 -> 177 us: every fence writes back or
    // invalidates the XCD's whole L2; and C3 via offsets -2 % from spills.)
    // (An empty launch -- C2 / C4, or a batch whose split buffers were all
    // joined in the fused kernel -- takes 4-5 us in the trace, with 64
    // workgroups as with one per CU: profiles/r03/fused_small/local_join/.)
    // (A grid of min(buffers, CUs) workgroups instead measured the same on
    // 1 x 16 MiB, 16 x 1 MiB and 64 x 16 MiB: profiles/r04/join_grid/.)
    if (longs && join)
        hipLaunchKernelGGL(lvk::combine_long_kernel, dim3(static_cast<uint32_t>(c.cus)), dim3(1024), 0, s, ws, longs,
                           P.part, c.base_tabs, out, flags, nullptr, nullptr, 0);
    return 0;
}


}  // namespace lvh

using namespace lvh;

extern "C" {

static int batch_device_impl(const uint8_t *d_arena, const uint64_t *d_off, const uint32_t *d_len,
                             const uint32_t *d_seed, uint32_t *d_out, size_t n, uint32_t flags,
                             void *stream, uint8_t *d_ws, size_t ws_bytes, const lv_batch_hint *hint = nullptr) {
    g_err.clear();
    if (n == 0) return LV_OK;
    if (!d_arena || !d_off || !d_len || !d_out) return set_err(LV_ERR_INVALID, "null device pointer");
    if (n > 0xffffffffull) return set_err(LV_ERR_INVALID, "more than 2^32-1 buffers per call");
    DevCtx *c = nullptr;
    if (int rc = current_ctx(&c)) return rc;
    const int gi = forced_gi(flags);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (gi >= 0) {
        launch_group(*c, false, gi, d_arena, d_off, d_len, 0, 0, d_seed, d_out, n, flags, s);
        return check_launch();
    }
    std::unique_lock<std::mutex> ws_lk;  // held through the last launch (library workspace)
    if (d_ws) {
        if (ws_bytes < sort_ws_bytes(n)) return set_err(LV_ERR_INVALID, "workspace too small");
        if (reinterpret_cast<uintptr_t>(d_ws) % 16) return set_err(LV_ERR_INVALID, "workspace must be 16-byte aligned");
        // no initialisation: every workspace word the sort reads, it wrote first
    }
    // the hint's facts travel to the kernels that read what they describe
    HintCheck hcv{nullptr, 0, 0, 0};
    const HintCheck *hc = nullptr;
    if (hint) {
        if (int rc = stream_err(*c, s, &hcv.err)) return rc;
        hcv.total = hint->total_bytes;
        hcv.len = hint->max_len;
        hcv.uniform = hint->uniform;
        hc = &hcv;
    }
    if (hint && (hint->uniform & LV_HINT_ALIGNED16) && hint->max_len &&
        reinterpret_cast<uintptr_t>(d_arena) % 16 == 0) {
        // aligned uniform buffers: the strided API's kernels with each start
        // read from d_off (no sort, no class kernel, no unsort)
        const UniformPlan pl = uniform_plan(c->cus, 0, 0, hint->max_len, n, -1);
        if (pl.applies() && (!d_ws || ws_bytes >= pl.scratch)) {
            uint8_t *scr = d_ws;
            if (pl.scratch && !scr)
                if (int rc = stream_ws_bytes(*c, s, pl.scratch, &scr, &ws_lk)) return rc;
            if (int rc = launch_uniform(*c, pl, d_arena, 0, d_off, d_len, hc, hint->max_len, n, d_seed, d_out, flags,
                                        s, scr))
                return rc;
            return check_launch();
        }
    }
    // Past this point the aligned path did not run (a misaligned arena, a
    // length that is not whole batches, a short caller workspace): the join
    // decision below must not assume it did.
    lv_batch_hint h2{};
    if (hint) {
        h2 = *hint;
        h2.uniform &= ~LV_HINT_ALIGNED16;
        hint = &h2;
    }
    if (!d_ws)
        if (int rc = stream_ws(*c, s, n, &d_ws, &ws_lk)) return rc;
    if (hint && hint->uniform && n > lvk::kFusedMax) {
        uint32_t p = 0;
        if (host_split_rule(hint->max_len, hint->total_bytes, &p) == 0) {
            // one sort key in index order and nothing to split: the class
            // kernel alone, its class ranges from the host (no sort, no join)
            lvk::Params P{};
            P.base = reinterpret_cast<uint64_t>(d_arena);
            P.off = d_off;
            P.len = d_len;
            P.seed = d_seed;
            P.out = d_out;
            P.n = n;
            P.nplain = n;
            P.flags = flags;
            const uint32_t L = hint->max_len;
            P.hident = 1u + (L <= 256u ? 0u : L <= 2048u ? 1u : L <= 32768u ? 2u : 3u);  // 1 + lvk::len_class(L)
            g_kernel = "hint_len_kernel+crc32c_classes_kernel";
            const uint64_t lg = std::min<uint64_t>(4ull * static_cast<uint64_t>(c->cus), (n + 1023) / 1024);
            hipLaunchKernelGGL(lvk::hint_len_kernel, dim3(static_cast<uint32_t>(lg)), dim3(256), 0, s, d_len,
                               static_cast<uint64_t>(n), L, hcv.err);
            launch_classes(*c, d_seed != nullptr, P, reinterpret_cast<const uint32_t *>(d_ws), s);
            return check_launch();
        }
    }
    const bool join = hint ? hint_needs_join(*hint, n, static_cast<uint32_t>(c->cus)) : true;
    if (int rc = launch_binned(*c, d_ws, d_arena, d_off, d_len, d_seed, d_out, n, flags, s, join, hc)) return rc;
    return check_launch();
}

int lv_crc32c_batch_device(const uint8_t *d_arena, const uint64_t *d_off, const uint32_t *d_len,
                           const uint32_t *d_seed, uint32_t *d_out, size_t n, uint32_t flags,
                           void *stream) {
    return batch_device_impl(d_arena, d_off, d_len, d_seed, d_out, n, flags, stream, nullptr, 0);
}

size_t lv_crc32c_workspace_bytes(size_t n) { return sort_ws_bytes(n); }

int lv_crc32c_hint_needs_join(const lv_batch_hint *hint, size_t n, uint32_t cus) {
    if (!hint) return 1;
    return hint_needs_join(*hint, n, cus) ? 1 : 0;
}

int lv_crc32c_batch_device_hint(const uint8_t *d_arena, const uint64_t *d_off, const uint32_t *d_len,
                                const uint32_t *d_seed, uint32_t *d_out, size_t n, uint32_t flags,
                                const lv_batch_hint *hint, void *d_workspace, size_t workspace_bytes, void *stream) {
    if (hint) {
        if (hint->uniform != 0 && hint->uniform != LV_HINT_UNIFORM &&
            hint->uniform != (LV_HINT_UNIFORM | LV_HINT_ALIGNED16))
            return set_err(LV_ERR_INVALID, "hint: uniform must be 0, LV_HINT_UNIFORM or LV_HINT_UNIFORM | LV_HINT_ALIGNED16");
        if (hint->uniform && hint->total_bytes != static_cast<uint64_t>(n) * hint->max_len)
            return set_err(LV_ERR_INVALID, "uniform hint: total_bytes != n * max_len");
        if (n && hint->max_len == 0 && hint->total_bytes != 0)
            return set_err(LV_ERR_INVALID, "hint: max_len 0 with nonzero total_bytes");
    }
    return batch_device_impl(d_arena, d_off, d_len, d_seed, d_out, n, flags, stream,
                             static_cast<uint8_t *>(d_workspace), d_workspace ? workspace_bytes : 0, hint);
}

int lv_crc32c_batch_device_ws(const uint8_t *d_arena, const uint64_t *d_off, const uint32_t *d_len,
                              const uint32_t *d_seed, uint32_t *d_out, size_t n, uint32_t flags,
                              void *d_workspace, size_t workspace_bytes, void *stream) {
    if (!d_workspace) return set_err(LV_ERR_INVALID, "null workspace");
    return batch_device_impl(d_arena, d_off, d_len, d_seed, d_out, n, flags, stream,
                             static_cast<uint8_t *>(d_workspace), workspace_bytes);
}

}  // extern "C"
