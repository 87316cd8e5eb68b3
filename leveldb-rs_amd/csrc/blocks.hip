// Strided batch API (lv_crc32c_batch_strided: fixed-size table blocks) and
// the group-size kernels behind the LV_CRC_GROUP override: the uniform-block
// kernel crc32c_blocks_kernel (wave-uniform batch control, no head/tail work),
// its long-block split with the fused or separate piece join
// (combine_pieces_kernel, combine_pieces_wg_kernel), and the per-group
// stream kernel crc32c_batch_kernel.  Algebra and table layout: lvk/core.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "lvh.h"

namespace lvk {

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
// GATHER: the offsets API with an aligned uniform hint (lv_batch_hint,
// LV_HINT_ALIGNED16) -- block k starts at base + off[k] instead of base +
// k * stride, every start 16-B aligned and every block blen bytes, so the
// walk is the strided one.  A wave needs the next round's offset when it
// leaves a block; it loads the offset of the block after that at every step
// (as it does the seed), so no batch load waits on an offset load.  The
// block's length is loaded beside its offset; where the offset is consumed
// both are checked against the hint (a misaligned offset or a length other
// than the hint's max_len is recorded in P.herr, lv_crc32c_batch_check), and
// the address uses the offset rounded down to 16 B, so a lying hint costs
// wrong CRCs it reports, never an unaligned or wider read.
template <int G, bool SEEDED, bool PIECES = false, bool FUSE = false, bool GATHER = false>
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
    // the start of block k's block (of piece k's block) relative to base
    auto block_off = [&](uint64_t k) -> uint64_t {
        const uint64_t kk = k < P.n ? k : 0;
        const uint64_t b = PIECES ? kk >> P.pshift : kk;
        if constexpr (GATHER) return P.off[b];
        return b * P.stride;
    };
    auto report = [&](uint32_t bad) {
        if constexpr (GATHER)
            if (bad && P.herr) atomicOr(P.herr, bad);
    };
    auto block_at = [&](uint64_t k, uint64_t bo) {
        const uint64_t kk = k < P.n ? k : 0;
        if constexpr (GATHER) bo &= ~static_cast<uint64_t>(15);
        if constexpr (PIECES) return P.base + bo + (kk & pmask) * P.plen + 16u * gl;
        return P.base + bo + 16u * gl;
    };
    auto block_ptr = [&](uint64_t k) { return block_at(k, block_off(k)); };
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
    const uint64_t o0 = block_off(blk);                    // this round's block offset
    uint64_t ptr = block_at(blk, o0);
    uint64_t o1 = GATHER ? block_off(blk + gstride) : 0;  // GATHER: the next round's block offset
    uint64_t o2 = o1;                                      // ... and the one after it, in flight
    uint32_t s0 = kVarS0 ? seed_ld(blk) : 0xffffffffu;
    uint32_t s0n = s0;
    uint4 slot0[U], slot1[U];
#pragma unroll
    for (uint32_t i = 0; i < U; ++i) slot0[i] = load16(ptr + kRow * i);
    // GATHER with a hint to check: every length, a grid-strided share per
    // thread (the walk itself never reads one).  The first four are requested
    // here and arrive under the table staging's round trip; more (> 4 x 1,024
    // blocks per workgroup) after it.
    const uint64_t nblk = PIECES ? (P.n >> P.pshift) : P.n;
    const uint64_t lstr = static_cast<uint64_t>(gridDim.x) * kThreads;
    const uint64_t lb0 = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x;
    uint32_t lq[4] = {0, 0, 0, 0};
    const bool lcheck = GATHER && P.herr;
    if (lcheck) {
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
            const uint64_t b = lb0 + i * lstr;
            lq[i] = b < nblk ? P.len[b] ^ P.hlen : 0u;
        }
    }
    uint32_t *const fm = &g_oidx[0][0];  // FUSE: matrix j at word 33 j (distinct banks per lane)
    if constexpr (FUSE) {
        const uint32_t nw = (1u << P.pshift) * 32u;
        for (uint32_t i = threadIdx.x; i < nw; i += kThreads) fm[(i >> 5) * 33 + (i & 31u)] = P.mats[i];
    }
    stage_tables(image);
    uint32_t lbad = lq[0] | lq[1] | lq[2] | lq[3];
    if (lcheck)
        for (uint64_t b = lb0 + 4 * lstr; b < nblk; b += lstr) lbad |= P.len[b] ^ P.hlen;
    // GATHER: the first block's offset and this thread's share of the lengths
    // (later offsets are checked as the walk consumes them)
    if constexpr (GATHER) report(((o0 & 15u) ? LV_HINT_ERR_MISALIGNED : 0u) | (lbad ? LV_HINT_ERR_NOT_UNIFORM : 0u));
    if (wblk0 >= P.n) {
        if constexpr (FUSE) fuse_pieces(P, fm, g_ocrc, lane, wave);  // the barrier is workgroup-wide
        return;
    }
    if constexpr (PIECES) {
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
        if constexpr (GATHER) o2 = block_off(blk + 2 * gstride);
        const uint64_t nptr = lastj ? (GATHER ? block_at(blk + gstride, o1) : block_ptr(blk + gstride)) : ptr + kBatch;
        // no next batch: a dummy read of the arena's first row, the same lines
        // for every wave (L2 hits); GATHER rereads this batch (the caller's
        // arena pointer need not be readable)
        const uint64_t lptr = more ? nptr : GATHER ? ptr : P.base + 16u * gl;
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
            if constexpr (GATHER) {
                if (o1 & 15u) report(LV_HINT_ERR_MISALIGNED);  // the block walked next (o1 was consumed above)
                o1 = o2;
            }
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

// Joins the raw piece registers of the long-block split: block b's pieces
// R_k = raw[b*s + k], k < s (s a power of two <= 4,096), give
//   R(~seed, block) = XOR_k Shift_{(s-1-k) plen}(R_k)
// (linearity, DESIGN "CRC algebra").
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

}  // namespace lvk

namespace lvh {

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

void launch_group(const DevCtx &c, bool strided, int gi, const uint8_t *arena, const uint64_t *off,
                  const uint32_t *len, uint64_t stride, uint32_t blen, const uint32_t *seed, uint32_t *out, uint64_t n,
                  uint32_t flags, hipStream_t s) {
    if (strided)
        launch_g<true>(c, gi, arena, off, len, stride, blen, seed, out, n, flags, s);
    else
        launch_g<false>(c, gi, arena, off, len, stride, blen, seed, out, n, flags, s);
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

template <int G, bool GATHER>
void launch_blocks_g(const DevCtx &c, int gi, const uint8_t *base, uint64_t stride, const uint64_t *off,
                     const uint32_t *len, const HintCheck *hc, uint32_t blen, uint64_t n, const uint32_t *seed,
                     uint32_t *out, uint32_t flags, hipStream_t s) {
    const uint64_t groups_per_wg = static_cast<uint64_t>(lvk::kWaves) * (64 / G);
    uint64_t grid = (n + groups_per_wg - 1) / groups_per_wg;
    if (grid > static_cast<uint64_t>(c.cus)) grid = c.cus;
    if (grid == 0) grid = 1;
    lvk::Params P{};
    P.base = reinterpret_cast<uint64_t>(base);
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
    set_hint(P, hc, blen);
    const uint32_t nb = static_cast<uint32_t>(blen / (16ull * G * lvk::U));
    static const std::string name = "crc32c_blocks_kernel<" + std::to_string(G) + (GATHER ? ",gather>" : ">");
    g_kernel = name.c_str();
    if (seed)
        hipLaunchKernelGGL((lvk::crc32c_blocks_kernel<G, true, false, false, GATHER>),
                           dim3(static_cast<uint32_t>(grid)), dim3(lvk::kThreads), 0, s, P, nb, c.image[gi]);
    else
        hipLaunchKernelGGL((lvk::crc32c_blocks_kernel<G, false, false, false, GATHER>),
                           dim3(static_cast<uint32_t>(grid)), dim3(lvk::kThreads), 0, s, P, nb, c.image[gi]);
}

template <bool GATHER>
void launch_blocks(const DevCtx &c, int gi, const uint8_t *base, uint64_t stride, const uint64_t *off,
                   const uint32_t *len, const HintCheck *hc, uint32_t blen, uint64_t n, const uint32_t *seed,
                   uint32_t *out, uint32_t flags, hipStream_t s) {
    switch (gi) {
        case 0: launch_blocks_g<1, GATHER>(c, gi, base, stride, off, len, hc, blen, n, seed, out, flags, s); break;
        case 1: launch_blocks_g<4, GATHER>(c, gi, base, stride, off, len, hc, blen, n, seed, out, flags, s); break;
        case 2: launch_blocks_g<16, GATHER>(c, gi, base, stride, off, len, hc, blen, n, seed, out, flags, s); break;
        default: launch_blocks_g<64, GATHER>(c, gi, base, stride, off, len, hc, blen, n, seed, out, flags, s); break;
    }
}

// The long-block split: the piece walk (the fused join when the pieces fill
// one round of <= kFuseMax per block) and, unfused, the join launch.
template <bool GATHER>
void launch_pieces(DevCtx &c, uint32_t ps, const uint32_t *mats, const uint32_t *tabs, const uint8_t *base,
                   uint64_t stride, const uint64_t *off, const uint32_t *len, const HintCheck *hc, uint32_t blen,
                   uint64_t n, const uint32_t *seed, uint32_t *out, uint32_t flags, hipStream_t hs, uint32_t *scr) {
    const uint64_t nv = n << ps, plen = blen >> ps;
    const uint32_t nb = static_cast<uint32_t>(plen / (16ull * 16 * lvk::U));
    lvk::Params P{};
    P.base = reinterpret_cast<uint64_t>(base);
    P.off = off;
    P.len = len;
    P.seed = seed;
    P.n = nv;
    P.stride = stride;
    P.blen = static_cast<uint32_t>(plen);
    P.flags = flags;
    P.plen = plen;
    P.pshift = ps;
    P.mats = mats;
    set_hint(P, hc, blen);
    if (!scr) {  // one round of the grid: each workgroup joins its own blocks' pieces
        P.out = out;
        const dim3 grid(static_cast<uint32_t>((nv + 63) / 64));
        if (seed)
            hipLaunchKernelGGL((lvk::crc32c_blocks_kernel<16, true, true, true, GATHER>), grid, dim3(lvk::kThreads), 0,
                               hs, P, nb, c.image[2]);
        else
            hipLaunchKernelGGL((lvk::crc32c_blocks_kernel<16, false, true, true, GATHER>), grid, dim3(lvk::kThreads),
                               0, hs, P, nb, c.image[2]);
        g_kernel = GATHER ? "crc32c_blocks_kernel<16,pieces,fused,gather>" : "crc32c_blocks_kernel<16,pieces,fused>";
        return;
    }
    P.out = scr;
    const uint64_t grid = std::min<uint64_t>(c.cus, (nv + 63) / 64);
    if (seed)
        hipLaunchKernelGGL((lvk::crc32c_blocks_kernel<16, true, true, false, GATHER>), dim3(static_cast<uint32_t>(grid)),
                           dim3(lvk::kThreads), 0, hs, P, nb, c.image[2]);
    else
        hipLaunchKernelGGL((lvk::crc32c_blocks_kernel<16, false, true, false, GATHER>),
                           dim3(static_cast<uint32_t>(grid)), dim3(lvk::kThreads), 0, hs, P, nb, c.image[2]);
    if (ps >= 11) {  // > 1,024 pieces per block: a workgroup per block
        hipLaunchKernelGGL(lvk::combine_pieces_wg_kernel, dim3(static_cast<uint32_t>(n)), dim3(1024), 0, hs, P.out,
                           1u << ps, tabs, out, flags);
        g_kernel = GATHER ? "crc32c_blocks_kernel<16,pieces,gather>+combine_pieces_wg_kernel"
                          : "crc32c_blocks_kernel<16,pieces>+combine_pieces_wg_kernel";
    } else {
        hipLaunchKernelGGL(lvk::combine_pieces_kernel, dim3(static_cast<uint32_t>(std::min<uint64_t>(1024, (n + 3) / 4))),
                           dim3(256), 0, hs, P.out, n, 1u << ps, mats, out, flags);
        g_kernel = GATHER ? "crc32c_blocks_kernel<16,pieces,gather>+combine_pieces_kernel"
                          : "crc32c_blocks_kernel<16,pieces>+combine_pieces_kernel";
    }
}

UniformPlan uniform_plan(int cus, uint64_t base, uint64_t stride, uint32_t blen, uint64_t n, int gi) {
    UniformPlan pl{};
    pl.ps = pick_split(base, stride, blen, n, gi, cus);
    pl.bgi = -1;
    if (pl.ps > 0) {
        const uint64_t nv = n << pl.ps;
        const bool fused = (1u << pl.ps) <= lvk::kFuseMax && nv <= 64ull * static_cast<uint64_t>(cus);
        pl.scratch = fused ? 0 : nv * 4;
    } else {
        pl.bgi = pick_block_gi(base, stride, blen, gi, n, cus);
    }
    return pl;
}

int launch_uniform(DevCtx &c, const UniformPlan &pl, const uint8_t *base, uint64_t stride, const uint64_t *off,
                   const uint32_t *len, const HintCheck *hc, uint32_t blen, uint64_t n, const uint32_t *seed,
                   uint32_t *out, uint32_t flags, hipStream_t hs, uint8_t *scr) {
    if (pl.ps > 0) {
        const uint64_t plen = blen >> pl.ps;
        const uint32_t *mats = nullptr, *tabs = nullptr;
        if (int rc = piece_mats(c, plen, &mats)) return rc;
        if (pl.scratch && pl.ps >= 11)
            if (int rc = piece_tabs(c, plen, &tabs)) return rc;
        uint32_t *s32 = pl.scratch ? reinterpret_cast<uint32_t *>(scr) : nullptr;
        if (off)
            launch_pieces<true>(c, pl.ps, mats, tabs, base, stride, off, len, hc, blen, n, seed, out, flags, hs, s32);
        else
            launch_pieces<false>(c, pl.ps, mats, tabs, base, stride, off, len, hc, blen, n, seed, out, flags, hs,
                                 s32);
        return 0;
    }
    if (off)
        launch_blocks<true>(c, pl.bgi, base, stride, off, len, hc, blen, n, seed, out, flags, hs);
    else
        launch_blocks<false>(c, pl.bgi, base, stride, off, len, hc, blen, n, seed, out, flags, hs);
    return 0;
}

}  // namespace lvh

using namespace lvh;

extern "C" {

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
    const UniformPlan pl = uniform_plan(c->cus, reinterpret_cast<uint64_t>(d_base), stride, block_len, n, gi);
    if (pl.applies()) {
        // aligned whole-batch blocks: the uniform-block kernel, or its split
        uint8_t *scr = nullptr;
        std::unique_lock<std::mutex> ws_lk;  // held through both launches
        if (pl.scratch)
            if (int rc = stream_ws_bytes(*c, hs, pl.scratch, &scr, &ws_lk)) return rc;
        if (int rc = launch_uniform(*c, pl, d_base, stride, nullptr, nullptr, nullptr, block_len, n, d_seed, d_out,
                                    flags, hs, scr))
            return rc;
        return check_launch();
    }
    launch_g<true>(*c, gi >= 0 ? gi : pick_gi(block_len), d_base, nullptr, nullptr, stride, block_len, d_seed,
                   d_out, n, flags, hs);
    return check_launch();
}

}  // extern "C"
