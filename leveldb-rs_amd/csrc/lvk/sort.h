// Length sort of the offsets API: keys, workspace layout and the wave-level
// counting helpers shared by the sort passes (sort.hip), the WAL framing
// (wal_scan.hip) and the walks (lvk/walk.h).
#pragma once
#include "core.h"

namespace lvk {

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
constexpr uint32_t kAlRows = LVK_AL_ROWS;

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
constexpr uint32_t kWsIdent = 4;  // 1: the sorted list is the identity (one key, no split): see sort_scatter
constexpr uint32_t kPieceBudget = 65536;  // piece entries per call (each split buffer takes <= kMaxPieces)
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

// Inclusive scan of v over a workgroup of W waves: wave scans (lane shuffles),
// then the earlier waves' totals from `wt` (W LDS words); one barrier
// (the caller's next write to `wt` must follow a barrier).  (Round 3: the
// Hillis-Steele scans in LDS, two barriers per step, cost the sort and WAL
// scatter passes ~1 us each.)
template <uint32_t W>
__device__ __forceinline__ uint32_t wg_incl_scan(uint32_t v, uint32_t *wt) {
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint32_t inc = v;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t x = __shfl_up(inc, d);
        if (lane >= d) inc += x;
    }
    if (lane == 63) wt[w] = inc;
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < W; ++k) inc += k < w ? wt[k] : 0u;
    return inc;
}

// Exclusive scan of the 256 key totals (one per thread of a 256-thread
// workgroup); sc[] gets the inclusive prefix; returns this thread's key start.
__device__ __forceinline__ uint32_t key_starts(const uint32_t *ws, uint32_t *sc) {
    __shared__ uint32_t wt[kKeys / 64];
    const uint32_t t = threadIdx.x;
    const uint32_t mine = ws[kWsTot + t];
    const uint32_t inc = wg_incl_scan<kKeys / 64>(mine, wt);
    sc[t] = inc;
    __syncthreads();
    return inc - mine;
}

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

// Pieces m of a buffer of L bytes in a batch of `total` payload bytes, and
// log2 of their length in *p; 0 when the buffer stays whole.  P >= batch
// bytes / 16,384 must hold for every batch (no cap below 31): it bounds the
// pieces of a call, sum m <= 16,384 + 8,192, and the split buffers, <= 8,192,
// inside kPieceBudget and kPieceBudget / 2.  A split needs L > 2P and
// L < 2^32, so split buffers have p <= 30, and the join's shifts Shift_{2^i},
// i <= p + lc + 5 <= 30 + 6 + 5, stay below kBaseMats.
// (pmin, maxp: the smallest piece, log2, and the most pieces of a buffer;
// the sort's split keeps 4 KiB and kMaxPieces, the fused small-batch path
// cuts finer, crc32c_fused_small_kernel.)
__device__ __forceinline__ uint32_t split_rule(uint32_t L, uint64_t total, uint32_t *p, uint32_t pmin = 12u,
                                               uint32_t maxp = kMaxPieces) {
    *p = 0;
    if (L <= 16384u) return 0u;
    uint32_t q = ceil_log2(total / 16384u);
    const uint32_t pl = ceil_log2((static_cast<uint64_t>(L) + maxp - 1) / maxp);
    q = q > pl ? q : pl;
    q = q > pmin ? q : pmin;
    q = q < 31u ? q : 31u;
    if (L <= (2ull << q)) return 0u;
    *p = q;
    return static_cast<uint32_t>((L + (1ull << q) - 1) >> q);
}

}  // namespace lvk
