// Length sort of the offsets API (lv_crc32c_batch_device): a counting sort
// by (length class, batch count) into 16-B entries, with the long-buffer
// split (pieces after the sorted entries), in three launches (sort_hist,
// sort_scan, sort_scatter) for batches of > 1,024 buffers (smaller ones:
// crc32c_fused_small_kernel, classes.hip).  No host sync, no device-scope
// fences.  Keys and workspace layout: lvk/sort.h.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "lvh.h"
#include "lvk/sort.h"

namespace lvk {

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
    __shared__ uint32_t part[64][17];  // padded: the transposed scan reads a column
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
    {  // inclusive scan over sub: wave w scans key w's 64 row ranges, one per lane (two barriers
       // instead of a 6-level Hillis-Steele over LDS with two barriers per level)
        const uint32_t lane = t & 63u, w = t >> 6;
        uint32_t x = part[lane][w];
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d);
            if (lane >= d) x += y;
        }
        part[lane][w] = x;
    }
    __syncthreads();
    if (sub == 63) ws[kWsTot + k] = part[63][kl];
    uint32_t run = part[sub][kl] - sum;  // exclusive
#pragma unroll
    for (uint32_t r = 0; r < 16; ++r) {
        if (r < R && r0 + r < wgs) M[static_cast<uint64_t>(r0 + r) * kKeys + k] = run;
        run += v[r];
    }
}

// Pass 3: same chunks as pass 1.  Workgroup w's slots for key k start at
// key_start[k] + M[w][k]; buffers claim them with wave-aggregated LDS
// atomics (order within a workgroup's run is not stable, which keeps metadata
// reads and CRC stores within one 4096-buffer window).  Entries carry
// off/len/index so the CRC kernel reads one 16-B record per buffer; seeds are
// permuted alongside.
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
    uint32_t p = 0;
    const uint32_t m = valid ? split_rule(L, total, &p) : 0u;
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
                                                             uint32_t *__restrict__ sseed, uint4 *__restrict__ longs,
                                                             uint32_t *__restrict__ spos) {
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
    const bool ident = __syncthreads_or(ident_ok);
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
                spos[i] = split ? 0xffffffffu : pos;  // in buffer order: coalesced
            }
        }
    }
}

}  // namespace lvk

namespace lvh {

// Sorting workgroups and elements per workgroup for n buffers.
// At 4,096 buffers per workgroup a batch under 1M buffers leaves most CUs
// idle in the sort passes: batches under 4M split into up to kSortMinWgs
// workgroups of >= 1,024 (262,144 buffers: 64 -> 256 workgroups, +2 % for
// the whole call; 1M buffers: 256 -> 1,024, +0.1 %).
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
    // the class kernel's CRCs by sorted position, and each buffer's sorted
    // position (combine_long_kernel's unsort)
    w.tmp = w.longs + (lvk::kPieceBudget / 2) * sizeof(uint4);
    w.pos = w.tmp + al16(n * sizeof(uint32_t));
    w.total = w.pos + al16(n * sizeof(uint32_t));
    return w;
}

size_t sort_ws_bytes(uint64_t n) { return ws_layout(n).total; }

uint4 *launch_sort(uint8_t *ws_bytes, const uint64_t *off, const uint32_t *len, const uint32_t *seed, uint64_t n,
                   hipStream_t s, lvk::Params *P) {
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
    // (n > 1,024: smaller batches take crc32c_fused_small_kernel, which
    // retired round 2's one-launch sort_small in round 3)
    hipLaunchKernelGGL(lvk::sort_hist, g, b, 0, s, len, n, chunk, M, ws, wgb);
    launch_sort_scan(M, static_cast<uint32_t>(wgs), ws, wgb, s);
    uint32_t *spos = reinterpret_cast<uint32_t *>(ws_bytes + lay.pos);
    hipLaunchKernelGGL(lvk::sort_scatter, g, b, 0, s, off, len, n, chunk, ws, M, ent, seed, sseed, longs, spos);
    P->ent = ent;
    P->tmp = reinterpret_cast<uint32_t *>(ws_bytes + lay.tmp);
    P->sseed = seed ? sseed : nullptr;
    P->part = longs ? part : nullptr;
    return longs;
}

void launch_sort_scan(uint32_t *M, uint32_t wgs, uint32_t *ws, uint64_t *wgb, hipStream_t s) {
    hipLaunchKernelGGL(lvk::sort_scan, dim3(lvk::kScanWgs), dim3(lvk::kScanThreads), 0, s, M, wgs, ws, wgb);
}

}  // namespace lvh
