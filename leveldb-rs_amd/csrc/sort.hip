// Length sort of the offsets API (lv_crc32c_batch_device): a counting sort
// by (length class, batch count) into 16-B entries, with the long-buffer
// split (pieces after the sorted entries), in one launch for small batches
// (sort_small) or three (sort_hist, sort_scan, sort_scatter).  No host sync,
// no device-scope fences.  Keys and workspace layout: lvk/sort.h.
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
        uint32_t p = 0;
        const uint32_t m = longs && valid ? split_rule(l[e], total, &p) : 0u;
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
    w.total = w.longs + (lvk::kPieceBudget / 2) * sizeof(uint4);
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
    if (n <= lvk::kSmallSort && LVK_SMALL_SORT) {  // one launch (sort_small)
        const dim3 gs(static_cast<uint32_t>(std::max<uint64_t>(wgs, lvk::kSmallSortWgs)));
        hipLaunchKernelGGL(lvk::sort_small, gs, b, 0, s, off, len, n, chunk, ws, ent, seed, sseed, longs);
    } else {
        hipLaunchKernelGGL(lvk::sort_hist, g, b, 0, s, len, n, chunk, M, ws, wgb);
        launch_sort_scan(M, static_cast<uint32_t>(wgs), ws, wgb, s);
        hipLaunchKernelGGL(lvk::sort_scatter, g, b, 0, s, off, len, n, chunk, ws, M, ent, seed, sseed, longs);
    }
    P->ent = ent;
    P->sseed = seed ? sseed : nullptr;
    P->part = longs ? part : nullptr;
    return longs;
}

void launch_sort_scan(uint32_t *M, uint32_t wgs, uint32_t *ws, uint64_t *wgb, hipStream_t s) {
    hipLaunchKernelGGL(lvk::sort_scan, dim3(lvk::kScanWgs), dim3(lvk::kScanThreads), 0, s, M, wgs, ws, wgb);
}

}  // namespace lvh
