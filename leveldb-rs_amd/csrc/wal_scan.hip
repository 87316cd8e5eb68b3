// Host-memory WAL scan (the reader side of SURVEY 8f row 1): upload, then
// the device scan lv_wal_scan_device (below: each 32 KiB block's
// header chain is walked inside the length sort's passes, as
// Reader::read_physical_record frames it, log_reader.rs:271-331, and every
// [type || payload] unit is checksummed), then the arrays come back.
// Headers past a checksum mismatch in the same block are also emitted: the
// host reader never consults them (it drops the rest of the block,
// log_reader.rs:337-342).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "../../include/lvgpu/crc32c.h"
#include "../../include/lvgpu/wal.h"
#include "lv_internal.h"
#include "lvh.h"
#include "lvk/sort.h"

namespace lvk {

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
// units (by sorted position; wal_unsort writes them in log order).  Five
// launches, no host synchronisation (round 1: count pass, hipCUB
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
// longest chain is 54.  (Touching after 8 / 12 / 24 hops instead of 16:
// 0.602 / 0.627 / 0.632 against 0.633, profiles/r04/wal_touch/.)
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

// One thread per block, kWalHistThreads per workgroup: with 64 (one wave,
// 33 KiB of header cache) the 32,768 blocks of a 1 GiB log spread over 512
// workgroups on all CUs; 256 threads (130 KiB each, one workgroup per CU)
// left half the CUs idle and put two chains per SIMD.
constexpr uint32_t kWalHistThreads = 64;
__global__ __launch_bounds__(kWalHistThreads) void wal_hist(const uint8_t *__restrict__ log, uint64_t size,
                                                            uint64_t nblocks, uint64_t chunk,
                                                            uint32_t *__restrict__ M, uint64_t *__restrict__ wgrec,
                                                            uint32_t *__restrict__ blkcnt,
                                                            uint64_t *__restrict__ hcache) {
    constexpr uint32_t T = kWalHistThreads;
    __shared__ uint32_t h[kKeys + 64];  // + a dummy bin per lane (finished lanes)
    __shared__ uint64_t wsum[T / 64];
    __shared__ uint64_t hcl[T * (kHdrCache + 1)];  // per-thread header cache
    const uint32_t t = threadIdx.x, lane = t & 63u;
    for (uint32_t k = t; k < kKeys; k += T) h[k] = 0;
    __syncthreads();
    const uint64_t lo = blockIdx.x * chunk, hi = lo + chunk < nblocks ? lo + chunk : nblocks;
    uint64_t mine = 0;
    uint32_t touched = 0;
    for (uint64_t b0 = lo; b0 < hi; b0 += T) {  // block-uniform
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
        // Branch-free hop (round 3): every lane runs every instruction of the
        // loop body (no exec-mask branches) but the loads; the next header's
        // loads are issued right after the decode, and this record's
        // bookkeeping -- the header cache slot in LDS and a fire-and-forget
        // LDS atomic on its sort key -- runs while they are in flight.
        // Finished lanes write their pad cache slot (64) and count into a
        // per-lane dummy bin.  One wave per SIMD runs this loop alone, so the
        // hop is bound by its instruction latency as much as by the load:
        // timing variants (profiles/r03/wal2/) put a chain walk with no
        // bookkeeping at 16.4 us of the round-2 body's 31.4; the wave-
        // aggregated count (ballots, a lane broadcast through LDS and its
        // wait) -> one atomic per record took 31.8 -> 26.9 us, the branch-free
        // body -> 22.8.  Loads for every lane (finished ones rereading their
        // last header from L2) made it 41.8 us: a load instruction's cost
        // grows with the lines its lanes touch, so the loads stay exec-masked.
        // The framing needs header bytes 4..6 (length, type): the two aligned
        // dwords around them and one v_alignbyte_b32 (+0.4 % over a 64-bit
        // funnel shift).  The second dword holds one of those bytes only when
        // they straddle; otherwise it is clamped to the log's last dword.
        // in-block 32-bit offsets (blocks start 32 KiB-aligned in the 8-B-aligned log; +0.4 %)
        const uint8_t *const blk = log + start;
        const uint32_t lastd = (blen - 1u) & ~3u;  // the block's last aligned dword
        uint32_t wlo = 0, whi = 0, wsh = 0;
        auto issue = [&](uint32_t p, bool on) {
            const uint32_t pr = p + 4u, ar = pr & ~3u;
            wsh = pr & 3u;
            if (on) {
                wlo = *reinterpret_cast<const uint32_t *>(blk + ar);
                whi = *reinterpret_cast<const uint32_t *>(blk + (ar + 4u < lastd ? ar + 4u : lastd));
            }
        };
        issue(0, active);
        while (__any(active)) {  // wave-uniform: the longest chain of the wave
            if (LVK_WAL_TOUCH_HOPS && hops++ == LVK_WAL_TOUCH_HOPS)
                touched ^= wal_touch(log, b0 + (t & ~63u), pos, blen, active, lane);
            const uint32_t hw = __builtin_amdgcn_alignbyte(whi, wlo, wsh);  // bytes pos + 4 .. pos + 7
            const uint32_t len = hw & 0xffffu;
            const uint32_t type = (hw >> 16) & 0xffu;
            // log_reader.rs:312-331: BAD_LENGTH past the block, ZERO at a 0/0 header
            const bool ok = kWalHeader + len <= blen - pos && (type | len) != 0u;
            const uint32_t npos = pos + kWalHeader + len;
            const bool nact = active && ok && blen - npos >= kWalHeader;
            issue(npos, nact);
            const uint32_t slot = active && cnt < kHdrCache ? cnt : kHdrCache;
            hl[slot] = hdr_pack(pos, len, type);
            const uint32_t key = active ? sort_key(ok ? len + 1u : 0u) : kKeys + lane;
            __hip_atomic_fetch_add(&h[key], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            cnt += active ? 1u : 0u;
            pos = npos;
            active = nact;
        }
        // (Writing the cache block by block with consecutive lanes -- one
        // contiguous run per block instead of 64 scattered 8-B stores per
        // step -- measured slower: 0.633 -> 0.622, profiles/r04/wal_hc/.)
        for (uint32_t c = 0; c < cnt && c < kHdrCache; ++c) hcache[b * kHdrCache + c] = hl[c];
        if (b < hi) blkcnt[b] = cnt;
        mine += cnt;
    }
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) mine += __shfl_xor(mine, k);
    if (lane == 0) wsum[t >> 6] = mine;
    asm volatile("" ::"v"(touched));  // the touches are kept
    __syncthreads();
    for (uint32_t k = t; k < kKeys; k += T) M[static_cast<uint64_t>(blockIdx.x) * kKeys + k] = h[k];
    if (t == 0) {
        uint64_t all = 0;
        for (uint32_t w = 0; w < T / 64; ++w) all += wsum[w];
        wgrec[blockIdx.x] = all;  // sort_scan sums these
    }
}

// Output of the WAL scan, in log order (lv_wal_scan_device).
struct WalOut {
    uint64_t *hdr_off;
    uint32_t *info;  // type | status << 8 | length << 16
    uint64_t *count;
    uint64_t cap;
    uint32_t *spos;  // each record's sorted position (wal_unsort), or null
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
    // this workgroup's first record in log order: the records of the ones
    // before (a wave reduction per wave, then the four wave sums)
    uint64_t pre = 0;
    for (uint32_t v = t; v < blockIdx.x; v += kSortThreads) pre += wgrec[v];
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) pre += __shfl_xor(pre, k);
    if (lane == 0) red[t >> 6] = pre;
    __syncthreads();
    uint64_t run = 0;
#pragma unroll
    for (uint32_t k = 0; k < kSortThreads / 64; ++k) run += red[k];
    __syncthreads();
    if (over) return;  // block-uniform
    __shared__ uint32_t wt[kSortThreads / 64];
    const uint64_t lo = blockIdx.x * chunk, hi = lo + chunk < nblocks ? lo + chunk : nblocks;
    for (uint64_t b0 = lo; b0 < hi; b0 += kSortThreads) {  // block-uniform
        const uint64_t b = b0 + t;
        const uint32_t c = b < hi ? blkcnt[b] : 0u;
        red[t] = wg_incl_scan<kSortThreads / 64>(c, wt);  // inclusive prefix of the block counts
        __syncthreads();
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
                if (o.spos) o.spos[rid] = slot;
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
                    if (o.spos) o.spos[rid] = slot;
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

// The class kernel stored each record's CRC at its sorted position (runs of
// consecutive words); crc[rid] = tmp[spos[rid]] writes them in log order,
// whole lines (scattered single-word stores from the class kernel cost the
// offsets API's C2 ~35 us, profiles/r04/outstore/).
__global__ __launch_bounds__(1024) void wal_unsort(const uint32_t *__restrict__ ws, const uint32_t *__restrict__ tmp,
                                                   const uint32_t *__restrict__ spos, uint32_t *__restrict__ crc,
                                                   uint64_t cap) {
    const uint64_t total = (static_cast<uint64_t>(ws[kWsBytes + 1]) << 32) | ws[kWsBytes];  // records
    if (total > cap) return;  // nothing was written: the caller retries with a larger capacity
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += stride)
        crc[i] = tmp[spos[i]];
}

}  // namespace lvk

using namespace lvh;

extern "C" {

// ---- WAL scan of a log in HBM (include/lvgpu/wal.h) ----
static uint64_t wal_wgs(uint64_t nblocks, uint64_t *chunk) {
    uint64_t wgs = (nblocks + lvk::kWalHistThreads - 1) / lvk::kWalHistThreads;
    wgs = std::max<uint64_t>(1, std::min<uint64_t>(wgs, lvk::kSortMaxWgs));
    *chunk = (nblocks + wgs - 1) / wgs;
    return wgs;
}

struct WalWs {
    size_t m, wgrec, blk, hc, ent, tmp, pos, total;
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
    // with LVK_WAL_UNSORT: the CRCs by sorted position and each record's sorted position
    w.tmp = w.ent + cap * sizeof(uint4);
    w.pos = w.tmp + (LVK_WAL_UNSORT ? al16(cap * sizeof(uint32_t)) : 0);
    w.total = w.pos + (LVK_WAL_UNSORT ? al16(cap * sizeof(uint32_t)) : 0);
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
    if (workspace_bytes < lv_wal_scan_workspace_bytes(bytes, cap)) return set_err(LV_ERR_INVALID, "workspace too small");
    DevCtx *c = nullptr;
    if (int rc = current_ctx(&c)) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint64_t nblocks = (bytes + lvk::kWalBlock - 1) / lvk::kWalBlock;
    if (nblocks == 0) {
        LV_HIP(hipMemsetAsync(d_count, 0, sizeof(uint64_t), s));
        return LV_OK;
    }
    uint8_t *wb = static_cast<uint8_t *>(d_workspace);
    // (Round 5 measured a one-launch scan beside this one -- every workgroup
    // framing, sorting and checksumming its own blocks -- at 0.622 of 8 TB/s
    // against 0.632: its per-workgroup rounds ended ragged and the slowest
    // workgroup set the launch, profiles/r05/wal_paths/.  Round 6 removed it.)
    uint32_t *ws = reinterpret_cast<uint32_t *>(wb);
    uint32_t *M = reinterpret_cast<uint32_t *>(wb + lay.m);
    uint64_t *wgrec = reinterpret_cast<uint64_t *>(wb + lay.wgrec);
    uint32_t *blk = reinterpret_cast<uint32_t *>(wb + lay.blk);
    uint64_t *hc = reinterpret_cast<uint64_t *>(wb + lay.hc);
    uint4 *ent = reinterpret_cast<uint4 *>(wb + lay.ent);
    uint64_t chunk = 0;
    const uint64_t wgs = wal_wgs(nblocks, &chunk);
    const dim3 g(static_cast<uint32_t>(wgs)), b(lvk::kSortThreads);
    hipLaunchKernelGGL(lvk::wal_hist, g, dim3(lvk::kWalHistThreads), 0, s, d_log, static_cast<uint64_t>(bytes), nblocks,
                       chunk, M, wgrec, blk, hc);
    // (Round 3: claiming each workgroup's key runs with device atomics in
    // wal_hist instead of this column scan -- a memset of the totals first --
    // measured 0.6 % slower: the memset launch and wal_hist's returning
    // atomics cost more than sort_scan, profiles/r03/wal2/atomic_totals/.)
    launch_sort_scan(M, static_cast<uint32_t>(wgs), ws, wgrec, s);
    uint32_t *tmp = LVK_WAL_UNSORT ? reinterpret_cast<uint32_t *>(wb + lay.tmp) : nullptr;
    uint32_t *spos = LVK_WAL_UNSORT ? reinterpret_cast<uint32_t *>(wb + lay.pos) : nullptr;
    lvk::WalOut o{d_hdr_off, d_info, d_count, cap, spos};
    hipLaunchKernelGGL(lvk::wal_scatter, g, b, 0, s, d_log, static_cast<uint64_t>(bytes), nblocks, chunk, ws, M, wgrec,
                       blk, hc, ent, o);
    lvk::Params P{};
    P.base = reinterpret_cast<uint64_t>(d_log);
    P.out = d_crc;
    P.n = cap;
    P.nplain = cap;
    P.ent = ent;
    P.tmp = tmp;
    launch_classes(*c, false, P, ws, s);
    g_kernel = "wal_hist+sort_scan+wal_scatter+crc32c_classes_kernel";
    if (tmp && cap) {
        hipLaunchKernelGGL(lvk::wal_unsort, dim3(static_cast<uint32_t>(std::min<uint64_t>(c->cus, (cap + 1023) / 1024))),
                           dim3(1024), 0, s, ws, tmp, spos, d_crc, static_cast<uint64_t>(cap));
        g_kernel = "wal_hist+sort_scan+wal_scatter+crc32c_classes_kernel+wal_unsort";
    }
    return check_launch();
}

}  // extern "C"

namespace {

constexpr size_t align16(size_t x) { return (x + 15) & ~static_cast<size_t>(15); }

int hip_err(hipError_t e, const char *what) {
    if (e == hipSuccess) return LV_OK;
    return lvgpu_internal::set_error(static_cast<int>(e), (std::string(what) + ": " + hipGetErrorString(e)).c_str());
}

}  // namespace

// The log goes to the device through the device's host path (cached arena;
// pinned input: one DMA, pageable: pipelined pinned staging); the scan is
// lv_wal_scan_device into the device's cached scratch buffer, so a scan
// allocates nothing on the device after the first call.  The capacity starts
// at a guess (one record per 256 log bytes, at least 8 per block); a log with
// more records is scanned again at its exact count.
int lvgpu_internal::scan_host_range(const uint8_t *log, size_t bytes, uint64_t base, int device, ScanChunk *out) {
    const uint64_t nblocks = (bytes + LV_WAL_BLOCK_SIZE - 1) / LV_WAL_BLOCK_SIZE;
    if (nblocks == 0) return LV_OK;
    lvgpu_internal::HostPath hp;
    if (int rc = lvgpu_internal::host_upload(device, log, bytes, 16, &hp)) return rc;
    hipStream_t s = static_cast<hipStream_t>(hp.stream);
    uint64_t cap = std::max<uint64_t>(bytes / 256, nblocks * 8), count = 0;
    int rc = LV_OK;
    for (int attempt = 0; attempt < 2; ++attempt) {
        const size_t wsb = align16(lv_wal_scan_workspace_bytes(bytes, cap));
        const size_t need = wsb + align16(cap * 8) + 2 * align16(cap * 4) + 16;
        uint8_t *scr = nullptr;
        if ((rc = lvgpu_internal::host_scratch(&hp, 0, need, &scr))) break;
        uint64_t *d_hdr = reinterpret_cast<uint64_t *>(scr + wsb);
        uint32_t *d_crc = reinterpret_cast<uint32_t *>(scr + wsb + align16(cap * 8));
        uint32_t *d_info = reinterpret_cast<uint32_t *>(scr + wsb + align16(cap * 8) + align16(cap * 4));
        uint64_t *d_count = reinterpret_cast<uint64_t *>(scr + need - 16);
        if ((rc = lv_wal_scan_device(hp.d_arena, bytes, d_hdr, d_crc, d_info, cap, d_count, scr, wsb, s))) break;
        if ((rc = hip_err(hipMemcpyAsync(&count, d_count, 8, hipMemcpyDeviceToHost, s), "D2H")) ||
            (rc = hip_err(hipStreamSynchronize(s), "sync")))
            break;
        lvgpu_internal::count_d2h(8);  // counted once it has arrived, on every attempt
        if (count > cap) {  // more records than the guess: once more at the exact count
            cap = count;
            continue;
        }
        out->off.resize(count);
        out->crc.resize(count);
        out->info.resize(count);
        if (count &&
            ((rc = hip_err(hipMemcpyAsync(out->off.data(), d_hdr, count * 8, hipMemcpyDeviceToHost, s), "D2H")) ||
             (rc = hip_err(hipMemcpyAsync(out->crc.data(), d_crc, count * 4, hipMemcpyDeviceToHost, s), "D2H")) ||
             (rc = hip_err(hipMemcpyAsync(out->info.data(), d_info, count * 4, hipMemcpyDeviceToHost, s), "D2H")) ||
             (rc = hip_err(hipStreamSynchronize(s), "sync"))))
            break;
        lvgpu_internal::count_d2h(count * 16);  // after the copies succeeded
        if (base)
            for (auto &o : out->off) o += base;
        return LV_OK;
    }
    (void)hipStreamSynchronize(s);
    if (!rc || !*lv_last_error()) rc = lvgpu_internal::set_error(rc ? rc : LV_ERR_INVALID, "WAL scan failed");
    return rc;
}

extern "C" lv_wal_scan *lv_wal_scan_host(const uint8_t *log, size_t bytes, int device) {
    if (!log && bytes) {
        lvgpu_internal::set_error(LV_ERR_INVALID, "null log");
        return nullptr;
    }
    lv_wal_scan *scan = new lv_wal_scan();
    lvgpu_internal::ScanChunk ch;
    if (lvgpu_internal::scan_host_range(log, bytes, 0, device, &ch)) {
        delete scan;
        return nullptr;
    }
    scan->off.swap(ch.off);
    scan->crc.swap(ch.crc);
    scan->info.swap(ch.info);
    return scan;
}

// Pipelined recovery pass (VERDICT r04 missing 3): the log is scanned in
// block-aligned chunks of kPipeChunk bytes by a worker thread while a Reader
// over the returned scan replays chunk k on the caller's thread (records never
// straddle a block, log_writer.rs:67-80, so a chunk's scan is exact on its
// own).  The Reader waits only for the chunk holding the header it reaches
// next.  The worker keeps two chunks in flight on two streams: while the GPU
// uploads and scans chunk k, the worker copies chunk k + 1 into the other
// pinned staging slot (a pageable log) and then collects chunk k's arrays.
// Round 6: the chunks ramp up from kPipeFirst, doubling to kPipeChunk, so
// the Reader starts after a small first chunk instead of after a whole 32 MiB
// one (and, for a pageable log, the CPU copy of the second one).
constexpr uint64_t kPipeChunk = static_cast<uint64_t>(LVK_PIPE_CHUNK_MB) << 20;  // 32 MiB: 1,024 blocks
constexpr uint64_t kPipeFirst = static_cast<uint64_t>(LVK_PIPE_FIRST_MB) << 20;  // 2 MiB
static_assert(kPipeChunk % LV_WAL_BLOCK_SIZE == 0, "chunks are whole blocks");
static_assert(kPipeFirst % LV_WAL_BLOCK_SIZE == 0 && kPipeFirst > 0 && kPipeFirst <= kPipeChunk,
              "the first chunk is whole blocks, at most a full chunk");
static_assert(kPipeChunk <= kStageBytes, "a chunk fits one staging slot");

namespace {

// One of the worker's two slots: stream, device copy of a chunk, scratch,
// pinned staging and count word, and the chunk it holds.
struct PipeSlot {
    hipStream_t s = nullptr;
    uint8_t **d_log = nullptr;
    size_t *d_log_cap = nullptr;
    uint8_t **scr = nullptr;
    size_t *scr_cap = nullptr;
    uint8_t *stage = nullptr;
    uint64_t *hcnt = nullptr;
    uint64_t lo = 0, len = 0, cap = 0;
    uint64_t *d_hdr = nullptr, *d_count = nullptr;
    uint32_t *d_crc = nullptr, *d_info = nullptr;
};

// The slot's chunk (already on the device) scanned at capacity sl.cap, the
// count copied back to the pinned word.
int pipe_scan(PipeSlot &sl) {
    const size_t wsb = align16(lv_wal_scan_workspace_bytes(sl.len, sl.cap));
    const size_t need = wsb + align16(sl.cap * 8) + 2 * align16(sl.cap * 4) + 16;
    if (int rc = grow_dev(sl.scr, sl.scr_cap, need)) return rc;
    uint8_t *scr = *sl.scr;
    sl.d_hdr = reinterpret_cast<uint64_t *>(scr + wsb);
    sl.d_crc = reinterpret_cast<uint32_t *>(scr + wsb + align16(sl.cap * 8));
    sl.d_info = reinterpret_cast<uint32_t *>(scr + wsb + align16(sl.cap * 8) + align16(sl.cap * 4));
    sl.d_count = reinterpret_cast<uint64_t *>(scr + need - 16);
    if (int rc = lv_wal_scan_device(*sl.d_log, sl.len, sl.d_hdr, sl.d_crc, sl.d_info, sl.cap, sl.d_count, scr, wsb,
                                    sl.s))
        return rc;
    return hip_err(hipMemcpyAsync(sl.hcnt, sl.d_count, 8, hipMemcpyDeviceToHost, sl.s), "D2H");
}

// Chunk [sl.lo, sl.lo + sl.len) onto the slot's stream: the copy (for a
// pageable log, through the slot's pinned staging -- the CPU copy overlaps
// the other slot's upload and scan), then the scan.
int pipe_enqueue(PipeSlot &sl, const uint8_t *log, bool pinned) {
    if (int rc = grow_dev(sl.d_log, sl.d_log_cap, sl.len + 16)) return rc;
    const uint8_t *src = log + sl.lo;
    if (!pinned) {
        // (4 copy threads, not the host path's 8: the Reader on the caller's
        // thread replays beside this copy, and with 8 it ran ~35 % slower --
        // recovery 21.4-22.1 GiB/s with 8, 26.7-26.9 with 4, the scan alone
        // 20.2-20.5 ms either way; profiles/r05/wal_host/)
        par_memcpy(sl.stage, src, sl.len, LVK_PIPE_COPY_THREADS);
        src = sl.stage;
    }
    if (int rc = hip_err(hipMemcpyAsync(*sl.d_log, src, sl.len, hipMemcpyHostToDevice, sl.s), "H2D")) return rc;
    if (int rc = hip_err(hipMemsetAsync(*sl.d_log + sl.len, 0, 16, sl.s), "memset")) return rc;
    lvgpu_internal::count_h2d(sl.len);
    return pipe_scan(sl);
}

// Waits for the slot's scan (once more at the exact count if the guess was
// short), then its arrays back.
int pipe_finish(PipeSlot &sl, lvgpu_internal::ScanChunk *out) {
    for (int attempt = 0;; ++attempt) {
        if (int rc = hip_err(hipStreamSynchronize(sl.s), "sync")) return rc;
        lvgpu_internal::count_d2h(8);
        const uint64_t count = *sl.hcnt;
        if (count > sl.cap && attempt < 1) {
            sl.cap = count;
            if (int rc = pipe_scan(sl)) return rc;
            continue;
        }
        if (count > sl.cap) return lvgpu_internal::set_error(LV_ERR_INVALID, "WAL scan failed");
        out->off.resize(count);
        out->crc.resize(count);
        out->info.resize(count);
        if (count) {
            int rc;
            if ((rc = hip_err(hipMemcpyAsync(out->off.data(), sl.d_hdr, count * 8, hipMemcpyDeviceToHost, sl.s), "D2H")) ||
                (rc = hip_err(hipMemcpyAsync(out->crc.data(), sl.d_crc, count * 4, hipMemcpyDeviceToHost, sl.s), "D2H")) ||
                (rc = hip_err(hipMemcpyAsync(out->info.data(), sl.d_info, count * 4, hipMemcpyDeviceToHost, sl.s),
                              "D2H")) ||
                (rc = hip_err(hipStreamSynchronize(sl.s), "sync")))
                return rc;
            lvgpu_internal::count_d2h(count * 16);
        }
        for (auto &o : out->off) o += sl.lo;
        return LV_OK;
    }
}

// The worker: every chunk of the log, two in flight, each published (in
// order) as soon as its arrays are back.
int pipe_run(lvgpu_internal::ScanPipe *p, const uint8_t *log, size_t bytes, int device) {
    lvgpu_internal::DeviceGuard dg;
    if (int rc = dg.set(device)) return rc;
    DevCtx *c = nullptr;
    if (int rc = current_ctx(&c)) return rc;
    std::lock_guard<std::mutex> lk(c->host_m);  // the device's host-path buffers and streams
    if (!c->stream) LV_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    if (!c->stream2) LV_HIP(hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking));
    // earlier host-path copies out of the staging slots are done
    for (auto &ev : c->ev)
        if (ev) LV_HIP(hipEventSynchronize(ev));
    const bool pinned = is_pinned(log);
    if (!pinned)
        for (int k = 0; k < 2; ++k)
            if (int rc = grow_pinned(&c->h_stage[k], &c->h_stage_cap[k], kStageBytes)) return rc;
    if (int rc = grow_pinned(&c->h_meta, &c->h_meta_cap, 16)) return rc;
    PipeSlot slot[2];
    slot[0].s = c->stream;
    slot[0].d_log = &c->d_arena;
    slot[0].d_log_cap = &c->d_arena_cap;
    slot[1].s = c->stream2;
    slot[1].d_log = &c->d_arena2;
    slot[1].d_log_cap = &c->d_arena2_cap;
    for (int k = 0; k < 2; ++k) {
        slot[k].scr = &c->d_scr[k];
        slot[k].scr_cap = &c->d_scr_cap[k];
        slot[k].stage = c->h_stage[k];
        slot[k].hcnt = reinterpret_cast<uint64_t *>(c->h_meta) + k;
    }
    auto publish = [&](size_t k) {
        std::lock_guard<std::mutex> g(p->m);
        p->ready = k + 1;
        p->ready_seen.store(k + 1, std::memory_order_release);
        p->cv.notify_all();
    };
    const size_t nch = p->chunks.size();
    int rc = LV_OK;
    for (size_t k = 0; k < nch && !rc; ++k) {
        PipeSlot &sl = slot[k & 1];
        sl.lo = p->lo[k];
        sl.len = p->lo[k + 1] - sl.lo;
        const uint64_t nblocks = (sl.len + LV_WAL_BLOCK_SIZE - 1) / LV_WAL_BLOCK_SIZE;
        sl.cap = std::max<uint64_t>(sl.len / 256, nblocks * 8);
        rc = pipe_enqueue(sl, log, pinned);
        if (!rc && k > 0 && !(rc = pipe_finish(slot[(k - 1) & 1], &p->chunks[k - 1]))) publish(k - 1);
    }
    if (!rc && !(rc = pipe_finish(slot[(nch - 1) & 1], &p->chunks[nch - 1]))) publish(nch - 1);
    // nothing of this scan is still reading the staging slots or scratch
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->stream2);
    return rc;
}

}  // namespace

extern "C" lv_wal_scan *lv_wal_scan_host_pipelined(const uint8_t *log, size_t bytes, int device) {
    if (!log && bytes) {
        lvgpu_internal::set_error(LV_ERR_INVALID, "null log");
        return nullptr;
    }
    lv_wal_scan *scan = new lv_wal_scan();
    auto *p = new lvgpu_internal::ScanPipe();
    scan->pipe.reset(p);
    for (uint64_t at = 0, c = kPipeFirst; at < bytes; at += c, c = std::min(2 * c, kPipeChunk)) p->lo.push_back(at);
    p->lo.push_back(bytes);
    const size_t nch = p->lo.size() - 1;
    p->chunks.resize(nch);
    if (nch == 0) {
        p->flat = true;
        return scan;
    }
    p->worker = std::thread([p, log, bytes, device] {
        const int rc = pipe_run(p, log, bytes, device);
        if (rc) {
            std::lock_guard<std::mutex> lk(p->m);
            p->rc = rc;
            p->err = lv_last_error();
            p->cv.notify_all();
        }
    });
    return scan;
}

int lvgpu_internal::scan_flatten(lv_wal_scan *scan) {
    if (!scan || !scan->pipe) return LV_OK;
    ScanPipe &p = *scan->pipe;
    if (p.chunks.size()) {
        if (int rc = p.wait(p.chunks.size() - 1)) return lvgpu_internal::set_error(rc, ("WAL scan: " + p.err).c_str());
    }
    std::lock_guard<std::mutex> lk(p.m);
    if (!p.flat) {
        size_t n = 0;
        for (const auto &c : p.chunks) n += c.off.size();
        scan->off.reserve(n);
        scan->crc.reserve(n);
        scan->info.reserve(n);
        for (const auto &c : p.chunks) {
            scan->off.insert(scan->off.end(), c.off.begin(), c.off.end());
            scan->crc.insert(scan->crc.end(), c.crc.begin(), c.crc.end());
            scan->info.insert(scan->info.end(), c.info.begin(), c.info.end());
        }
        p.flat = true;
    }
    return LV_OK;
}
