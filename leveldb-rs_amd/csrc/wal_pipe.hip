// The device WAL scan in ONE persistent launch (round 5; lv_wal_scan_device,
// the reader side of SURVEY 8f row 1: log_reader.rs:271-364).
//
// Round 4's scan ran five launches: the header chains of every 32 KiB block
// (wal_hist, ~22 us: dependent HBM misses, most of the chip idle), a column
// scan, a scatter into one global length sort, the class kernel (174 us) and
// an unsort.  The chains were ~17 % of the call and ran before any CRC.
//
// Here workgroup w owns a contiguous range of blocks (~4 MiB of a 1 GiB log
// on 256 CUs) and does everything for it:
//   1. every thread reads the first header of one block (one round trip,
//      under the table staging): each block's first record is known at once
//      -- 59 % of the bench log's bytes (a FIRST / MIDDLE fragment fills its
//      block);
//   2. the first records of > 2 KiB units are counting-sorted in LDS (longest
//      first) and 14-16 waves start checksumming them ("phase A") with the
//      class kernel's G = 16 aligned-row walk;
//   3. meanwhile one or two framer waves walk the rest of every block's chain
//      (as read_physical_record frames it, log_reader.rs:271-331), caching
//      headers and counting sort keys -- hidden under phase A;
//   4. the last framer wave publishes the workgroup's record count (an 8-B
//      {tag, count} granule, agent-scope sc1 store), reads every other
//      workgroup's (a bounded relaxed poll: the counts of the workgroups before
//      it give its base in the log-order output, all of them the total for
//      the capacity check), writes hdr_off / info of its records in log order
//      and counting-sorts the rest of its records into ent[base, ...) by
//      (class, batches) -- the same key as the global sort -- then raises an
//      LDS flag;
//   5. the waves walk that local list (classes 2, 1, 0 with G = 16, 4, 1),
//      CRCs staged in LDS by record index, and the workgroup writes its CRCs
//      in log order at the end.
// (Round 5: phase-B rounds shared across workgroups -- per-workgroup round
// counters in global memory, claimed with device-scope atomics one round
// ahead, idle waves taking rounds of the workgroup with the most left -- ran
// the call in 0.42-0.44 ms instead of 0.21; with the same code on LDS
// counters and no sharing 0.256 ms (profiles/r05/wal_steal/).  A device
// atomic under the scan's read stream costs far more than a round of the
// small classes, and the direct scattered CRC stores of that version cost
// ~40 us more than staging them in LDS.  Not kept.)
// No cross-workgroup data moves but the 8-B counts: one granule array per
// stream (library-owned, zeroed once when made), which every launch leaves
// zeroed again -- the last workgroup to finish its look-back clears it -- so
// a call is one kernel launch and no memset.  A per-workgroup sort of
// ~700 records keeps rounds as uniform as the global sort did (simulated:
// 0.99 of the batch-count efficiency of the global sort).
// LDS: the image without region B (the aligned walk's merge reads the plain
// combine tables 4 / 5 instead, merge_al<PLAIN>), so region B's 64 KiB hold
// the workgroup's block tables, key histograms and the CRC staging.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/lvgpu/wal.h"
#include "lvh.h"
#include "lvk/walk.h"

namespace lvk {

constexpr uint32_t kPipeBlockSize = 32768;  // log_format.rs:63
constexpr uint32_t kPipeHeader = 7;         // log_format.rs:66
constexpr uint32_t kPipeMaxBlocks = 1024;   // blocks per workgroup (the LDS block tables)
constexpr uint32_t kPipeCache = 64;         // headers per block in the global header cache
constexpr uint32_t kPipeAMin = LVK_PIPE_AMIN;  // phase A: first records of units >= this (class 2: > 2 KiB)

// Region B carve-out (word offsets into g_lds).
constexpr uint32_t kPB = kRegionB / 4;
constexpr uint32_t kPCnt = kPB;                          // records per block
constexpr uint32_t kPPre = kPCnt + kPipeMaxBlocks;       // exclusive prefix of kPCnt
constexpr uint32_t kPRecA = kPPre + kPipeMaxBlocks;      // first record: len | type << 16 | status << 24, ~0 none
constexpr uint32_t kPCrcA = kPRecA + kPipeMaxBlocks;     // phase-A CRCs by block
constexpr uint32_t kPSortA = kPCrcA + kPipeMaxBlocks;    // phase-A list: block indices, longest first
constexpr uint32_t kPHist = kPSortA + kPipeMaxBlocks;    // phase-B key counts, then cursors
constexpr uint32_t kPHistA = kPHist + kKeys;             // phase-A bucket counts, then cursors
constexpr uint32_t kPCtl = kPHistA + 64;                 // control words (below)
constexpr uint32_t kPStage = kPCtl + 64;                 // CRCs by local record index
constexpr uint32_t kPStageN = kPB + 16384 - kPStage;     // records whose CRC is staged (10,880)
enum : uint32_t {
    kCPoolA,    // round counters of the four lists
    kCPool16,
    kCPool4,
    kCPool1,
    kCNA,       // phase-A entries
    kCN16,      // phase-B entries per group size
    kCN4,
    kCN1,
    kCReady,    // phase-B list written (ent[], hdr_off, info)
    kCAbort,    // write nothing: the records exceed cap, or a count never arrived
    kCFramed,   // framer waves done
    kCBaseLo,   // this workgroup's first record in log order
    kCBaseHi,
    kCCount,    // this workgroup's records
    kCDense,    // the phase-B list is in ent[base, ...) (more records than the local slice holds)
};
static_assert(kPStage + kPStageN == kPB + 16384, "carve-out fits region B");

struct WalPipe {
    const uint8_t *log;
    uint64_t size, nblocks;
    uint64_t *gran;  // one {tag 1 | count} granule per workgroup, then the retire counter (zero at launch)
    uint64_t *hc;    // header cache: kPipeCache per block (pos | len << 16 | type << 32)
    uint4 *ent;      // a dense workgroup's phase-B entries (8 B each) from its base on
    uint64_t *lst;   // phase-B entries of the other workgroups: kPipeCache per block of each
    uint64_t *hdr_off;
    uint32_t *crc, *info;
    uint64_t *count;
    uint64_t cap;
    uint32_t *err;  // set when a workgroup's count never arrived (bounded poll)
    uint64_t *trace;  // LVK_WAL_PIPE_TRACE: kPipeTrace s_memrealtime stamps per workgroup
};

// Timing variant (LVK_WAL_PIPE_TRACE): stamps of the phases per workgroup.
constexpr uint32_t kPipeTrace = 64;
#if LVK_WAL_PIPE_TRACE
#define PTRACE(slot)                                                                                   \
    do {                                                                                               \
        if ((threadIdx.x & 63u) == 0) a.trace[blockIdx.x * kPipeTrace + (slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define PTRACE(slot) \
    do {             \
    } while (0)
#endif

__device__ __forceinline__ uint32_t &pctl(uint32_t k) { return g_lds[kPCtl + k]; }

// Phase A: the sorted first records, geometry from LDS (no memory load).
struct PipeFirst {
    static constexpr uint32_t kFlush = 16;
    static constexpr bool kAlMid = true;
    static constexpr bool kOneRound = false;
    static constexpr uint32_t kExact = LVK_WALK_EXACT;
    static constexpr bool kPlainMerge = true;  // region B is the carve-out
    uint64_t blk0;  // address of the workgroup's first block
    __device__ __forceinline__ RGeo load(const Params &P, uint64_t e) const {
        const bool valid = e < P.n;
        const uint32_t i = static_cast<uint32_t>(valid ? e : P.n - 1);
        const uint32_t bl = g_lds[kPSortA + i];
        const uint32_t r = g_lds[kPRecA + bl];
        RGeo q;
        q.a = blk0 + static_cast<uint64_t>(bl) * kPipeBlockSize + 6u;  // [type || payload], log_reader.rs:336
        q.len = (r & 0xffffu) + 1u;
        q.seed = 0;
        q.bid = valid ? bl : 0xffffffffu;
        q.aux = 0;
        return q;
    }
    __device__ __forceinline__ uint2 trailer(const RGeo &, uint32_t) const { return make_uint2(0, 0); }
    __device__ __forceinline__ void stage(const Params &, uint32_t, uint32_t, const RGeo &q, uint32_t X,
                                          uint2) const {
        if (q.bid != 0xffffffffu) g_lds[kPCrcA + q.bid] = ~X;
    }
    __device__ __forceinline__ void flush(const Params &, uint32_t, uint32_t, uint32_t) const {}
};

// Phase B: the workgroup's sorted rest.  An entry is 8 bytes: record index
// (23 bits) | unit length << 23 (15 bits) | the unit's offset from the
// workgroup's first block << 38 -- in the workgroup's slice of the workspace
// (written by its own builder wave: same CU, loaded after an LDS flag), or
// for a dense workgroup in ent[base, ...).  CRCs by record index: the LDS
// staging, or (a dense workgroup's records past it) straight to the output
// in the flush, every kFlush rounds like the class kernel's stores.
struct PipeRest {
    static constexpr uint32_t kFlush = 16;
    static constexpr bool kAlMid = true;
    static constexpr bool kOneRound = false;
    static constexpr uint32_t kExact = LVK_WALK_EXACT;
    static constexpr bool kPlainMerge = true;
    const uint64_t *lst;
    uint64_t blk0;  // address of the workgroup's first block
    uint32_t *crc;  // a dense workgroup: d_crc + its base
    __device__ __forceinline__ RGeo load(const Params &P, uint64_t e) const {
        const bool valid = e < P.n;
        const uint64_t ec = valid ? e : P.n - 1;
        const uint64_t v = lst[ec];
        RGeo q;
        q.len = static_cast<uint32_t>(v >> 23) & 0x7fffu;
        q.a = blk0 + (q.len ? (v >> 38) : 0u);
        q.seed = 0;
        q.bid = valid ? static_cast<uint32_t>(v) & 0x7fffffu : 0xffffffffu;
        q.aux = 0;
        return q;
    }
    __device__ __forceinline__ uint2 trailer(const RGeo &, uint32_t) const { return make_uint2(0, 0); }
    __device__ __forceinline__ void stage(const Params &, uint32_t wave, uint32_t slot, const RGeo &q, uint32_t X,
                                          uint2) const {
        g_oidx[wave][slot] = q.bid;
        g_ocrc[wave][slot] = ~X;
    }
    __device__ __forceinline__ void flush(const Params &, uint32_t wave, uint32_t lane, uint32_t nslots) const {
        const uint32_t li = g_oidx[wave][lane], c = g_ocrc[wave][lane];
        if (lane >= nslots || li == 0xffffffffu) return;
        if (li < kPStageN)
            g_lds[kPStage + li] = c;
        else
            crc[li] = c;
    }
};

// The rest of a long chain through L2: one dword of every 128-B line of the
// rest of each block still being walked, four blocks per round trip (wal_hist's
// touch, wal_scan.hip: the bench log's longest chain is 54 records).
constexpr uint32_t kPipeTouchHops = 16;
__device__ __forceinline__ uint32_t pipe_touch(const uint8_t *blk, uint32_t pos, uint32_t blen, bool active,
                                               uint32_t lane) {
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
            const uint64_t b = __shfl(reinterpret_cast<uint64_t>(blk), l0);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t o = (p0 & ~127u) + 128u * (lane + 64u * k);
                v[g][k] = o < bl ? *reinterpret_cast<const uint32_t *>(b + o) : 0u;
            }
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) x ^= xor3(v[g][0], v[g][1], v[g][2]) ^ v[g][3];
    }
    return x;
}

// Region A and the combine tables of the G = 16 image (region B stays the
// carve-out): every thread issues its loads before its first LDS store.
__device__ __forceinline__ void stage_tables_ab(const uint4 *__restrict__ image) {
    constexpr int kA = kRegionB / 16, kC0 = kComb / 16, kC = (kImageWords * 4 - kComb) / 16;  // uint4 counts
    constexpr int kN = kA + kC;
    constexpr int kPer = (kN + kThreads - 1) / kThreads;
    uint4 *l4 = reinterpret_cast<uint4 *>(g_lds);
    g_u32x4 *src = reinterpret_cast<g_u32x4 *>(reinterpret_cast<uint64_t>(image));
    u32x4 r[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = threadIdx.x + k * kThreads;
        const int s = i < kA ? i : kC0 + (i - kA);
        if (i < kN) r[k] = src[s];
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int i = threadIdx.x + k * kThreads;
        const int s = i < kA ? i : kC0 + (i - kA);
        if (i < kN) l4[s] = to_uint4(r[k]);
    }
}

// A record header at in-block position pos: status and unit length
// (log_reader.rs:305-331).
__device__ __forceinline__ uint32_t pipe_status(uint32_t len, uint32_t type, uint32_t blen, uint32_t pos) {
    if (kPipeHeader + len > blen - pos) return LV_WAL_REC_BAD_LENGTH;  // log_reader.rs:312-324
    if (type == 0 && len == 0) return LV_WAL_REC_ZERO;                 // log_reader.rs:326-331
    return LV_WAL_REC_OK;
}

// Sort-key walk order: class 2 (longest first), class 1, class 0, then the
// (empty: units <= 32,762 B) class 3.
__device__ __forceinline__ uint32_t pipe_order_key(uint32_t o) {
    return o < 64u ? 128u + o : o < 128u ? o : o < 192u ? o - 128u : o;
}

__global__ __launch_bounds__(kThreads) void wal_pipe_kernel(WalPipe a, const uint4 *__restrict__ image) {
    const uint32_t t = threadIdx.x, lane = t & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const uint32_t grid = gridDim.x, w = blockIdx.x;
    const uint64_t lo = a.nblocks * w / grid, hi = a.nblocks * (w + 1) / grid;
    const uint32_t nblk = static_cast<uint32_t>(hi - lo);  // <= kPipeMaxBlocks (host)
    const uint64_t blk0 = reinterpret_cast<uint64_t>(a.log) + lo * kPipeBlockSize;
    const uint8_t *const log = a.log;
    if (wave == 0) PTRACE(0);

    // ---- 1. the first header of every block (under the table staging) ----
    uint32_t w1 = 0, blen1 = 0;
    if (t < nblk) {
        const uint64_t start = (lo + t) * kPipeBlockSize;
        blen1 = static_cast<uint32_t>(a.size - start < kPipeBlockSize ? a.size - start : kPipeBlockSize);
        // header bytes 4..6 (length, type) in the aligned dword at +4 (an
        // aligned dword never crosses a page: its 4th byte may lie past a
        // 7-byte last block)
        if (blen1 >= kPipeHeader) w1 = *reinterpret_cast<const uint32_t *>(log + start + 4);
    }
    for (uint32_t k = t; k < kKeys + 64 + 64; k += kThreads) g_lds[kPHist + k] = 0;  // hist, histA, ctl
    stage_tables_ab(image);
    __syncthreads();
    if (t < nblk) {
        uint32_t r = 0xffffffffu;
        if (blen1 >= kPipeHeader) {
            const uint32_t len = w1 & 0xffffu, type = (w1 >> 16) & 0xffu;
            const uint32_t st = pipe_status(len, type, blen1, 0);
            r = len | (type << 16) | (st << 24);
            const uint32_t ulen = st == LV_WAL_REC_OK ? len + 1u : 0u;
            if (ulen >= kPipeAMin)
                atomicAdd(&g_lds[kPHistA + (sort_key(ulen) & 63u)], 1u);
            else
                atomicAdd(&g_lds[kPHist + sort_key(ulen)], 1u);
        }
        g_lds[kPRecA + t] = r;
    }
    __syncthreads();
    if (wave == 0) {  // bucket starts of phase A (64 buckets, longest first)
        const uint32_t c = g_lds[kPHistA + lane];
        uint32_t inc = c;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t x = __shfl_up(inc, d);
            if (lane >= d) inc += x;
        }
        g_lds[kPHistA + lane] = inc - c;
        if (lane == 63) pctl(kCNA) = inc;
    }
    __syncthreads();
    if (t < nblk) {
        const uint32_t r = g_lds[kPRecA + t];
        if (r != 0xffffffffu && (r >> 24) == LV_WAL_REC_OK && (r & 0xffffu) + 1u >= kPipeAMin) {
            const uint32_t slot = atomicAdd(&g_lds[kPHistA + (sort_key((r & 0xffffu) + 1u) & 63u)], 1u);
            g_lds[kPSortA + slot] = t;
        }
    }
    __syncthreads();
    if (wave == 0) PTRACE(1);
    // (values read from LDS are wave-uniform: readfirstlane keeps them in
    // scalar registers, where the walk's list bounds and pointers belong)
    auto uni = [](uint32_t v) { return __builtin_amdgcn_readfirstlane(v); };
    const uint32_t nA = uni(pctl(kCNA));
    const Lut L = make_lut(lane);
    auto pool = [&](uint32_t word) {
        uint32_t k = 0;
        if (lane == 0) k = atomicAdd(&g_lds[kPCtl + word], 1u);
        return static_cast<uint64_t>(__shfl(k, 0));
    };
    auto nextA = [&]() { return pool(kCPoolA); };
    auto walk_first = [&]() {
        Params P{};
        P.n = nA;
        sorted_stream<16, PipeFirst, decltype(nextA), 4>(P, PipeFirst{blk0}, lane, L, nextA(), nextA);  // (plain merge: 4 rows)
    };

    // ---- 2. framer waves: the rest of every chain; the others: phase A ----
    const uint32_t nframers = nblk > 64u ? 2u : 1u;
    if (wave < nframers) {
        const uint32_t fl = wave * 64u + lane;
        uint32_t touched = 0;
        for (uint32_t b0 = 0; b0 < nblk; b0 += 64u * nframers) {  // wave-uniform
            const uint32_t bl = b0 + fl;
            const uint64_t start = (lo + bl) * kPipeBlockSize;
            uint32_t blen = 0, pos = 0, cnt = 0, hops = 0;
            bool active = false;
            if (bl < nblk) {
                blen = static_cast<uint32_t>(a.size - start < kPipeBlockSize ? a.size - start : kPipeBlockSize);
                const uint32_t r = g_lds[kPRecA + bl];
                cnt = r == 0xffffffffu ? 0u : 1u;
                if (r != 0xffffffffu && (r >> 24) == LV_WAL_REC_OK) {
                    pos = kPipeHeader + (r & 0xffffu);
                    active = blen - pos >= kPipeHeader;
                }
            }
            // the header's length / type: the two aligned dwords around
            // bytes pos + 4 .. pos + 6 (the second clamped to the block's last)
            const uint8_t *const blk = log + start;
            const uint32_t lastd = blen ? (blen - 1u) & ~3u : 0u;
            uint32_t wlo = 0, whi = 0, wsh = 0;
            auto issue = [&](uint32_t p, bool on) {
                const uint32_t pr = p + 4u, ar = pr & ~3u;
                wsh = pr & 3u;
                if (on) {
                    wlo = *reinterpret_cast<const uint32_t *>(blk + ar);
                    whi = *reinterpret_cast<const uint32_t *>(blk + (ar + 4u < lastd ? ar + 4u : lastd));
                }
            };
            issue(pos, active);
            while (__any(active)) {  // wave-uniform: the longest chain of the wave
                // after kPipeTouchHops hops, the rest of each block still being
                // walked is touched into L2 (one dword per 128-B line, four
                // blocks per round trip), so the rest of a long chain of short
                // records hops through L2 instead of HBM (as wal_hist does)
                if (hops++ == kPipeTouchHops) touched ^= pipe_touch(blk, pos, blen, active, lane);
                const uint32_t hw = __builtin_amdgcn_alignbyte(whi, wlo, wsh);  // bytes pos + 4 .. pos + 7
                const uint32_t len = hw & 0xffffu, type = (hw >> 16) & 0xffu;
                const bool ok = kPipeHeader + len <= blen - pos && (type | len) != 0u;
                const uint32_t npos = pos + kPipeHeader + len;
                const bool nact = active && ok && blen - npos >= kPipeHeader;
                issue(npos, nact);  // the next header's loads before this record's store
                if (active) {
                    if (cnt < kPipeCache)
                        a.hc[(lo + bl) * kPipeCache + cnt] =
                            pos | (static_cast<uint64_t>(len) << 16) | (static_cast<uint64_t>(type) << 32);
                    __hip_atomic_fetch_add(&g_lds[kPHist + sort_key(ok ? len + 1u : 0u)], 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                    ++cnt;
                }
                pos = npos;
                active = nact;
            }
            if (bl < nblk) g_lds[kPCnt + bl] = cnt;
        }
        asm volatile("" ::"v"(touched));  // the touches are kept
        // the header cache and this wave's LDS writes are complete before the
        // count that elects the builder
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        PTRACE(2 + wave);
        uint32_t done = 0;
        if (lane == 0)
            done = __hip_atomic_fetch_add(&pctl(kCFramed), 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
        done = __shfl(done, 0);
        if (done + 1u == nframers) {
            // ---- 3. the builder ----
            uint32_t run = 0;
            for (uint32_t b0 = 0; b0 < nblk; b0 += 64u) {  // exclusive prefix of the block counts
                const uint32_t bl = b0 + lane;
                const uint32_t c = bl < nblk ? g_lds[kPCnt + bl] : 0u;
                uint32_t inc = c;
#pragma unroll
                for (uint32_t d = 1; d < 64; d <<= 1) {
                    const uint32_t x = __shfl_up(inc, d);
                    if (lane >= d) inc += x;
                }
                if (bl < nblk) g_lds[kPPre + bl] = run + inc - c;
                run += __shfl(inc, 63);
            }
            const uint32_t count_w = run;
            PTRACE(4);
            // (global address space: an agent-scope sc1 store / load, never flat)
            typedef __attribute__((address_space(1))) uint64_t gu64;
            gu64 *const gran = reinterpret_cast<gu64 *>(reinterpret_cast<uint64_t>(a.gran));
            if (lane == 0) __hip_atomic_store(gran + w, (1ull << 32) | count_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // phase-B key starts in walk order (class 2, 1, 0); lanes 0-15
            // hold class 2, 16-31 class 1, 32-47 class 0 (48-63: class 3, empty)
            {
                uint32_t c4[4], inc4 = 0;
#pragma unroll
                for (uint32_t i = 0; i < 4; ++i) {
                    c4[i] = g_lds[kPHist + pipe_order_key(4u * lane + i)];
                    inc4 += c4[i];
                }
                uint32_t inc = inc4;
#pragma unroll
                for (uint32_t d = 1; d < 64; d <<= 1) {
                    const uint32_t x = __shfl_up(inc, d);
                    if (lane >= d) inc += x;
                }
                uint32_t s = inc - inc4;
#pragma unroll
                for (uint32_t i = 0; i < 4; ++i) {
                    g_lds[kPHist + pipe_order_key(4u * lane + i)] = s;
                    s += c4[i];
                }
                const uint32_t e16 = __shfl(inc, 15), e4 = __shfl(inc, 31), e1 = __shfl(inc, 47);
                if (lane == 0) {
                    pctl(kCN16) = e16;  // (class 3 is empty: a unit is at most 32,762 B)
                    pctl(kCN4) = e4 - e16;
                    pctl(kCN1) = e1 - e4;
                    pctl(kCCount) = count_w;
                }
            }
            // Every record of the workgroup in log order: record q is record
            // k = q - pre[bl] of the last block bl with pre[bl] <= q.  LIST:
            // its phase-B entry (claimed slot); OUT: hdr_off / info at base.
            // Blocks of more than kPipeCache records walk on from the last
            // cached header (one lane per block; rare: a 32 KiB block holds
            // more than 64 records only when they are a few bytes long).
            const uint64_t lb = lo * kPipeBlockSize;
            auto emit = [&](uint64_t *list, uint64_t *hdr, uint32_t *info) {
                auto one = [&](uint32_t q, uint32_t bl, uint32_t pos, uint32_t len, uint32_t type, uint32_t blen,
                               bool rec, bool inb) {
                    const uint32_t st = pipe_status(len, type, blen, pos);
                    const uint32_t ulen = st == LV_WAL_REC_OK ? len + 1u : 0u;
                    const uint32_t slot = list ? wave_claim(&g_lds[kPHist], sort_key(ulen), rec && inb, lane) : 0u;
                    if (rec && hdr) {
                        hdr[q] = lb + static_cast<uint64_t>(bl) * kPipeBlockSize + pos;
                        info[q] = type | (st << 8) | (len << 16);
                    }
                    if (rec && inb && list) {
                        const uint64_t ua = static_cast<uint64_t>(bl) * kPipeBlockSize + pos + 6u;  // [type || payload]
                        list[slot] = q | (static_cast<uint64_t>(ulen) << 23) | (ua << 38);
                    }
                    return st;
                };
                // record q's block (binary search of the prefix) and its
                // cached header, requested one round of 64 records ahead so
                // the header cache's round trip overlaps the previous round
                struct Loc {
                    uint32_t q, bl, k;
                    uint64_t h;
                };
                auto locate = [&](uint32_t q0) {
                    Loc x;
                    x.q = q0 + lane;
                    x.bl = 0;
                    for (uint32_t step = kPipeMaxBlocks / 2; step >= 1; step >>= 1)
                        if (x.bl + step < nblk && g_lds[kPPre + x.bl + step] <= x.q) x.bl += step;
                    x.k = x.q - g_lds[kPPre + x.bl];
                    x.h = x.q < count_w && x.k - 1u < kPipeCache - 1u ? a.hc[(lo + x.bl) * kPipeCache + x.k] : 0ull;
                    return x;
                };
                Loc cur = locate(0);
                for (uint32_t q0 = 0; q0 < count_w; q0 += 64u) {  // wave-uniform
                    const Loc nx = q0 + 64u < count_w ? locate(q0 + 64u) : cur;  // wave-uniform choice
                    const uint32_t q = cur.q, bl = cur.bl, k = cur.k;
                    const bool rec = q < count_w && k < kPipeCache;
                    const uint64_t start = lb + static_cast<uint64_t>(bl) * kPipeBlockSize;
                    const uint32_t blen =
                        static_cast<uint32_t>(a.size - start < kPipeBlockSize ? a.size - start : kPipeBlockSize);
                    uint32_t pos = 0, len = 0, type = 0;
                    if (rec) {
                        if (k == 0) {
                            const uint32_t r = g_lds[kPRecA + bl];
                            len = r & 0xffffu;
                            type = (r >> 16) & 0xffu;
                        } else {
                            pos = static_cast<uint32_t>(cur.h) & 0xffffu;
                            len = static_cast<uint32_t>(cur.h >> 16) & 0xffffu;
                            type = static_cast<uint32_t>(cur.h >> 32) & 0xffu;
                        }
                    }
                    const bool firstA = k == 0 && pipe_status(len, type, blen, 0) == LV_WAL_REC_OK &&
                                        len + 1u >= kPipeAMin;  // phase A walked it
                    one(q, bl, pos, len, type, blen, rec, !firstA);
                    cur = nx;
                }
                for (uint32_t b0 = 0; b0 < nblk; b0 += 64u) {  // wave-uniform
                    const uint32_t bl = b0 + lane;
                    const uint32_t c = bl < nblk ? g_lds[kPCnt + bl] : 0u;
                    bool active = c > kPipeCache;
                    const uint64_t start = lb + static_cast<uint64_t>(bl) * kPipeBlockSize;
                    const uint32_t blen =
                        active ? static_cast<uint32_t>(a.size - start < kPipeBlockSize ? a.size - start : kPipeBlockSize)
                               : 0u;
                    uint32_t pos = 0, q = 0;
                    if (active) {
                        const uint64_t h = a.hc[(lo + bl) * kPipeCache + kPipeCache - 1];
                        pos = (static_cast<uint32_t>(h) & 0xffffu) + kPipeHeader + (static_cast<uint32_t>(h >> 16) & 0xffffu);
                        q = g_lds[kPPre + bl] + kPipeCache;
                    }
                    while (__any(active)) {
                        uint32_t len = 0, type = 0;
                        if (active) {
                            const uint64_t hb = start + pos + 4u;
                            len = static_cast<uint32_t>(log[hb]) | (static_cast<uint32_t>(log[hb + 1]) << 8);
                            type = log[hb + 2];
                        }
                        const uint32_t st = one(q, bl, pos, len, type, blen, active, true);
                        if (active) {
                            ++q;
                            pos += kPipeHeader + len;
                            active = st == LV_WAL_REC_OK && blen - pos >= kPipeHeader;
                        }
                    }
                }
            };
            auto ready = [&]() {  // the list is in memory before the flag (same CU: walkers load after it)
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                if (lane == 0) __hip_atomic_store(&pctl(kCReady), 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                PTRACE(6);
            };
            // Every workgroup's count (bounded poll, ~0.2 s of s_memrealtime
            // at 100 MHz): this one's base in the log-order output and the
            // total for the capacity check.
            uint64_t base = 0, total = 0;
            bool timeout = false;
            auto lookback = [&]() {
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                for (uint32_t j0 = 0; j0 < grid; j0 += 64u) {  // wave-uniform
                    const uint32_t j = j0 + lane;
                    uint64_t v = 0;
                    for (;;) {
                        if (j < grid) v = __hip_atomic_load(gran + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (__all(j >= grid || (v >> 32) == 1u)) break;
                        if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {
                            timeout = true;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(8);
                    }
                    const uint64_t c = j < grid ? (v & 0xffffffffull) : 0u;
                    base += j < w ? c : 0u;
                    total += c;
                }
#pragma unroll
                for (int k = 32; k >= 1; k >>= 1) {
                    base += __shfl_xor(base, k);
                    total += __shfl_xor(total, k);
                }
                PTRACE(5);
                // retire: every granule has been read; the last workgroup to
                // get here clears them (and the counter) for the stream's next
                // launch -- each workgroup published before it retired
                uint64_t d = 0;
                if (lane == 0)
                    d = __hip_atomic_fetch_add(gran + 1024, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
                if (__shfl(d, 0) + 1u == grid) {  // wave-uniform
                    for (uint32_t j = lane; j < grid; j += 64u)
                        __hip_atomic_store(gran + j, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (lane == 0) __hip_atomic_store(gran + 1024, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                const bool abort = timeout || total > a.cap;
                if (w == 0 && lane == 0) *a.count = timeout ? ~0ull : total;
                if (timeout && lane == 0) atomicOr(a.err, 1u);
                if (lane == 0) {
                    pctl(kCBaseLo) = static_cast<uint32_t>(base);
                    pctl(kCBaseHi) = static_cast<uint32_t>(base >> 32);
                    pctl(kCAbort) = abort ? 1u : 0u;
                }
                return abort;
            };
            const bool local = count_w <= kPStageN && count_w <= kPipeCache * nblk;
            if (local) {
                // the list in this workgroup's slice of the workspace: ready
                // as soon as the framing is done, before any other workgroup's
                // count is known
                emit(a.lst + lo * kPipeCache, nullptr, nullptr);
                ready();
                if (!lookback()) emit(nullptr, a.hdr_off + base, a.info + base);
            } else {
                // a dense workgroup: the list goes to ent[base, ...) (at most
                // cap entries in all), so it waits for the base
                if (!lookback())
                    emit(reinterpret_cast<uint64_t *>(a.ent) + base, a.hdr_off + base, a.info + base);
                else if (lane == 0)
                    pctl(kCN16) = pctl(kCN4) = pctl(kCN1) = 0u;
                if (lane == 0) pctl(kCDense) = 1u;
                ready();
            }
        }
    }

    // ---- 4. every wave: phase A, then (after the flag) the phase-B lists ----
    walk_first();
    PTRACE(8 + wave);
    while (__hip_atomic_load(&pctl(kCReady), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
        __builtin_amdgcn_s_sleep(16);
    PTRACE(24 + wave);
    {
        const bool dense = uni(pctl(kCDense)) != 0u;
        const uint32_t n16 = uni(pctl(kCN16)), n4 = uni(pctl(kCN4)), n1 = uni(pctl(kCN1));
        const uint64_t base = dense ? (static_cast<uint64_t>(uni(pctl(kCBaseHi))) << 32) | uni(pctl(kCBaseLo)) : 0u;
        const uint64_t *const lst = dense ? reinterpret_cast<const uint64_t *>(a.ent) + base : a.lst + lo * kPipeCache;
        uint32_t *const crcd = a.crc + base;  // dense: records past the LDS staging go straight out
        const PipeRest r16{lst, blk0, crcd};
        const PipeRest r4{lst + n16, blk0, crcd};
        const PipeRest r1{lst + n16 + n4, blk0, crcd};
        Params P{};
        auto next16 = [&]() { return pool(kCPool16); };
        auto next4 = [&]() { return pool(kCPool4); };
        auto next1 = [&]() { return pool(kCPool1); };
        if constexpr (LVK_PIPE_B_SMALL_FIRST) {  // classes 1, 0, then 2 (longest first: the round ends short)
            P.n = n4;
            sorted_stream<4>(P, r4, lane, L, next4(), next4);
            P.n = n1;
            sorted_stream<1>(P, r1, lane, L, next1(), next1);
            P.n = n16;
            sorted_stream<16, PipeRest, decltype(next16), 4>(P, r16, lane, L, next16(), next16);
        } else {
            P.n = n16;
            sorted_stream<16, PipeRest, decltype(next16), 4>(P, r16, lane, L, next16(), next16);
            P.n = n4;
            sorted_stream<4>(P, r4, lane, L, next4(), next4);
            P.n = n1;
            sorted_stream<1>(P, r1, lane, L, next1(), next1);
        }
    }
    PTRACE(40 + wave);
    __syncthreads();
    if (uni(pctl(kCAbort))) return;
    // ---- 5. the workgroup's CRCs in log order ----
    const uint64_t base = (static_cast<uint64_t>(uni(pctl(kCBaseHi))) << 32) | uni(pctl(kCBaseLo));
    const uint32_t count_w = uni(pctl(kCCount));
    uint32_t *const crc = a.crc + base;
    for (uint32_t bl = t; bl < nblk; bl += kThreads) {  // phase A's CRCs to their record index
        const uint32_t r = g_lds[kPRecA + bl];
        if (r != 0xffffffffu && (r >> 24) == LV_WAL_REC_OK && (r & 0xffffu) + 1u >= kPipeAMin) {
            const uint32_t li = g_lds[kPPre + bl];
            if (li < kPStageN)
                g_lds[kPStage + li] = g_lds[kPCrcA + bl];
            else
                crc[li] = g_lds[kPCrcA + bl];
        }
    }
    __syncthreads();
    const uint32_t ns = count_w < kPStageN ? count_w : kPStageN;
    for (uint32_t i = t; i < ns; i += kThreads) crc[i] = g_lds[kPStage + i];
    if (wave == 0) PTRACE(56);
}

}  // namespace lvk

namespace lvh {

// The one-launch scan's workspace: an error word, the header cache, the
// phase-B entries (the count granules are the stream's, stream_gran).
struct PipeWs {
    size_t hc, lst, ent, err, total;
};

static PipeWs pipe_ws_layout(uint64_t nblocks, uint64_t cap) {
    PipeWs w;
    w.err = 0;
    // (LVK_WAL_PIPE_TRACE: the stamps right after the error word, at byte 16
    // of the workspace: tools/wal_pipe_trace.py reads them there)
    w.hc = w.err + 16 + (LVK_WAL_PIPE_TRACE ? 1024 * lvk::kPipeTrace * sizeof(uint64_t) : 0);
    w.lst = w.hc + al16(nblocks * lvk::kPipeCache * sizeof(uint64_t));
    w.ent = w.lst + al16(nblocks * lvk::kPipeCache * sizeof(uint64_t));
    w.total = w.ent + al16(cap * sizeof(uint64_t));
    return w;
}

size_t wal_pipe_ws_bytes(uint64_t bytes, uint64_t cap) {
    const uint64_t nblocks = (bytes + lvk::kPipeBlockSize - 1) / lvk::kPipeBlockSize;
    return pipe_ws_layout(nblocks, cap).total;
}

bool wal_pipe_applies(const DevCtx &c, uint64_t bytes) {
    const uint64_t nblocks = (bytes + lvk::kPipeBlockSize - 1) / lvk::kPipeBlockSize;
    const uint64_t grid = std::min<uint64_t>(static_cast<uint64_t>(c.cus), nblocks);
    return LVK_WAL_LOCAL && nblocks > 0 && grid <= 1024 && (nblocks + grid - 1) / grid <= lvk::kPipeMaxBlocks;
}

int launch_wal_pipe(DevCtx &c, const uint8_t *d_log, uint64_t bytes, uint64_t *d_hdr_off, uint32_t *d_crc,
                    uint32_t *d_info, uint64_t cap, uint64_t *d_count, uint8_t *ws, hipStream_t s) {
    const uint64_t nblocks = (bytes + lvk::kPipeBlockSize - 1) / lvk::kPipeBlockSize;
    const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>(static_cast<uint64_t>(c.cus), nblocks));
    const PipeWs lay = pipe_ws_layout(nblocks, cap);
    lvk::WalPipe a{};
    a.log = d_log;
    a.size = bytes;
    a.nblocks = nblocks;
    if (int rc = stream_gran(c, s, &a.gran)) return rc;
    a.hc = reinterpret_cast<uint64_t *>(ws + lay.hc);
    a.ent = reinterpret_cast<uint4 *>(ws + lay.ent);
    a.lst = reinterpret_cast<uint64_t *>(ws + lay.lst);
    a.hdr_off = d_hdr_off;
    a.crc = d_crc;
    a.info = d_info;
    a.count = d_count;
    a.cap = cap;
    a.err = reinterpret_cast<uint32_t *>(ws + lay.err);
    a.trace = LVK_WAL_PIPE_TRACE ? reinterpret_cast<uint64_t *>(ws + lay.err + 16) : nullptr;
    hipLaunchKernelGGL(lvk::wal_pipe_kernel, dim3(grid), dim3(lvk::kThreads), 0, s, a, c.image[2]);  // 4-row batches (merge_al<4, PLAIN>)
    return 0;
}

}  // namespace lvh
