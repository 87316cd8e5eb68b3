// SSTable block trailers on MI355X: seal (builder side)
// and verify (ReadOptions::verify_checksums, options.rs:84) of many blocks
// at once.  Each block's CRC unit is contents||type, contiguous in the file;
// one kernel launch (handles -> CRC walk of lvk/walk.h -> trailer epilogue).
// Trailer layout: see include/lvgpu/table.h.
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/lvgpu/crc32c.h"
#include "../../include/lvgpu/table.h"
#include "lv_internal.h"
#include "lvh.h"
#include "lvk/walk.h"

namespace lvk {

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

// File-order runs (round 6): a unit's first 256-B row is
// the previous unit's last one (blocks follow each other in the file, 4-5 B
// of trailer apart), and with one unit per group per round the two reads of
// that line came from different waves ~17 rows apart -- two HBM fetches
// (FETCH 1.061x the algorithmic bytes).  Now each group walks kSstRun
// consecutive blocks in successive rounds: a wave round rho = R k + i gives
// group g block R 4k + g k + i, so the edge line it needs first was loaded by
// the same group one batch earlier (an L2 hit), and only 1 of k edges is
// fetched twice.  k = 1 is the old order.
constexpr uint32_t kSstRun = LVK_SST_RUN;

__device__ __forceinline__ uint64_t sst_unit(uint64_t e) {  // e = rho * 4 + group
    const uint64_t rho = e >> 2, g = e & 3u;
    return (rho / kSstRun) * (4u * kSstRun) + g * kSstRun + rho % kSstRun;
}

template <bool SEAL, bool CRCOUT = false>
struct TableUnits {
    const uint2 *handles;  // {offset, size} u64 pairs per block
    const uint8_t *types;  // seal: per-block type byte (NULL: 0 = no compression)
    uint32_t *status;      // verify: LV_SST_BLOCK_* per block
    uint32_t *crc_out;     // verify: optional crc32c(contents || type)
    uint64_t file_bytes;
    uint64_t nblocks;      // the blocks (P.n: the run-padded entry count)
    // seal: 64 slots of {block, masked crc} (16 rounds of 4 blocks per flush;
    // the trailer stores are partial-line writes, and fewer, larger bursts of
    // them measured faster); verify: 64 slots of {block, status}, or with
    // crc_out 32 slots of four words
    static constexpr uint32_t kFlush = SEAL ? LVK_SEAL_FLUSH : !CRCOUT ? 16 : 8;
    static constexpr bool kAlMid = false;  // measured -0.7 % here (load_rbatch_al)
    static constexpr bool kOneRound = false;
    // Wait-count mode (walk.h sorted_stream): verify runs mode 2 (every load
    // unconditional within its path: 0.703 -> 0.723 against the session-start
    // build, profiles/r04/final_ab/), the seal keeps the masked loads (mode
    // 2: 0.667 -> 0.639, and with its trailer stores unconditional too 0.667
    // -> 0.640, seal_exact/; mode 1, the tail and trailer re-read every step:
    // seal 0.67 -> 0.61, verify 0.69 -> 0.64; mode2_ab/, exact_ab/)
    static constexpr uint32_t kExact = SEAL ? 0u : 2u;

    __device__ __forceinline__ RGeo load(const Params &P, uint64_t e) const {
        const uint64_t u = sst_unit(e);
        const bool valid = u < nblocks;
        const uint64_t ec = valid ? u : nblocks - 1;
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
        if constexpr (kExact != 0) {
            if (SEAL && types) t = ok ? types[ec] : 0u;  // every lane loads (ec is clamped)
        } else if (SEAL && types && ok) {
            t = types[ec];
        }
        q.aux = (ok ? 1u : 0u) | (t << 8);
        return q;
    }
    // verify: the stored masked crc at the unit's end (two aligned dwords)
    __device__ __forceinline__ uint2 trailer(const RGeo &q, uint32_t gl) const {
        if (SEAL) return make_uint2(0, 0);
        if constexpr (kExact != 0) {  // every lane loads two dwords (others: the zero block)
            const bool on = gl == 0 && (q.aux & 1u);
            const uint64_t end = q.a + q.len;
            const uint32_t *w = on ? reinterpret_cast<const uint32_t *>(end & ~static_cast<uint64_t>(3))
                                   : reinterpret_cast<const uint32_t *>(&g_zero_granules[0]);
            const uint32_t w0 = w[0], w1 = w[(end & 3u) ? 1 : 0];  // (aligned: no dword past the stored crc)
            return on ? make_uint2(w0, (end & 3u) ? w1 : 0u) : make_uint2(0, 0);
        }
        if (gl != 0 || !(q.aux & 1u)) return make_uint2(0, 0);
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
            if (bi == 0xffffffffu) return;
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


template <bool SEAL, bool CRCOUT>
__global__ __launch_bounds__(kThreads) void sst_blocks_kernel(Params P, const uint4 *__restrict__ image,
                                                              TableUnits<SEAL, CRCOUT> src) {
    stage_tables(image);
    if (threadIdx.x == 0) g_lds[kPoolWord] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const Lut L = make_lut(lane);
    const uint64_t grid = gridDim.x;
    // a wave claims kSstRun rounds at a time (its groups' runs of blocks)
    auto claim = [&]() -> uint64_t {
        uint32_t k = 0;
        if (lane == 0) k = atomicAdd(&g_lds[kPoolWord], 1u);
        return (blockIdx.x + grid * static_cast<uint64_t>(__shfl(k, 0))) * kSstRun;
    };
    uint64_t r0 = claim();
    uint32_t i = 0;
    auto next = [&]() -> uint64_t {
        if (++i == kSstRun) {
            i = 0;
            r0 = claim();
        }
        return r0 + i;
    };
    sorted_stream<16, TableUnits<SEAL, CRCOUT>, decltype(next), SEAL ? kSealRows : kSstRows>(P, src, lane, L, r0,
                                                                                          next);
}

// ---------------------------------------------------------------------------
// Continuous file-order walk (round 6).  The per-unit walk
// above starts every block on its own: its rows are padded to whole batches
// (17-19 rows of data in 18-21 rows), the wave runs the longest of its four
// blocks, and the merge and the tail fold run inside the loop, for every
// lane of the wave.  Here a 16-lane group streams one row (256 B on the
// absolute grid) per step over a run of consecutive blocks, in file order,
// with one Horner accumulator per lane (A = Shift_256(A) ^ R(0, granule));
// the blocks' boundaries only change what each lane's granule is masked to:
//  * unit j's whole granules (ending at or before its end b_j) fold into A;
//    a lane's first granule past them starts the next unit (A snapshotted
//    into S, then restarted) -- bytes before that unit's start are zeroed and
//    its first 4 bytes take the seed, as the per-unit head fix-up does;
//  * the granule holding unit j's last b_j & 15 bytes (and the stored CRC of
//    a verify) and the one after it are kept raw;
//  * once every lane has passed unit j (the row after its last whole
//    granule's row), the 16 snapshots and the two raw granules go to LDS.
// After the claim's rows, lane u of the wave finishes unit u of the claim
// alone: Horner over the 16 snapshots in lane order from the lane furthest
// from the end (X = Shift_16(X) ^ S_l), the tail fold, then the compare
// (verify) or the trailer (seal).  The per-unit merge and tail work thus runs
// once per unit on one lane instead of once per unit on every lane.
// Blocks are streamed together only when they follow each other (the next
// starts 0-64 B after this one's end, both >= 1 KiB: a lane then switches
// units at most once per row); any other block -- short, out of range,
// shuffled, overlapping -- is a stream of its own (its rows may be re-read).
// LDS: region A of the G = 4 image (T0..T3 and Shift_256, Latin), combine
// table 0 (Shift_16); region B holds the claim's unit states.
constexpr uint32_t kStreamRing = 8;                 // rows in flight per lane
constexpr uint32_t kClaimUnits = 4 * kSstRun;       // blocks per wave claim (group g: kSstRun of them)
constexpr int32_t kStreamMin = 1024;                // a chained block's minimum length (4 rows)
constexpr int32_t kStreamGap = 64;                  // ... and its largest gap to the block before it
constexpr int32_t kFar = 0x7f000000;                // start of "no next unit"
constexpr uint32_t kStateWords = 24;                // per unit: 16 snapshots, 2 raw granules
constexpr uint32_t kStatePerWave = kClaimUnits * kStateWords;
static_assert(kWaves * kStatePerWave * 4 <= 65536, "unit states fit region B");
static_assert(kSstRun == 4, "the run plan holds four blocks per group");

struct SstStream {
    uint64_t origin;  // the file's address rounded down to 256 B: positions below are origin-relative
    int32_t fbeg, fend;  // the file's bytes [fbeg, fend)
    const uint2 *handles;
    const uint8_t *types;
    uint32_t *status;
    uint32_t *crc_out;
    uint64_t file_bytes;
    uint64_t n;
};

template <bool SEAL, bool CRCOUT>
__global__ __launch_bounds__(kThreads) void sst_stream_kernel(SstStream a, const uint4 *__restrict__ image) {
    stage_words(g_lds, reinterpret_cast<const uint32_t *>(image), kRegionB / 16);
    stage_words(g_lds + kComb / 4, reinterpret_cast<const uint32_t *>(image) + kComb / 4, 256);
    if (threadIdx.x == 0) g_lds[kPoolWord] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, gl = lane & 15u, grp = lane >> 4;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const Lut L = make_lut(lane);
    uint32_t *const st = g_lds + kRegionB / 4 + wave * kStatePerWave;
    const uint64_t nclaims = (a.n + kClaimUnits - 1) / kClaimUnits;
    // Lane u < 16 finishes unit u of a claim whose walk is done (its states
    // in st): Horner over the 16 snapshots from the lane furthest from the
    // block's last whole granule, the tail fold, then the compare or trailer.
    auto finish = [&](uint64_t fum, bool fok, int32_t fua, int32_t fub) {
        __builtin_amdgcn_wave_barrier();
        if (lane < 16 && fum < a.n) {
            const uint32_t *su = st + lane * kStateWords;
            uint32_t crc = 0, stv = LV_SST_BLOCK_OUT_OF_RANGE;
            if (fok) {
                const int32_t ge = (fub >> 4) - 1;
                const uint32_t e = static_cast<uint32_t>(ge) & 15u;
                uint32_t X = 0;
#pragma unroll
                for (uint32_t t2 = 0; t2 < 16; ++t2) X = comb_shift(X, 0) ^ su[(e + 1u + t2) & 15u];
                const uint4 t1 = make_uint4(su[16], su[17], su[18], su[19]);
                RGeo g;
                g.a = a.origin + static_cast<uint32_t>(fua);
                g.len = static_cast<uint32_t>(fub - fua);
                g.seed = 0;
                g.bid = 0;
                g.aux = 0;
                X = finish_raw(g, X, t1, 0u, L);
                if constexpr (SEAL) {
                    const uint32_t ty = a.types ? a.types[fum] : 0u;
                    crc = mask_crc(~byte_step(X, ty));
                    uint8_t *p = reinterpret_cast<uint8_t *>(a.origin + static_cast<uint32_t>(fub));  // type, LE32(mask(crc))
                    p[0] = static_cast<uint8_t>(ty);
                    p[1] = static_cast<uint8_t>(crc);
                    p[2] = static_cast<uint8_t>(crc >> 8);
                    p[3] = static_cast<uint8_t>(crc >> 16);
                    p[4] = static_cast<uint8_t>(crc >> 24);
                } else {
                    crc = ~X;
                    const uint32_t k = static_cast<uint32_t>(fub) & 15u;  // the stored CRC: bytes k..k+3 of T1 || T2
                    const uint32_t w[8] = {su[16], su[17], su[18], su[19], su[20], su[21], su[22], su[23]};
                    const uint32_t d = k >> 2, sh = (k & 3u) * 8u;
                    uint32_t lo = 0, hi = 0;
#pragma unroll
                    for (uint32_t i = 0; i < 7; ++i)
                        if (i == d) {
                            lo = w[i];
                            hi = w[i + 1];
                        }
                    const uint32_t stored = sh ? (lo >> sh) | (hi << (32u - sh)) : lo;
                    const uint32_t r = stored - 0xa282ead8u;  // unmask, crc32c.rs:59-63
                    stv = ((r >> 17) | (r << 15)) == crc ? LV_SST_BLOCK_OK : LV_SST_BLOCK_CHECKSUM_MISMATCH;
                }
            }
            if constexpr (!SEAL) {
                a.status[fum] = stv;
                if (CRCOUT && a.crc_out) a.crc_out[fum] = fok ? crc : 0u;
            }
        }
        __builtin_amdgcn_wave_barrier();  // the states are read before the next walk writes them
    };
    // Claims are pipelined: the next claim's handles are requested when a walk
    // starts, and a claim's unit finish runs after the next claim's first rows
    // are requested, so neither round trip sits between two walks.
    auto take = [&]() -> uint64_t {
        uint32_t kc = 0;
        if (lane == 0) kc = atomicAdd(&g_lds[kPoolWord], 1u);
        return blockIdx.x + gridDim.x * static_cast<uint64_t>(__shfl(kc, 0));
    };
    // lane l < 16 loads block c * kClaimUnits + l (group l / 4, run position
    // l % 4); the others load a copy
    auto handles_of = [&](uint64_t c, uint2 &h0, uint2 &h1) {
        const uint64_t u = c * kClaimUnits + (lane & 15u), uc = u < a.n ? u : a.n - 1;
        h0 = a.handles[2 * uc];
        h1 = a.handles[2 * uc + 1];
    };
    uint64_t claim = take();
    if (claim >= nclaims) return;  // wave-uniform
    uint2 ho, hs, hon, hsn;
    handles_of(claim, ho, hs);
    uint64_t prv_um = 0;
    bool prv_ok = false, have_prv = false;
    int32_t prv_a = 0, prv_b = 0;
    for (;;) {
        const uint64_t u0 = claim * kClaimUnits;
        const uint64_t um = u0 + (lane & 15u);
        const uint64_t next = take();
        handles_of(next < nclaims ? next : claim, hon, hsn);
        const uint64_t o = (static_cast<uint64_t>(ho.y) << 32) | ho.x, sz = (static_cast<uint64_t>(hs.y) << 32) | hs.x;
        const bool uok = um < a.n && sst_in_range(o, sz, a.file_bytes);
        const int32_t ua = uok ? a.fbeg + static_cast<int32_t>(o) : 0;
        const int32_t ub = uok ? ua + static_cast<int32_t>(SEAL ? sz : sz + 1) : 0;
        // the group's run plan: unit i = lane grp * 4 + i
        int32_t pa[4], pb[4], pge[4], pst[4], pen[4];
        bool pch[5], pok[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int src = static_cast<int>(grp * 4u) + i;
            pa[i] = __shfl(ua, src);
            pb[i] = __shfl(ub, src);
            pok[i] = __shfl(uok ? 1 : 0, src) != 0;
            pge[i] = (pb[i] >> 4) - 1;  // last granule wholly inside the unit (ends <= b)
        }
        pch[0] = false;
        pch[4] = false;
#pragma unroll
        for (int i = 1; i < 4; ++i)
            pch[i] = pok[i - 1] && pok[i] && pb[i - 1] - pa[i - 1] >= kStreamMin && pb[i] - pa[i] >= kStreamMin &&
                     pa[i] >= pb[i - 1] + (SEAL ? 5 : 0) && pa[i] - pb[i - 1] <= kStreamGap;
        uint32_t total = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            // rows of unit i: from the row after the previous unit's last one
            // when chained, else from its own first row; to the row after its
            // last whole granule's row when the next one is chained (every
            // lane has then passed it), else to the row of granule ge + 2
            pst[i] = pch[i] ? pen[i > 0 ? i - 1 : 0] + 1 : pa[i] >> 8;
            pen[i] = pch[i + 1] ? (pge[i] >> 4) + 1 : (pge[i] + 2) >> 4;
            if (!pok[i]) pen[i] = pst[i] - 1;  // no rows
            total += static_cast<uint32_t>(pen[i] - pst[i] + 1);
        }
        const uint32_t steps = wave_max_u32(total, 16);
        uint32_t A = 0, S = 0;
        bool sw = false, h1 = false, h2 = false;
        uint4 T1 = make_uint4(0, 0, 0, 0), T2 = T1;
        // granule load of row r for this lane (zeros outside the file or past the plan)
        auto load_row = [&](int32_t r, bool on) -> uint4 {
            const int32_t q16 = r * 256 + static_cast<int32_t>(gl) * 16;
            const bool in = on && q16 + 16 > a.fbeg && q16 < a.fend;
            return load16(in ? a.origin + static_cast<uint32_t>(q16) : reinterpret_cast<uint64_t>(&g_zero_granules[gl]));
        };
        // The row step every path shares: fix-up, snapshot, fold, tail capture.
        // cA / cAn: starts of the current and next unit, cGe: the current unit's
        // last whole granule (all origin-relative), s0 / s0n their seed words.
        auto fold_row = [&](const uint4 &vr, int32_t row, int32_t cA, int32_t cAn, int32_t cGe, uint32_t s0,
                            uint32_t s0n, bool act) {
            const int32_t q = row * 16 + static_cast<int32_t>(gl);
            const bool onNext = q > cGe;
            uint4 v = vr;
            const int32_t at = onNext ? cAn : cA;
            if (__any(act && q * 16 < at + 4)) {  // bytes before a unit's start, or its first 4
                const int32_t rel = q * 16 - at;
                const uint32_t sd = onNext ? s0n : s0;
                v.x = fix_word(v.x, rel, sd);
                v.y = fix_word(v.y, rel + 4, sd);
                v.z = fix_word(v.z, rel + 8, sd);
                v.w = fix_word(v.w, rel + 12, sd);
            }
            const bool swn = onNext && !sw;  // this lane's first granule past the unit
            S = swn ? A : S;
            A = swn ? 0u : A;
            sw = sw || onNext;
            A = lookup4x<kRegionA + kHalf>(A, r0_granule(v, L), L);  // Shift_256(A) ^ R(0, v)
            if (__any(act && (q == cGe + 1 || q == cGe + 2))) {
                if (q == cGe + 1) {
                    T1 = vr;
                    h1 = true;
                }
                if (q == cGe + 2) {
                    T2 = vr;
                    h2 = true;
                }
            }
        };
        // unit slot k's state: the 16 snapshots and the raw granules
        auto emit = [&](uint32_t k) {
            uint32_t *su = st + (grp * 4u + k) * kStateWords;
            su[gl] = sw ? S : A;
            if (h1) {
                su[16] = T1.x;
                su[17] = T1.y;
                su[18] = T1.z;
                su[19] = T1.w;
            }
            if (h2) {
                su[20] = T2.x;
                su[21] = T2.y;
                su[22] = T2.z;
                su[23] = T2.w;
            }
            h1 = h2 = sw = false;
        };
        const int32_t rfirst = pa[0] >> 8, rlast = (pge[3] + 2) >> 4;
        if (__all(pok[0] && pch[1] && pch[2] && pch[3] && rfirst * 256 >= a.fbeg && (rlast + 1) * 256 <= a.fend)) {
            // Every group's four blocks follow each other (the bench's and a
            // table's layout) and its rows lie inside the file: one row range
            // per group, the units a queue, rows loaded unguarded.
            int32_t row = rfirst, prow = row;
            int32_t qa0 = pa[0], qa1 = pa[1], qa2 = pa[2], qa3 = pa[3];
            int32_t qg0 = pge[0], qg1 = pge[1], qg2 = pge[2], qg3 = pge[3];
            int32_t cEnd = (qg0 >> 4) + 1;
            uint32_t k = 0;
            const uint64_t zero = reinterpret_cast<uint64_t>(&g_zero_granules[gl]);
            uint64_t pp = a.origin + static_cast<uint32_t>(row * 256) + 16u * gl;  // row prow's granule
            uint4 ring[kStreamRing];
#pragma unroll
            for (uint32_t i = 0; i < kStreamRing; ++i, ++prow, pp += 256) ring[i] = load16(prow <= rlast ? pp : zero);
            if (have_prv) finish(prv_um, prv_ok, prv_a, prv_b);  // under the first rows' round trip
            // One row per step.  Every use of the slot's granule comes before
            // its one refill, so each ring slot keeps its registers (a refill
            // on two paths, or a copy of a slot past its refill, made the
            // compiler copy loads still in flight and wait for them all).
            auto fstep = [&](uint4 &slot) {
                const int32_t q = row * 16 + static_cast<int32_t>(gl);
                const bool onNext = q > qg0;  // past the current block's last whole granule
                const int32_t at = onNext ? qa1 : qa0;
                // the raw granules first, then the fix-up in place (the slot is
                // dead after its fold: no copy of it)
                if (__any(k < 4u && (q == qg0 + 1 || q == qg0 + 2))) {
                    if (q == qg0 + 1) {
                        T1 = slot;
                        h1 = true;
                    }
                    if (q == qg0 + 2) {
                        T2 = slot;
                        h2 = true;
                    }
                }
                if (__any(k < 4u && q * 16 < at + 4)) {  // bytes before a block's start, or its first 4
                    // (chained blocks are >= 1 KiB: the seed word is ~0)
                    const int32_t rel = q * 16 - at;
                    slot.x = fix_word(slot.x, rel, 0xffffffffu);
                    slot.y = fix_word(slot.y, rel + 4, 0xffffffffu);
                    slot.z = fix_word(slot.z, rel + 8, 0xffffffffu);
                    slot.w = fix_word(slot.w, rel + 12, 0xffffffffu);
                }
                const uint32_t f = r0_granule(slot, L);
                slot = load16(prow <= rlast ? pp : zero);
                ++prow;
                pp += 256;
                uint32_t wa = lookup4<kRegionA + kHalf>(A, L);  // Shift_256(A)
                const bool swn = onNext && !sw;  // this lane's first granule past the block: snapshot, restart
                S = swn ? A : S;
                wa = swn ? 0u : wa;
                sw = sw || onNext;
                A = wa ^ f;
                if (__any(row == cEnd)) {
                    if (row == cEnd) {
                        emit(k);
                        ++k;
                        qa0 = qa1;
                        qa1 = qa2;
                        qa2 = qa3;
                        qa3 = kFar;
                        qg0 = qg1;
                        qg1 = qg2;
                        qg2 = qg3;
                        cEnd = k < 3u ? (qg0 >> 4) + 1 : (k == 3u ? rlast : -1);
                    }
                }
                ++row;
            };
            // exits leave the loop: only the path through all kStreamRing steps
            // returns to its head (an exit back to the head made the compiler
            // wait for every load there)
            // (the compiler still waits for every load at the loop's head: two
            // passes over the ring per iteration halve those waits)
            for (uint32_t t = 0;;) {
                static_assert(kStreamRing == 8, "the ring's steps are spelled out");
#pragma unroll
                for (uint32_t i = 0; i < 2 * kStreamRing; ++i) {
                    fstep(ring[i % kStreamRing]);
                    if (++t >= steps) goto done;
                }
            }
        done:;
        } else {
        // The general plan: any block that does not follow its predecessor is
        // a stream of its own.  Current unit (cursor c) and prefetch cursor
        // (p): unit index, row
        // (v[i] for a run-time i as selects of copies: an indexed read of the
        // array put the arrays in scratch)
        const int32_t pa0 = pa[0], pa1 = pa[1], pa2 = pa[2], pa3 = pa[3];
        const int32_t pb0 = pb[0], pb1 = pb[1], pb2 = pb[2], pb3 = pb[3];
        const int32_t pg0 = pge[0], pg1 = pge[1], pg2 = pge[2], pg3 = pge[3];
        const int32_t ps0 = pst[0], ps1 = pst[1], ps2 = pst[2], ps3 = pst[3];
        const int32_t pe0 = pen[0], pe1 = pen[1], pe2 = pen[2], pe3 = pen[3];
        auto sel4 = [](int i, int32_t v0, int32_t v1, int32_t v2, int32_t v3) {
            return i == 0 ? v0 : i == 1 ? v1 : i == 2 ? v2 : v3;
        };
#define SST_SEL(arr, i) sel4((i), arr##0, arr##1, arr##2, arr##3)
        auto chained = [&](int i) { return i == 1 ? pch[1] : i == 2 ? pch[2] : i == 3 ? pch[3] : false; };
        auto skip = [&](int &i) {  // the first unit at or after i with rows (constant-index selects: no scratch)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (i < 4 && SST_SEL(pe, i) < SST_SEL(ps, i)) ++i;
        };
        int ci = 0;
        skip(ci);
        int pi = ci;
        int32_t prow = pi < 4 ? SST_SEL(ps, pi) : 0;
        auto pf_next = [&]() -> uint4 {  // the prefetch cursor's row, then advance it
            const bool on = pi < 4;
            const uint4 v = load_row(prow, on);
            if (on) {
                ++prow;
                if (prow > SST_SEL(pe, pi)) {
                    ++pi;
                    skip(pi);
                    prow = pi < 4 ? SST_SEL(ps, pi) : prow;  // (chained: the row after the last one)
                }
            }
            return v;
        };
        uint4 ring[kStreamRing];
#pragma unroll
        for (uint32_t s = 0; s < kStreamRing; ++s) ring[s] = pf_next();
        if (have_prv) finish(prv_um, prv_ok, prv_a, prv_b);
        // current unit's values
        int32_t row = ci < 4 ? SST_SEL(ps, ci) : 0;
        int32_t cA = 0, cGe = -1, cEnd = -1, cAn = kFar;
        uint32_t cS0 = 0, cS0n = 0;
        auto load_cur = [&]() {
            if (ci < 4) {
                cA = SST_SEL(pa, ci);
                cGe = SST_SEL(pg, ci);
                cEnd = SST_SEL(pe, ci);
                cS0 = SST_SEL(pb, ci) - cA >= 4 ? 0xffffffffu : 0u;
                const bool ch = chained(ci + 1);
                cAn = ch ? SST_SEL(pa, ci + 1) : kFar;
                cS0n = ch && SST_SEL(pb, ci + 1) - SST_SEL(pa, ci + 1) >= 4 ? 0xffffffffu : 0u;
            }
        };
        load_cur();
        auto step = [&](uint4 &slot) {
            const uint4 vr = slot;
            slot = pf_next();
            const bool act = ci < 4;
            fold_row(vr, row, cA, cAn, cGe, cS0, cS0n, act);
            if (__any(act && row == cEnd)) {
                if (act && row == cEnd) {  // group-uniform: unit ci is done for every lane
                    emit(static_cast<uint32_t>(ci));
                    const bool ch = chained(ci + 1);
                    if (!ch) A = 0u;
                    ++ci;
                    skip(ci);
                    load_cur();
                    row = ch ? row + 1 : (ci < 4 ? SST_SEL(ps, ci) : row + 1);
                    return;
                }
            }
            ++row;
        };
        for (uint32_t t = 0; t < steps; t += kStreamRing) {  // wave-uniform
#pragma unroll
            for (uint32_t s = 0; s < kStreamRing; ++s) {
                if (t + s >= steps) break;
                step(ring[s]);
            }
        }
#undef SST_SEL
        }
        prv_um = um;
        prv_ok = uok;
        prv_a = ua;
        prv_b = ub;
        have_prv = true;
        if (next >= nclaims) break;  // wave-uniform
        claim = next;
        ho = hon;
        hs = hsn;
    }
    if (have_prv) finish(prv_um, prv_ok, prv_a, prv_b);
}

}  // namespace lvk

namespace lvgpu_internal {
using namespace lvh;
// SSTable trailers (csrc/sst.hip): one sst_blocks_kernel launch.
int launch_sst_blocks(bool seal, const uint8_t *d_file, uint64_t file_bytes, const uint64_t *d_handles,
                      const uint8_t *d_types, size_t n, uint32_t *d_status, uint32_t *d_crc, void *stream) {
    DevCtx *c = nullptr;
    if (int rc = current_ctx(&c)) return rc;
    lvk::Params P{};
    P.base = reinterpret_cast<uint64_t>(d_file);
    constexpr uint64_t kRunUnits = 4ull * lvk::kSstRun;  // blocks per wave claim
    const uint64_t claims = (n + kRunUnits - 1) / kRunUnits;
    P.n = claims * kRunUnits;  // entries of the walk; those past the last block are empty lanes
    P.flags = 0;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 grid(static_cast<uint32_t>(std::min<uint64_t>(c->cus, claims))), block(lvk::kThreads);
    // the continuous walk (sst_stream_kernel) for files whose positions fit
    // its 32-bit arithmetic; the per-unit walk otherwise
    const uint64_t fb = reinterpret_cast<uint64_t>(d_file), origin = fb & ~static_cast<uint64_t>(255);
    if (LVK_SST_STREAM && (fb - origin) + file_bytes + 64 < (1ull << 31) - (1ull << 25)) {  // (below kFar)
        lvk::SstStream a{origin,
                         static_cast<int32_t>(fb - origin),
                         static_cast<int32_t>(fb - origin + file_bytes),
                         reinterpret_cast<const uint2 *>(d_handles),
                         d_types,
                         d_status,
                         d_crc,
                         file_bytes,
                         n};
        const uint64_t sclaims = (n + lvk::kClaimUnits - 1) / lvk::kClaimUnits;
        const dim3 sgrid(static_cast<uint32_t>(std::min<uint64_t>(c->cus, sclaims)));
        if (seal) {
            g_kernel = "sst_stream_kernel<seal>";
            hipLaunchKernelGGL((lvk::sst_stream_kernel<true, false>), sgrid, block, 0, s, a, c->image[1]);
        } else if (d_crc) {
            g_kernel = "sst_stream_kernel<verify,crc>";
            hipLaunchKernelGGL((lvk::sst_stream_kernel<false, true>), sgrid, block, 0, s, a, c->image[1]);
        } else {
            g_kernel = "sst_stream_kernel<verify>";
            hipLaunchKernelGGL((lvk::sst_stream_kernel<false, false>), sgrid, block, 0, s, a, c->image[1]);
        }
        return check_launch();
    }
    if (seal) {
        lvk::TableUnits<true> u{reinterpret_cast<const uint2 *>(d_handles), d_types, nullptr, nullptr, file_bytes, n};
        g_kernel = "sst_blocks_kernel<seal>";
        // (4 rows per batch: Shift_1024 is the G = 16 image's own row shift)
        hipLaunchKernelGGL((lvk::sst_blocks_kernel<true, false>), grid, block, 0, s, P,
                           c->image[lvk::kSealRows == 4 ? 2 : kTableImage], u);
    } else if (d_crc) {
        lvk::TableUnits<false, true> u{reinterpret_cast<const uint2 *>(d_handles), nullptr, d_status, d_crc, file_bytes,
                                        n};
        g_kernel = "sst_blocks_kernel<verify,crc>";
        hipLaunchKernelGGL((lvk::sst_blocks_kernel<false, true>), grid, block, 0, s, P, c->image[kTableImage], u);
    } else {
        lvk::TableUnits<false, false> u{reinterpret_cast<const uint2 *>(d_handles), nullptr, d_status, nullptr,
                                        file_bytes, n};
        g_kernel = "sst_blocks_kernel<verify>";
        hipLaunchKernelGGL((lvk::sst_blocks_kernel<false, false>), grid, block, 0, s, P, c->image[kTableImage], u);
    }
    return check_launch();
}

}  // namespace lvgpu_internal

namespace lvs {

int check_args(const void *file, const uint64_t *handles, size_t n) {
    if (!file || !handles) return lvgpu_internal::set_error(LV_ERR_INVALID, "null device pointer");
    if (n > 0xffffffffull) return lvgpu_internal::set_error(LV_ERR_INVALID, "more than 2^32-1 blocks per call");
    if (reinterpret_cast<uintptr_t>(handles) % 8) return lvgpu_internal::set_error(LV_ERR_INVALID, "handles must be 8-byte aligned");
    return LV_OK;
}

}  // namespace lvs

extern "C" {

// Both device entry points are ONE kernel launch (lvk::sst_blocks_kernel,
// above): the handles are read in file order, the CRC walk is the
// offsets API's G = 16 aligned-row walk, and the trailer compare / write is
// its epilogue.
int lv_sst_seal_blocks_device(uint8_t *d_file, uint64_t file_bytes, const uint64_t *d_handles,
                              const uint8_t *d_types, size_t n, void *stream) {
    lvgpu_internal::clear_error();
    if (n == 0) return LV_OK;
    if (int rc = lvs::check_args(d_file, d_handles, n)) return rc;
    return lvgpu_internal::launch_sst_blocks(true, d_file, file_bytes, d_handles, d_types, n, nullptr, nullptr, stream);
}

int lv_sst_verify_blocks_device(const uint8_t *d_file, uint64_t file_bytes, const uint64_t *d_handles, size_t n,
                                uint32_t *d_status, uint32_t *d_crc, void *stream) {
    lvgpu_internal::clear_error();
    if (n == 0) return LV_OK;
    if (int rc = lvs::check_args(d_file, d_handles, n)) return rc;
    if (!d_status) return lvgpu_internal::set_error(LV_ERR_INVALID, "null status pointer");
    return lvgpu_internal::launch_sst_blocks(false, d_file, file_bytes, d_handles, nullptr, n, d_status, d_crc, stream);
}

// The file goes to the device through the device's host path (cached arena;
// pinned input: one DMA, pageable: pipelined pinned staging), the handles and
// the status words through its cached scratch buffer, as lv_wal_scan_host
// does: after the first call of a given size nothing is allocated on the
// device.
int lv_sst_verify_blocks_host(const uint8_t *file, uint64_t file_bytes, const uint64_t *handles, size_t n,
                              uint32_t *status, int device) {
    lvgpu_internal::clear_error();
    if (n == 0) return LV_OK;
    if ((!file && file_bytes) || !handles || !status)
        return lvgpu_internal::set_error(LV_ERR_INVALID, "null host pointer");
    if (n > 0xffffffffull) return lvgpu_internal::set_error(LV_ERR_INVALID, "more than 2^32-1 blocks per call");
    lvgpu_internal::HostPath hp;
    if (int rc = lvgpu_internal::host_upload(device, file, file_bytes, 16, &hp)) return rc;
    hipStream_t s = static_cast<hipStream_t>(hp.stream);
    const size_t hbytes = n * 16, sbytes = (n * 4 + 15) & ~static_cast<size_t>(15);
    uint8_t *scr = nullptr;
    if (int rc = lvgpu_internal::host_scratch(&hp, 0, hbytes + sbytes, &scr)) return rc;
    uint64_t *d_h = reinterpret_cast<uint64_t *>(scr);
    uint32_t *d_st = reinterpret_cast<uint32_t *>(scr + hbytes);
    auto hip = [&](hipError_t e, const char *what) {
        if (e == hipSuccess) return LV_OK;
        (void)hipStreamSynchronize(s);
        return lvgpu_internal::set_error(static_cast<int>(e), (std::string(what) + ": " + hipGetErrorString(e)).c_str());
    };
    if (int rc = hip(hipMemcpyAsync(d_h, handles, hbytes, hipMemcpyHostToDevice, s), "H2D")) return rc;
    lvgpu_internal::count_h2d(hbytes);
    if (int rc = lv_sst_verify_blocks_device(hp.d_arena, file_bytes, d_h, n, d_st, nullptr, s)) {
        (void)hipStreamSynchronize(s);
        return rc;
    }
    if (int rc = hip(hipMemcpyAsync(status, d_st, n * 4, hipMemcpyDeviceToHost, s), "D2H")) return rc;
    lvgpu_internal::count_d2h(n * 4);
    return hip(hipStreamSynchronize(s), "sync");
}

}  // extern "C"
