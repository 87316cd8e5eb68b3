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
    // Wait-count mode (walk.h sorted_stream): both run mode 2, every load
    // unconditional within its path (verify: 0.703 -> 0.723 in round 4,
    // profiles/r04/final_ab/).  The seal also waits explicitly for the batch
    // it folds (kCurWait): with mode 2 alone the compiler's merge over the
    // loop's paths still waited vmcnt(0) in the head batches' fix-up, i.e. for
    // the prefetch as well, and the seal ran slower than with masked loads
    // (0.628 vs 0.669, profiles/r06/seal_exact/); with the explicit wait
    // 0.683-0.688 against 0.665-0.669 (profiles/r06/seal_curwait/).  The
    // verify walk's own counts are already exact (the explicit wait there
    // measured flat, profiles/r06/curwait/).
    static constexpr uint32_t kExact = 2u;
    static constexpr bool kCurWait = SEAL;  // walk.h sorted_stream: explicit wait for the folded batch
    static constexpr uint32_t kTrailerLoads = SEAL ? 0u : 2u;  // loads trailer() issues per lane

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
