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
    const uint32_t *cls = ws + kWsCls;
    const bool ident = ws[kWsIdent] != 0u;  // sort_scatter skipped a one-key batch
    stage_tables(image);
    if (threadIdx.x == 0) g_lds[kPoolWord] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const Lut L = make_lut(lane);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t grid = gridDim.x;
    const uint32_t n23 = cls[6] + cls[7];
    // pieces of split long buffers (walked after classes 2+3; a split buffer
    // is longer than 16 KiB, so class 2 or 3, and n23 > 0 whenever there are
    // pieces)
    const uint32_t np = P.part ? min(ws[kWsPieces], kPieceBudget) : 0u;
    // With no large buffers at all, every wave walks the small classes.
#if LVK_SMALL_ALL
    const uint32_t nsmall = n23 ? kSmallWaves : kWaves;
#else
    constexpr uint32_t nsmall = kSmallWaves;
#endif
    if (wave < nsmall) {
        const uint64_t sw = blockIdx.x * nsmall + wave, nsw = grid * nsmall;
        uint64_t k = 0;
        auto stride = [&]() { return sw + (++k) * nsw; };
        if (cls[4]) {
            sorted_stream<1>(sub_list(P, cls[0], cls[4]), SortedList<SEEDED>{ident}, lane, L, sw, stride);
            k = 0;
        }
        if (cls[5]) sorted_stream<4>(sub_list(P, cls[1], cls[5]), SortedList<SEEDED>{ident}, lane, L, sw, stride);
    }
    if (n23) {
#if LVK_CLASS_STAGGER
        // A list of mostly long-buffer pieces (>= 3/4 of the entries), with
        // >= 64 KiB per wave, is the blocks kernel's long-block regime: waves
        // that start together stream their pieces in lockstep, which reads
        // slower; stagger them as crc32c_blocks_kernel does (64 x 16 MiB:
        // 223 -> 201 us per call).
        const uint64_t bytes = (static_cast<uint64_t>(ws[kWsBytes + 1]) << 32) | ws[kWsBytes];
        if (4ull * np >= 3ull * (n23 + np) && bytes >= (64ull << 10) * grid * kWaves)
            for (uint32_t k = 0; k < wave * LVK_STAGGER; ++k) __builtin_amdgcn_s_sleep(32);
#endif
        auto pool = [&]() -> uint64_t {
            uint32_t k = 0;
            if (lane == 0) k = atomicAdd(&g_lds[kPoolWord], 1u);
            return blockIdx.x + grid * static_cast<uint64_t>(__shfl(k, 0));
        };
        sorted_stream<16>(sub_list(P, cls[6] ? cls[2] : cls[3], n23, np), SortedList<SEEDED>{ident}, lane, L, pool(),
                          pool);
    }
}

// Joins the pieces of the offsets API's split long buffers (sort_scatter,
// split_wave): long record {buffer, first piece slot, m, p}, pieces of
// P = 2^p bytes aligned to the buffer end; piece 0's register is
// R_0 = R(~seed, piece 0) and piece k > 0 was walked as a seed-0 buffer,
// part = R(~0, piece k) = R(0, piece k) ^ Shift_P(~0) (the seed trick), so
// R_k = part ^ Shift_P(~0) and R(~seed, buffer) = XOR_k Shift_{(m-1-k) P}(R_k).  One wave
// per buffer, Horner within lanes and a tree across them, every shift a
// wave-uniform base matrix (round 2 before: per-lane shifts by the set bits
// of m - 1 - k, 9.9 us for 64 x 16 MiB).  A lane's run of c pieces is up to
// 8 independent Horner chains joined by an in-lane tree: each Horner step is
// a dependent L2 round trip (~0.18 us), and 4,096 pieces are c = 64.
__global__ __launch_bounds__(256) void combine_long_kernel(const uint32_t *__restrict__ ws,
                                                           const uint4 *__restrict__ longs,
                                                           const uint32_t *__restrict__ part,
                                                           const uint32_t *__restrict__ base,
                                                           const uint32_t *__restrict__ tabs,
                                                           uint32_t *__restrict__ out, uint32_t flags) {
    // the counter counts every claim; records exist only below the budget
    const uint32_t nl = min(ws[kWsLongs], kPieceBudget / 2);
    if (static_cast<uint64_t>(blockIdx.x) * (blockDim.x / 64) >= nl) return;  // block-uniform
#if !LVK_LONG_TABS
    __shared__ uint32_t M[kBaseMats * 32];
    for (uint32_t i = threadIdx.x; i < kBaseMats * 32; i += blockDim.x) M[i] = base[i];
    __syncthreads();
    auto shift = [&](uint32_t i, uint32_t v) { return gf2_apply(M + i * 32, v); };
#else
    // Shift_{2^i}(v) by four byte-table lookups (tables in HBM, L2-resident:
    // 192 KiB for every i) instead of a staged 32-column matrix product
    auto shift = [&](uint32_t i, uint32_t v) { return tab_shift(tabs + i * 1024u, v); };
#endif
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * (blockDim.x / 64);
#if LVK_LONG_TABS && LVK_LONG_LDSP
    __shared__ uint32_t TP[4][1024];  // per wave: Shift_P of its record
    uint32_t *const tp = TP[threadIdx.x >> 6];
#endif
    for (uint32_t w = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); w < nl; w += nw) {
        const uint4 r = longs[w];  // {buffer, first, m, p}
        const uint32_t m = r.z, p = r.w;
        if (m == 0) continue;  // a claim past the piece budget: the buffer was walked whole
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
#if LVK_LONG_TABS && LVK_LONG_LDSP
        // d - 1 dependent Shift_P steps: from an LDS copy (one HBM round trip
        // to stage 4 KiB) instead of an L2 / HBM round trip each
        if (d > 1) {  // wave-uniform
            const uint4 *src = reinterpret_cast<const uint4 *>(tabs + p * 1024u);
            uint4 *dst = reinterpret_cast<uint4 *>(tp);
            const uint4 v0 = src[lane], v1 = src[64u + lane], v2 = src[128u + lane], v3 = src[192u + lane];
            __builtin_amdgcn_wave_barrier();  // the previous record's reads of tp are done
            dst[lane] = v0;
            dst[64u + lane] = v1;
            dst[128u + lane] = v2;
            dst[192u + lane] = v3;
            __builtin_amdgcn_wave_barrier();
        }
        for (uint32_t i = 1; i < d; ++i) {  // wave-uniform trip count
            uint32_t rk[8];
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q) rk[q] = piece(q, i);
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q) ch[q] = tab_shift(tp, ch[q]) ^ rk[q];
        }
#else
        for (uint32_t i = 1; i < d; ++i) {  // wave-uniform trip count
            uint32_t rk[8];
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q) rk[q] = piece(q, i);
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q) ch[q] = shift(p, ch[q]) ^ rk[q];
        }
#endif
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
}

}  // namespace lvk

namespace lvh {

void launch_classes(const DevCtx &c, bool seeded, const lvk::Params &P, const uint32_t *ws, hipStream_t s) {
    if (seeded)
        hipLaunchKernelGGL(lvk::crc32c_classes_kernel<true>, dim3(static_cast<uint32_t>(c.cus)), dim3(lvk::kThreads), 0,
                           s, P, c.image[2], ws);
    else
        hipLaunchKernelGGL(lvk::crc32c_classes_kernel<false>, dim3(static_cast<uint32_t>(c.cus)), dim3(lvk::kThreads),
                           0, s, P, c.image[2], ws);
}

// Length-sorted launch of the offsets API, no host sync: the sort (one or
// three launches), the persistent class kernel, the long-buffer join.
int launch_binned(DevCtx &c, uint8_t *ws_bytes, const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                  const uint32_t *seed, uint32_t *out, uint64_t n, uint32_t flags, hipStream_t s) {
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
    uint4 *longs = launch_sort(ws_bytes, off, len, seed, n, s, &P);
    g_kernel = "sort+crc32c_classes_kernel";
    launch_classes(c, seed != nullptr, P, ws, s);
    // joins split long buffers (exits at once when the sort split none).  (A
    // last-finisher join inside the class kernel -- agent-scope release and
    // acquire around a per-buffer counter -- measured 64 x 16 MiB 200 -> 345
    // us and 1,024 x 64 KiB 41 -> 177 us: every fence writes back or
    // invalidates the XCD's whole L2; and C3 via offsets -2 % from spills.)
    if (longs)
        hipLaunchKernelGGL(lvk::combine_long_kernel, dim3(static_cast<uint32_t>(c.cus)), dim3(256), 0, s, ws, longs,
                           P.part, c.base_mats, c.base_tabs, out, flags);
    return 0;
}


}  // namespace lvh

using namespace lvh;

extern "C" {

static int batch_device_impl(const uint8_t *d_arena, const uint64_t *d_off, const uint32_t *d_len,
                             const uint32_t *d_seed, uint32_t *d_out, size_t n, uint32_t flags,
                             void *stream, uint8_t *d_ws, size_t ws_bytes) {
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
    } else if (int rc = stream_ws(*c, s, n, &d_ws, &ws_lk)) {
        return rc;
    }
    if (int rc = launch_binned(*c, d_ws, d_arena, d_off, d_len, d_seed, d_out, n, flags, s)) return rc;
    return check_launch();
}

int lv_crc32c_batch_device(const uint8_t *d_arena, const uint64_t *d_off, const uint32_t *d_len,
                           const uint32_t *d_seed, uint32_t *d_out, size_t n, uint32_t flags,
                           void *stream) {
    return batch_device_impl(d_arena, d_off, d_len, d_seed, d_out, n, flags, stream, nullptr, 0);
}

size_t lv_crc32c_workspace_bytes(size_t n) { return sort_ws_bytes(n); }

int lv_crc32c_batch_device_ws(const uint8_t *d_arena, const uint64_t *d_off, const uint32_t *d_len,
                              const uint32_t *d_seed, uint32_t *d_out, size_t n, uint32_t flags,
                              void *d_workspace, size_t workspace_bytes, void *stream) {
    if (!d_workspace) return set_err(LV_ERR_INVALID, "null workspace");
    return batch_device_impl(d_arena, d_off, d_len, d_seed, d_out, n, flags, stream,
                             static_cast<uint8_t *>(d_workspace), workspace_bytes);
}

}  // extern "C"
