// Host internals shared by the product library's HIP translation units
// (blocks.hip, sort.hip, classes.hip, wal_scan.hip, sst.hip, context.hip):
// lv_last_error plumbing, the per-device context (table images, sort
// workspaces, piece matrices, host-path staging) and the launchers one
// component exports to another.  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/lvgpu/crc32c.h"
#include "lv_internal.h"
#include "lvk/core.h"

namespace lvh {

extern thread_local std::string g_err;
// Kernel the calling thread's last batch call launched (lv_crc32c_last_kernel).
extern thread_local const char *g_kernel;
int set_err(int code, const std::string &msg);

#define LV_HIP(call)                                                                   \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess)                                                          \
            return set_err(static_cast<int>(e_), std::string(#call) + ": " +           \
                                                     hipGetErrorString(e_));           \
    } while (0)


constexpr int kGs[4] = {1, 4, 16, 64};
// The table walk's image: the G = 16 one with region A's row shift
// Shift_{256 kSstRows} (Shift_768 for three-row batches).
constexpr int kTableImage = 4;
// The image of the G = 16 aligned-row walks over length-sorted lists (class
// and fused kernels): region A's row shift is Shift_{256 *
// kAlRows} -- the G = 16 image's Shift_1024, or the table image's Shift_768
// (kSstRows = 3) for 3 rows per batch.
constexpr uint32_t kAlRowsH = LVK_AL_ROWS;  // = lvk::kAlRows (lvk/sort.h)
constexpr int kAlImage = kAlRowsH == 4 ? 2 : kTableImage;
static_assert(kAlRowsH == 4 || kAlRowsH == lvk::kSstRows, "aligned rows: 4, or the table image's");
constexpr int kImages = 5;

// Host copy of the LDS image for each G (index into kGs), and the table
// image; layout in lvk/core.h.
const std::vector<uint32_t> &host_image(int gi);

// Library-owned sort workspace of one (device, stream).  Calls on one stream
// are stream-ordered on the GPU, but two host threads enqueueing on the same
// stream would interleave their four kernels: `m` is held from the workspace
// lookup through the last launch of a call, so one call's sort passes are
// enqueued back to back and a growing hipFree never frees a buffer another
// thread has been handed but not yet launched on.
struct StreamWs {
    std::mutex m;
    uint8_t *p = nullptr;
    size_t cap = 0;
    // hint violations of this stream's calls (lv_crc32c_batch_check): a device
    // word and a pinned host word to read it into, made once under em
    std::mutex em;
    uint32_t *err = nullptr;
    uint32_t *herr = nullptr;
};

struct DevCtx {
    std::mutex m;  // one-time init
    bool ready = false;
    int cus = 0;
    uint4 *image[kImages] = {};  // per G (kGs), then the table image
    uint32_t *base_tabs = nullptr;  // Shift_{2^i}, i < lvk::kBaseMats, as byte tables (4 x 256 words each)
    std::mutex ws_m;  // guards the map (entries are never erased)
    std::map<hipStream_t, std::unique_ptr<StreamWs>> ws;
    // long-block split: Shift matrices per piece length (immutable once built)
    std::mutex mats_m;
    std::map<uint64_t, uint32_t *> piece_mats;
    std::map<uint64_t, uint32_t *> piece_tabs;
    // host-path staging (grown on demand), serialised by host_m
    std::mutex host_m;
    uint8_t *d_arena = nullptr;
    size_t d_arena_cap = 0;
    uint8_t *d_meta = nullptr;
    size_t d_meta_cap = 0;
    uint8_t *h_meta = nullptr;
    size_t h_meta_cap = 0;
    uint8_t *h_stage[2] = {nullptr, nullptr};
    size_t h_stage_cap[2] = {0, 0};
    hipEvent_t ev[2] = {nullptr, nullptr};
    hipStream_t stream = nullptr;
    // the pipelined WAL scan's second slot: a stream and a device chunk copy
    hipStream_t stream2 = nullptr;
    uint8_t *d_arena2 = nullptr;
    size_t d_arena2_cap = 0;
    uint8_t *d_scr[2] = {nullptr, nullptr};  // scratch for other host paths (WAL scan)
    size_t d_scr_cap[2] = {0, 0};
    int dev = 0;
};

constexpr size_t kStageBytes = 64ull << 20;  // pinned staging slot for pageable input

// lv_device_counters: per-device host-path traffic and allocations
struct DevCounters {
    std::atomic<uint64_t> h2d{0}, d2h{0}, allocs{0};
};
extern DevCounters g_count[64];
DevCounters &counters();


int grow_dev(uint8_t **p, size_t *cap, size_t need);
int grow_pinned(uint8_t **p, size_t *cap, size_t need);
// True if p is page-locked host memory (hipHostMalloc / hipHostRegister).
bool is_pinned(const void *p);
// memcpy split over up to 8 host threads (pageable -> pinned staging).
void par_memcpy(uint8_t *dst, const uint8_t *src, size_t bytes, unsigned threads = LVK_MEMCPY_THREADS);
// The calling thread's current device's context, initialised on first use.
int current_ctx(DevCtx **out);
// Buffers-per-group choice for a known (uniform) length.
int pick_gi(uint64_t len);
// Group-size override from flags (LV_CRC_GROUP), or -1.
int forced_gi(uint32_t flags);
// hipGetLastError -> status + lv_last_error.
int check_launch();

constexpr size_t al16(size_t x) { return (x + 15) & ~static_cast<size_t>(15); }

// ---- sort workspace (sort.hip) ----
// Sorting workgroups and elements per workgroup for n buffers.
uint64_t sort_wgs(uint64_t n, uint64_t *chunk);
// Byte offsets of the sort workspace regions (layout in lvk/sort.h).
struct WsLayout {
    size_t m, wgb, ent, sseed, part, longs, tmp, pos, total;
};
WsLayout ws_layout(uint64_t n);
size_t sort_ws_bytes(uint64_t n);
// The library-owned workspace of (device, stream), grown on demand; returns
// with its lock held in `lk` (the caller keeps it through its last launch).
int stream_ws_bytes(DevCtx &c, hipStream_t s, size_t need, uint8_t **out, std::unique_lock<std::mutex> *lk);
int stream_ws(DevCtx &c, hipStream_t s, uint64_t n, uint8_t **out, std::unique_lock<std::mutex> *lk);
// Shift_{j plen} GF(2) matrices / Shift_{2^v plen} byte tables on the device,
// built once per plen (context.hip).
int piece_mats(DevCtx &c, uint64_t plen, const uint32_t **out);
int piece_tabs(DevCtx &c, uint64_t plen, const uint32_t **out);

// The facts of a caller's lv_batch_hint, for the kernels' checks (err: the
// stream's violation word, lv_crc32c_batch_check); null = nothing to check.
struct HintCheck {
    uint32_t *err;
    uint64_t total;
    uint32_t len;
    uint32_t uniform;
};
inline void set_hint(lvk::Params &P, const HintCheck *hc, uint32_t dflt_len) {
    P.herr = hc ? hc->err : nullptr;
    P.htotal = hc ? hc->total : 0;
    P.hlen = hc ? hc->len : dflt_len;
    P.huni = hc ? hc->uniform : 0;
}
// The violation word of (device, stream), allocated and zeroed on first use.
int stream_err(DevCtx &c, hipStream_t s, uint32_t **out);
// Reads and clears the current device's violation word of stream s.
int check_hints(hipStream_t s, uint32_t *violations);

// ---- launchers ----
// The length sort of the offsets API (sort.hip) for n > 1,024 buffers:
// histogram + column scan + scatter.  Fills P.ent,
// P.sseed and P.part (the long-buffer split's piece registers, or null when
// splitting is off) and returns the long-buffer records (or null).
uint4 *launch_sort(uint8_t *ws_bytes, const uint64_t *off, const uint32_t *len, const uint32_t *seed, uint64_t n,
                   hipStream_t s, lvk::Params *P);
// sort_scan over a wgs-row histogram matrix M (sort.hip; the WAL framing
// shares it).
void launch_sort_scan(uint32_t *M, uint32_t wgs, uint32_t *ws, uint64_t *wgb, hipStream_t s);
// The whole offsets API on a workspace: sort, class kernel, long-buffer
// join (classes.hip).
// join = false leaves out the join launch (the caller proved it empty with
// hint_needs_join).
int launch_binned(DevCtx &c, uint8_t *ws_bytes, const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                  const uint32_t *seed, uint32_t *out, uint64_t n, uint32_t flags, hipStream_t s, bool join = true,
                  const HintCheck *hc = nullptr);
// Whether a batch with these host-side facts needs the long-buffer join
// (lv_crc32c_batch_device_hint; classes.hip).
bool hint_needs_join(const lv_batch_hint &h, uint64_t n, uint32_t cus);
// The persistent class kernel over a sorted list (classes.hip).
void launch_classes(const DevCtx &c, bool seeded, const lvk::Params &P, const uint32_t *ws, hipStream_t s);
// One group-size kernel over a batch, offsets or strided (blocks.hip).
void launch_group(const DevCtx &c, bool strided, int gi, const uint8_t *arena, const uint64_t *off,
                  const uint32_t *len, uint64_t stride, uint32_t blen, const uint32_t *seed, uint32_t *out, uint64_t n,
                  uint32_t flags, hipStream_t s);
// The uniform-block kernels (blocks.hip) for n blocks of blen bytes, 16-B
// aligned: the long-block split (ps > 0; `scratch` bytes of piece registers
// unless the pieces join inside the walk) or crc32c_blocks_kernel with group
// size kGs[bgi]; neither when the blocks are not whole 1 KiB batches.
struct UniformPlan {
    uint32_t ps;
    int bgi;
    uint64_t scratch;
    bool applies() const { return ps > 0 || bgi >= 0; }
};
UniformPlan uniform_plan(int cus, uint64_t base, uint64_t stride, uint32_t blen, uint64_t n, int gi);
// Launches a plan that applies: block k at base + off[k] (off != null, the
// offsets API with an aligned uniform hint; len = the device lengths, checked
// against hc when it is not null) or base + k * stride.
int launch_uniform(DevCtx &c, const UniformPlan &pl, const uint8_t *base, uint64_t stride, const uint64_t *off,
                   const uint32_t *len, const HintCheck *hc, uint32_t blen, uint64_t n, const uint32_t *seed,
                   uint32_t *out, uint32_t flags, hipStream_t hs, uint8_t *scr);

}  // namespace lvh
