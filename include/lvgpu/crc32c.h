/*
 * lvgpu — MI355X-native batched CRC32C for leveldb-rs's WAL and table-block
 * checksum path.  C ABI (no HIP, torch or C++ types in any signature).
 *
 * The reference exposes Rust free functions in `leveldb::util::crc32c`
 * (src/util/mod.rs:23); each scalar entry point below is the C twin of one of
 * them, bit-identical on every input, so a Rust `extern "C"` shim maps
 * `&[u8]` to (ptr, len) one-to-one.  The batch entry points
 * are new: they checksum many independent buffers per call on the GPU.
 *
 * Conventions
 *   - Scalar functions: pure, reentrant, infallible, never allocate
 *     (crc32c.rs:40-118).  They run on the host CPU: a single WAL record is
 *     far below a kernel launch's cost.
 *   - Batch functions: device buffers are caller-owned and never freed by the
 *     library; calls are stream-ordered and asynchronous on `stream` (a
 *     hipStream_t passed as void*, NULL = default stream); the return is 0 or
 *     a nonzero lv_status / hipError_t code, with lv_last_error() describing
 *     it.  No host fallback exists: without a usable GPU the batch calls fail.
 */
#ifndef LVGPU_CRC32C_H
#define LVGPU_CRC32C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- scalar drop-ins (host) -------------------------------------------- */

/* crc32c.rs:40      pub fn value(data: &[u8]) -> u32 */
uint32_t lv_crc32c_value(const uint8_t *data, size_t n);
/* crc32c.rs:42-51   pub fn extend(crc: u32, data: &[u8]) -> u32 */
uint32_t lv_crc32c_extend(uint32_t crc, const uint8_t *data, size_t n);
/* crc32c.rs:53-57   pub fn mask(crc: u32) -> u32 */
uint32_t lv_crc32c_mask(uint32_t crc);
/* crc32c.rs:59-63   pub fn unmask(masked_crc: u32) -> u32 */
uint32_t lv_crc32c_unmask(uint32_t masked_crc);
/* crc32c.rs:65-84   pub fn extend_sw(crc: u32, data: &[u8]) -> u32 */
uint32_t lv_crc32c_extend_sw(uint32_t crc, const uint8_t *data, size_t n);
/* crc32c.rs:86-118  pub unsafe fn extend_hw(crc: u32, data: &[u8]) -> u32
 * (requires SSE4.2 on the host, as the reference's #[target_feature] does) */
uint32_t lv_crc32c_extend_hw(uint32_t crc, const uint8_t *data, size_t n);
/* Not in the reference (an addition for callers that split long buffers):
 * extend(s, A || B) from crc_a = extend(s, A) and crc_b = value(B), len_b =
 * |B|: Shift_{len_b}(crc_a) ^ crc_b with GF(2) shift matrices, O(log len_b). */
uint32_t lv_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

/* ---- batch API (device) ------------------------------------------------- */

/* flags */
#define LV_CRC_MASK 0x1u /* store mask(crc) (crc32c.rs:54) instead of crc      */
/* Tuning/test hook: force the lanes-per-buffer group size G of the kernel
 * (g in {1,4,16,64}) instead of the library's choice by length. */
#define LV_CRC_GROUP(g) ((g) == 1 ? 0x100u : (g) == 4 ? 0x200u : (g) == 16 ? 0x300u : (g) == 64 ? 0x400u : 0u)
#define LV_CRC_GROUP_MASK 0x700u

/* status codes (besides hipError_t values passed through) */
#define LV_OK 0
#define LV_ERR_INVALID (-1) /* bad argument                                   */
#define LV_ERR_NO_DEVICE (-2) /* no usable GPU / HIP runtime error at init     */
#define LV_ERR_CORRUPTION (-3) /* malformed on-disk data (table format decode)  */

/* out[i] = [mask](extend(seed ? seed[i] : 0, arena[off[i] .. off[i]+len[i])))
 * for i < n.  All pointers are device pointers; `d_seed` may be NULL (all
 * seeds 0, i.e. value()).  Buffers may start at any byte offset and overlap.
 * This is the batched form of the per-record calls at log_writer.rs:123-124
 * (seed = type_crc[t], LV_CRC_MASK) and log_reader.rs:335-336 (seed 0). */
int lv_crc32c_batch_device(const uint8_t *d_arena, const uint64_t *d_off, const uint32_t *d_len,
                           const uint32_t *d_seed, uint32_t *d_out, size_t n, uint32_t flags,
                           void *stream);

/* Same as lv_crc32c_batch_device with a caller-owned device workspace of at
 * least lv_crc32c_workspace_bytes(n) bytes (the per-call length sort).  Use it
 * for stream capture into a HIP graph, or to run concurrent calls on several
 * streams without the library's per-stream workspace. */
size_t lv_crc32c_workspace_bytes(size_t n);
int lv_crc32c_batch_device_ws(const uint8_t *d_arena, const uint64_t *d_off, const uint32_t *d_len,
                              const uint32_t *d_seed, uint32_t *d_out, size_t n, uint32_t flags,
                              void *d_workspace, size_t workspace_bytes, void *stream);

/* Host-side facts about a batch whose lengths live on the device.  The WAL
 * group-commit writer and the SST sealer know their fragment / block lengths
 * on the host; with them the library can leave out launches that the facts
 * prove empty -- for batches of <= 1,024 buffers the long-buffer join when no
 * buffer can be split, or when every split buffer of a uniform batch is
 * joined inside the walk; for larger uniform batches that cannot split, the
 * whole length sort and the join (the buffers are walked in index order) --
 * which the device-only call cannot know without a host sync.
 * The facts must be exact (max_len may be any upper bound of the lengths).
 * The kernels check them where they read what the facts describe (every
 * offset and length on the aligned path, every length on the identity and
 * small-batch paths, the total on the small-batch path) and record a
 * violation for lv_crc32c_batch_check instead of failing silently; a call
 * whose hint was violated leaves its CRCs undefined.
 * A uniform batch whose buffers all start 16-byte aligned (uniform ==
 * LV_HINT_UNIFORM | LV_HINT_ALIGNED16; SST blocks of a fixed size, pages) and
 * whose length is a multiple of 1 KiB runs on the kernels of
 * lv_crc32c_batch_strided with each buffer's start read from d_off: no sort,
 * no join, the long-buffer split of the strided API (the library checks that
 * d_arena is 16-byte aligned and otherwise ignores the bit).  `uniform` must
 * be 0, LV_HINT_UNIFORM or LV_HINT_UNIFORM | LV_HINT_ALIGNED16; any other
 * value is LV_ERR_INVALID. */
#define LV_HINT_UNIFORM 1u
#define LV_HINT_ALIGNED16 2u
typedef struct lv_batch_hint {
    uint64_t total_bytes; /* sum of d_len[i] */
    uint32_t max_len;     /* an upper bound of every d_len[i] */
    uint32_t uniform;     /* nonzero: every d_len[i] == max_len (then total_bytes == n * max_len); bit
                             LV_HINT_ALIGNED16: also every d_arena + d_off[i] is 16-byte aligned */
} lv_batch_hint;

/* lv_crc32c_batch_device(_ws) with an optional hint (NULL = no hint) and an
 * optional caller workspace (NULL = the library's per-stream workspace). */
int lv_crc32c_batch_device_hint(const uint8_t *d_arena, const uint64_t *d_off, const uint32_t *d_len,
                                const uint32_t *d_seed, uint32_t *d_out, size_t n, uint32_t flags,
                                const lv_batch_hint *hint, void *d_workspace, size_t workspace_bytes,
                                void *stream);

/* Hint violations found on the device (bits of lv_crc32c_batch_check's
 * *violations). */
#define LV_HINT_ERR_MISALIGNED 0x1u /* LV_HINT_ALIGNED16: d_off[i] % 16 != 0          */
#define LV_HINT_ERR_NOT_UNIFORM 0x2u /* LV_HINT_UNIFORM: d_len[i] != max_len          */
#define LV_HINT_ERR_LONGER 0x4u /* d_len[i] > max_len                                  */
#define LV_HINT_ERR_TOTAL 0x8u /* sum of d_len[i] != total_bytes                      */
#define LV_ERR_HINT (-4) /* a batch hint contradicted the device-side lengths/offsets */

/* Stream-ordered check of the hints of every lv_crc32c_batch_device_hint call
 * enqueued on `stream` (on the calling thread's current device) since the last
 * check: waits for the stream, then returns LV_OK, or LV_ERR_HINT with the
 * violated facts in *violations (may be NULL) and lv_last_error naming them;
 * the record is cleared.  Not needed after lv_crc32c_batch_host (its hint is
 * derived from the host arrays). */
int lv_crc32c_batch_check(void *stream, uint32_t *violations);

/* Debug query: 1 if a batch of n buffers with these facts, on a device with
 * `cus` compute units, launches the long-buffer join (the decision
 * lv_crc32c_batch_device_hint makes on the host), 0 if it is left out.  A
 * sorted batch (> 1,024 buffers, not uniform-and-unsplittable) always
 * launches it: that launch also puts the CRCs back in buffer order.  With
 * LV_HINT_ALIGNED16 (an aligned d_arena assumed) and whole-KiB lengths, the
 * join is the strided API's, launched when a split's pieces are not joined
 * inside the walk. */
int lv_crc32c_hint_needs_join(const lv_batch_hint *hint, size_t n, uint32_t cus);

/* Fixed-stride form for table blocks: buffer i is
 * d_base[i*stride .. i*stride + block_len).  Same semantics as above. */
int lv_crc32c_batch_strided(const uint8_t *d_base, uint64_t stride, uint32_t block_len, size_t n,
                            const uint32_t *d_seed, uint32_t *d_out, uint32_t flags, void *stream);

/* Host-memory form (the path starts and ends in host memory: log/SST file
 * buffers).  Copies arena[0 .. arena_bytes) and the metadata to `device`
 * through pinned staging with hipMemcpyAsync, runs the batch kernel and
 * copies the n results back; synchronous.  Offsets index into h_arena. */
int lv_crc32c_batch_host(const uint8_t *h_arena, size_t arena_bytes, const uint64_t *h_off,
                         const uint32_t *h_len, const uint32_t *h_seed, uint32_t *h_out, size_t n,
                         uint32_t flags, int device);

/* Multi-GPU host batch: lv_crc32c_batch_host semantics, with
 * the buffers split into contiguous ranges balanced by payload bytes, one per
 * device (0..ngpu-1), one host thread per device; each device receives only
 * its range's arena span.  No collective.  A device that is not present fails
 * the call (lv_last_error names it). */
int lv_crc32c_batch_multi(const uint8_t *h_arena, size_t arena_bytes, const uint64_t *h_off, const uint32_t *h_len,
                          const uint32_t *h_seed, uint32_t *h_out, size_t n, uint32_t flags, int ngpu);
/* The same over an explicit device list (a device may repeat: its ranges
 * then run one after another). */
int lv_crc32c_batch_multi_devices(const uint8_t *h_arena, size_t arena_bytes, const uint64_t *h_off,
                                  const uint32_t *h_len, const uint32_t *h_seed, uint32_t *h_out, size_t n,
                                  uint32_t flags, const int *devices, int ndev);

/* ---- runtime ----------------------------------------------------------- */

/* Uploads the lookup tables to the current device (idempotent; the batch
 * calls do it on first use).  Returns 0 or an error code. */
int lv_device_init(void);
/* Human-readable description of the last error on this thread ("" if none). */
const char *lv_last_error(void);
/* Library version string. */
const char *lv_version(void);
/* Debug query: name of the kernel the calling thread's last batch call
 * launched ("crc32c_blocks_kernel<16>", "sort+crc32c_classes_kernel", ...;
 * "" before any).  Lets tests assert which path a geometry takes. */
const char *lv_crc32c_last_kernel(void);

/* Debug query: what the library's host entry points (lv_crc32c_batch_host,
 * lv_crc32c_batch_multi*, lv_wal_scan_host, lv_sst_verify_blocks_host) have
 * moved and allocated on `device` since the process started.  Fills
 * out[0..min(n, 3)): [0] bytes copied host -> device (payload, metadata and
 * handles), [1] bytes copied device -> host, [2] device or pinned-host
 * allocations the library made on the device (hipMalloc / hipHostMalloc).
 * Lets tests assert that a multi-device batch ships each device only its
 * buffers and that cached host paths stop allocating.  0 or LV_ERR_INVALID. */
int lv_device_counters(int device, uint64_t *out, size_t n);

/* ---- page-locked host memory for callers' file buffers ------------------- */

/* Page-locked (pinned) host memory: a caller that reads a log or table file
 * into a buffer from lv_host_alloc hands the host entry points input the GPU
 * reads by DMA directly -- no staging copy on the CPU (lv_wal_scan_host*,
 * lv_crc32c_batch_host, lv_sst_verify_blocks_host detect pinned input).
 * NULL on failure (lv_last_error).  Free with lv_host_free. */
void *lv_host_alloc(size_t bytes);
/* Frees lv_host_alloc memory (NULL is a no-op): 0 or an error code. */
int lv_host_free(void *p);

/* ---- synthetic data (bench / tests) ------------------------------------- */

/* d_dst[k] = byte ((begin+k) & 7) of splitmix64(seed ^ ((begin+k) >> 3)) for
 * k < nbytes: the payload generator of the benchmark configurations (SURVEY
 * 8d), generated in place in HBM.  Stream-ordered. */
int lv_fill_splitmix(uint8_t *d_dst, uint64_t begin, uint64_t nbytes, uint64_t seed, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* LVGPU_CRC32C_H */
