/*
 * lvgpu hash — the block cache's key hash, batched on MI355X.
 *
 * Replaces sunchao/leveldb-rs `util::hash::hash(data: &[u8], seed: u32) -> u32`
 * (src/util/hash.rs:20-51), whose callers are the cache's SliceHasher
 * (src/util/cache.rs:182) and shard choice (src/util/cache.rs:394-399).
 * Arithmetic is wrapping u32, as a release build of the reference computes
 * and as its KATs (hash.rs:58-75) hold.
 */
#ifndef LVGPU_HASH_H
#define LVGPU_HASH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Batch flags */
#define LV_HASH_SHARD 0x1u /* write cache shard indices (hash >> 28) instead of hashes */

/* hash(data, seed), hash.rs:20-51.  Host scalar. */
uint32_t lv_hash(const uint8_t *data, size_t n, uint32_t seed);
/* shard(hash) = hash >> (32 - NUM_SHARD_BITS), NUM_SHARD_BITS = 4 (cache.rs:370, :399). */
uint32_t lv_cache_shard(uint32_t hash);

/* out[i] = hash(d_arena[d_off[i] .. d_off[i] + d_len[i]], d_seed ? d_seed[i] : 0)
 * (or its shard with LV_HASH_SHARD), for i < n, stream-ordered on `stream`
 * (a hipStream_t, NULL = default stream).  All pointers are device memory the
 * caller owns; buffers may start at any byte.  Returns LV_OK or an error code
 * (lv_last_error()). */
int lv_hash_batch_device(const uint8_t *d_arena, const uint64_t *d_off, const uint32_t *d_len,
                         const uint32_t *d_seed, uint32_t *d_out, size_t n, uint32_t flags, void *stream);

/* Packed keys (keys laid end to end, as a block's or an Arrow-style string
 * array's): key i = d_arena[b[i] .. b[i+1]) for n + 1 bounds b of
 * `bound_bytes` bytes each (4: uint32_t, 8: uint64_t; nondecreasing), at
 * d_bounds (device memory, aligned to bound_bytes).  Same output as
 * lv_hash_batch_device, with 4 or 8 B of metadata per key instead of 12. */
int lv_hash_batch_packed(const uint8_t *d_arena, const void *d_bounds, uint32_t bound_bytes, const uint32_t *d_seed,
                         uint32_t *d_out, size_t n, uint32_t flags, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* LVGPU_HASH_H */
