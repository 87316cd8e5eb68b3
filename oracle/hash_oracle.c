/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of sunchao/leveldb-rs `src/util/hash.rs:20-51` (the
 * murmur-like hash behind the block cache's shard choice, `util/cache.rs:182`,
 * `:394-399`).  Checker for the batched GPU hash; the product never links it.
 * Pinned by the reference KATs `hash.rs:58-75` (tests/test_hash.py).
 *
 * Overflow: `h += w` / `h += byte << k` are plain `+=` on u32 in the reference;
 * a release build (and upstream LevelDB's Hash) wraps, which is what the KATs
 * hold, so the restatement wraps.
 */
#include <stddef.h>
#include <stdint.h>

/* decode_fixed_32, coding.rs:70-77 */
static inline uint32_t hor_le32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* hash.rs:20-51 */
uint32_t oracle_hash(const uint8_t *data, size_t n, uint32_t seed) {
    const uint32_t m = 0xc6a4a793u;
    const uint32_t r = 24;
    uint32_t h = seed ^ (m * (uint32_t)n);
    size_t i = 0;
    while (i + 4 <= n) {               /* :29-36 */
        uint32_t w = hor_le32(data + i);
        i += 4;
        h += w;
        h *= m;
        h ^= h >> 16;
    }
    size_t diff = n - i;               /* :38-48 */
    if (diff >= 3) h += (uint32_t)data[i + 2] << 16;
    if (diff >= 2) h += (uint32_t)data[i + 1] << 8;
    if (diff >= 1) {
        h += data[i];
        h *= m;
        h ^= h >> r;
    }
    return h;
}

void oracle_hash_batch(const uint8_t *arena, const uint64_t *off, const uint32_t *len, const uint32_t *seed,
                       uint32_t *out, size_t n) {
    for (size_t i = 0; i < n; ++i) out[i] = oracle_hash(arena + off[i], len[i], seed ? seed[i] : 0u);
}

/* cache.rs:399 — shard(hash) = hash >> (32 - NUM_SHARD_BITS), NUM_SHARD_BITS = 4 (:370) */
uint32_t oracle_cache_shard(uint32_t hash) { return hash >> (32 - 4); }
