/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference CRC32C module, sunchao/leveldb-rs
 * `src/util/crc32c.rs`, used as the parity checker for the MI355X batch
 * engine.  Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
 * `cpu_baseline` leg may load this library; the product (`leveldb-rs_amd/`)
 * never links, calls or falls back to it.
 *
 * Parity pinning: the reference's own known-answer tests
 * (`crc32c.rs:147-171`, `standard_results`) and property tests
 * (`:174-193`) are replayed against this file by `tests/test_oracle.py`
 * from `tests/golden/crc32c_kat.json`.  The reference itself (Rust, ~2019
 * nightly, un-vendored crates) cannot be compiled in this image; see
 * DESIGN.md "Oracle".
 *
 * Every function cites the reference line range it restates.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <nmmintrin.h> /* SSE4.2 crc32 — the instruction extend_hw uses */

/* crc32c.rs:21-23 */
#define ORC_XOR 0xffffffffu
#define ORC_POLY 0x82f63b78u /* reflected Castagnoli */
#define ORC_MASK_DELTA 0xa282ead8u

static uint32_t g_tab[16][256];
static int g_tab_ready = 0;

/* crc32c.rs:126-140 make_table: bit-at-a-time reflected table. */
static void orc_make_table(uint32_t poly, uint32_t *out) {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int b = 0; b < 8; ++b) c = (c & 1u) ? (c >> 1) ^ poly : (c >> 1);
        out[i] = c;
    }
}

/* crc32c.rs:25-38 TABLE16: tab[j][i] = (tab[j-1][i] >> 8) ^ tab[0][low byte]. */
static void orc_init(void) {
    if (g_tab_ready) return;
    orc_make_table(ORC_POLY, g_tab[0]);
    for (int i = 0; i < 256; ++i) {
        uint32_t c = g_tab[0][i];
        for (int j = 1; j < 16; ++j) {
            c = (c >> 8) ^ g_tab[0][c & 0xffu];
            g_tab[j][i] = c;
        }
    }
    g_tab_ready = 1;
}

static inline uint32_t le32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

static inline uint64_t le64(const uint8_t *p) {
    return (uint64_t)le32(p) | ((uint64_t)le32(p + 4) << 32);
}

/* crc32c.rs:53-57 mask: rotate right 15, wrapping add delta. */
uint32_t oracle_mask(uint32_t crc) {
    return ((crc >> 15) | (crc << 17)) + ORC_MASK_DELTA;
}

/* crc32c.rs:59-63 unmask. */
uint32_t oracle_unmask(uint32_t masked) {
    uint32_t rot = masked - ORC_MASK_DELTA;
    return (rot >> 17) | (rot << 15);
}

/* crc32c.rs:65-84 extend_sw: slice-by-8 over 8-byte steps, bytewise tail. */
uint32_t oracle_extend_sw(uint32_t crc, const uint8_t *data, size_t n) {
    orc_init();
    uint32_t l = crc ^ ORC_XOR;
    while (n >= 8) {
        l ^= le32(data);
        l = g_tab[0][data[7]] ^ g_tab[1][data[6]] ^ g_tab[2][data[5]] ^ g_tab[3][data[4]] ^
            g_tab[4][(l >> 24) & 0xffu] ^ g_tab[5][(l >> 16) & 0xffu] ^
            g_tab[6][(l >> 8) & 0xffu] ^ g_tab[7][l & 0xffu];
        data += 8;
        n -= 8;
    }
    for (size_t i = 0; i < n; ++i) l = g_tab[0][(l ^ data[i]) & 0xffu] ^ (l >> 8);
    return l ^ ORC_XOR;
}

/* crc32c.rs:120-124 align_offset. */
static size_t orc_align_offset(size_t align, const uint8_t *p) {
    uintptr_t v = (uintptr_t)p;
    return ((v + (align - 1)) & ~(uintptr_t)(align - 1)) - v;
}

/* crc32c.rs:86-118 extend_hw: SSE4.2 crc32 u8 prologue to 8-byte alignment,
 * u64 body, one u32 step, u8 tail; buffers <= 16 bytes go bytewise. */
__attribute__((target("sse4.2")))
uint32_t oracle_extend_hw(uint32_t crc, const uint8_t *data, size_t size) {
    uint32_t l = crc ^ ORC_XOR;
    size_t off = 0;
    if (size > 16) {
        size_t start = orc_align_offset(8, data);
        while (off != start) l = _mm_crc32_u8(l, data[off++]);
        while (size - off >= 8) {
            l = (uint32_t)_mm_crc32_u64(l, le64(data + off));
            off += 8;
        }
        while (size - off >= 4) {
            l = _mm_crc32_u32(l, le32(data + off));
            off += 4;
        }
    }
    while (off != size) l = _mm_crc32_u8(l, data[off++]);
    return l ^ ORC_XOR;
}

/* crc32c.rs:42-51 extend: SSE4.2 when present, else slice-by-8. */
uint32_t oracle_extend(uint32_t crc, const uint8_t *data, size_t n) {
    if (__builtin_cpu_supports("sse4.2")) return oracle_extend_hw(crc, data, n);
    return oracle_extend_sw(crc, data, n);
}

/* crc32c.rs:40 value. */
uint32_t oracle_value(const uint8_t *data, size_t n) { return oracle_extend(0, data, n); }

/* Independent bit-at-a-time CRC-32C (not in the reference): a third
 * implementation used only to cross-check sw == hw == bitwise. */
uint32_t oracle_extend_bitwise(uint32_t crc, const uint8_t *data, size_t n) {
    uint32_t l = crc ^ ORC_XOR;
    for (size_t i = 0; i < n; ++i) {
        l ^= data[i];
        for (int b = 0; b < 8; ++b) l = (l & 1u) ? (l >> 1) ^ ORC_POLY : (l >> 1);
    }
    return l ^ ORC_XOR;
}

/* Exposes TABLE16 (crc32c.rs:25-38) so tests can compare table constants. */
void oracle_table16(uint32_t *out /* 16*256 */) {
    orc_init();
    memcpy(out, g_tab, sizeof(g_tab));
}

/* Batch driver for the checker: out[i] = [mask](extend(seed[i] or 0,
 * arena[off[i] .. off[i]+len[i]))).  flags bit0 = mask (crc32c.rs:54).
 * Calls the reference-dispatched `extend` (crc32c.rs:42-51) per buffer,
 * exactly as the WAL callers do (log_writer.rs:123-124, log_reader.rs:336). */
void oracle_batch(const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                  const uint32_t *seed, uint32_t *out, size_t n, uint32_t flags) {
    for (size_t i = 0; i < n; ++i) {
        uint32_t c = oracle_extend(seed ? seed[i] : 0u, arena + off[i], len[i]);
        out[i] = (flags & 1u) ? oracle_mask(c) : c;
    }
}

/* Same, forcing the slice-by-8 path (crc32c.rs:65-84). */
void oracle_batch_sw(const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                     const uint32_t *seed, uint32_t *out, size_t n, uint32_t flags) {
    for (size_t i = 0; i < n; ++i) {
        uint32_t c = oracle_extend_sw(seed ? seed[i] : 0u, arena + off[i], len[i]);
        out[i] = (flags & 1u) ? oracle_mask(c) : c;
    }
}

/* Restatement of benches/crc32c.rs:23-49: hash one buffer `iters` times with
 * extend_sw (which=0) or extend_hw (which=1) from seed 0; returns the xor of
 * results so the loop is not optimised away.  Timing is done by the caller. */
uint32_t oracle_bench_loop(const uint8_t *buf, size_t n, uint64_t iters, int which) {
    uint32_t acc = 0;
    for (uint64_t i = 0; i < iters; ++i)
        acc ^= which ? oracle_extend_hw(0, buf, n) : oracle_extend_sw(0, buf, n);
    return acc;
}

/* Synthetic payload generator shared with the device generator in the
 * product (lv_fill_splitmix): byte k of the arena is byte (k & 7) of
 * splitmix64(seed ^ (k >> 3)).  Test infrastructure only. */
static inline uint64_t orc_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

void oracle_fill_splitmix(uint8_t *dst, uint64_t byte_begin, uint64_t nbytes, uint64_t seed) {
    uint64_t k = byte_begin;
    uint64_t end = byte_begin + nbytes;
    while (k < end && (k & 7)) {  /* head up to the next word boundary */
        *dst++ = (uint8_t)(orc_splitmix64(seed ^ (k >> 3)) >> (8 * (k & 7)));
        ++k;
    }
    for (; k + 8 <= end; k += 8, dst += 8) {  /* whole words, little-endian */
        uint64_t w = orc_splitmix64(seed ^ (k >> 3));
        memcpy(dst, &w, 8);  /* x86-64 hosts only: little-endian */
    }
    for (; k < end; ++k)  /* tail */
        *dst++ = (uint8_t)(orc_splitmix64(seed ^ (k >> 3)) >> (8 * (k & 7)));
}
