/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatements of the reference's checksum VERIFY loops, used as the
 * checker and as the `cpu_baseline` of bench.py's SURVEY 8f lines (never by
 * the product, which does this work on the GPU):
 *
 *  - oracle_wal_verify: the framing + CRC check of sunchao/leveldb-rs
 *    `Reader::read_physical_record` (`src/log_reader.rs:271-364`) over a
 *    whole log held in memory: 32 KiB reads (`:274-292`), header parse
 *    (`:305-310`), the length bound (`:312-324`), the zero-record skip
 *    (`:326-331`) and `unmask(decode_fixed_32(hdr)) == value(hdr[6..7+len])`
 *    (`:333-343`).  The fragment state machine (`read_record`, `:120-265`)
 *    does no checksum work and is left to the caller.
 *  - oracle_units_verify: the same compare for units at given offsets with
 *    the masked CRC stored at another offset (the SSTable trailer check:
 *    `value(contents || type)` against the LE32 after it).
 *  - oracle_units_seal: `mask(extend(value(contents), [type]))` written as
 *    LE32 after the type byte (the trailer writer).
 *
 * CRCs come from the reference-dispatched `oracle_extend` (crc32c.rs:42-51).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

uint32_t oracle_extend(uint32_t crc, const uint8_t *data, size_t n);
uint32_t oracle_mask(uint32_t crc);
uint32_t oracle_unmask(uint32_t masked);

#define OV_BLOCK 32768u /* log_format.rs:63 */
#define OV_HEADER 7u    /* log_format.rs:66 */

/* coding.rs:70-77 */
static inline uint32_t ov_le32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* Whole-log verify (log_reader.rs:271-364).  Returns the number of physical
 * records that passed the CRC; *mismatch counts "checksum mismatch" drops,
 * *bad_length "bad record length" drops. */
uint64_t oracle_wal_verify(const uint8_t *log, uint64_t size, uint64_t *mismatch, uint64_t *bad_length) {
    uint64_t ok = 0, mm = 0, bl = 0;
    for (uint64_t blk = 0; blk < size; blk += OV_BLOCK) {
        /* file.read(BLOCK_SIZE): a short read marks EOF (:283-289) */
        uint64_t len = size - blk < OV_BLOCK ? size - blk : OV_BLOCK;
        int eof = len < OV_BLOCK;
        const uint8_t *p = log + blk;
        while (len >= OV_HEADER) {
            uint32_t length = (uint32_t)p[4] | ((uint32_t)p[5] << 8); /* :305-310 */
            uint32_t type = p[6];
            if (OV_HEADER + length > len) { /* :312-324 */
                if (!eof) ++bl;
                break;
            }
            if (type == 0 && length == 0) break; /* :326-331: skip the rest */
            if (oracle_unmask(ov_le32(p)) != oracle_extend(0, p + 6, 1 + (size_t)length)) { /* :333-343 */
                ++mm;
                break; /* the buffer (rest of the block) is dropped */
            }
            ++ok;
            p += OV_HEADER + length;
            len -= OV_HEADER + length;
        }
    }
    if (mismatch) *mismatch = mm;
    if (bad_length) *bad_length = bl;
    return ok;
}

/* Unit verify: unit i = base[unit_off[i] .. +unit_len[i]), its masked CRC is
 * LE32 at base + crc_off[i].  Returns the number of mismatches. */
uint64_t oracle_units_verify(const uint8_t *base, const uint64_t *unit_off, const uint32_t *unit_len,
                             const uint64_t *crc_off, size_t n) {
    uint64_t bad = 0;
    for (size_t i = 0; i < n; ++i)
        bad += oracle_unmask(ov_le32(base + crc_off[i])) != oracle_extend(0, base + unit_off[i], unit_len[i]);
    return bad;
}

/* Trailer seal: block i = base[off[i] .. +size[i]) followed by its type byte;
 * writes LE32(mask(extend(value(contents), [type]))) after the type. */
void oracle_units_seal(uint8_t *base, const uint64_t *off, const uint32_t *size, size_t n) {
    for (size_t i = 0; i < n; ++i) {
        uint8_t *b = base + off[i];
        uint32_t c = oracle_extend(oracle_extend(0, b, size[i]), b + size[i], 1);
        uint32_t m = oracle_mask(c);
        uint8_t *t = b + size[i] + 1;
        t[0] = (uint8_t)m;
        t[1] = (uint8_t)(m >> 8);
        t[2] = (uint8_t)(m >> 16);
        t[3] = (uint8_t)(m >> 24);
    }
}
