/*
 * lvgpu table — SSTable block trailers on MI355X and the table-format codecs
 * around them.
 *
 * Format (src/table/format.rs): BlockHandle {offset, size} as two varint64s
 * (format.rs:26-50, coding.rs:144-166, 223-241, 284-288) and the 48-byte
 * Footer {metaindex handle, index handle, zero pad to 40 B, LE64 magic
 * 0xdb4775248b80fb57} (format.rs:52-104).
 *
 * Block trailer: the reference declares Options::verify_checksums
 * (options.rs:84) but has no block trailer yet, so the layout is upstream
 * LevelDB's: block contents, then type (1 B, 0 = no compression), then
 * LE32(mask(crc32c(contents || type))) — 5 bytes after each handle's extent.
 * Parity beyond the crc32c KATs is unpinned (no reference code or fixture).
 */
#ifndef LVGPU_TABLE_H
#define LVGPU_TABLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LV_SST_MAGIC 0xdb4775248b80fb57ull   /* format.rs:24 */
#define LV_SST_BLOCK_HANDLE_MAX 20u          /* format.rs:35 */
#define LV_SST_FOOTER_SIZE 48u               /* format.rs:70 */
#define LV_SST_TRAILER_SIZE 5u               /* type + masked crc */
#define LV_SST_NO_COMPRESSION 0u

/* Per-block verify status */
#define LV_SST_BLOCK_OK 0u
#define LV_SST_BLOCK_CHECKSUM_MISMATCH 1u
#define LV_SST_BLOCK_OUT_OF_RANGE 2u  /* offset + size + 5 > file bytes, or size >= 2^32 - 1 */

/* BlockHandle::encode_to (format.rs:37-40): writes <= 20 bytes, returns the count. */
size_t lv_sst_block_handle_encode(uint64_t offset, uint64_t size, uint8_t *dst);
/* BlockHandle::decode_from (format.rs:42-49) over src[0..n): LV_OK and the
 * bytes consumed, or LV_ERR_CORRUPTION ("bad handle"). */
int lv_sst_block_handle_decode(const uint8_t *src, size_t n, uint64_t *offset, uint64_t *size, size_t *consumed);
/* Footer::encode_to (format.rs:72-80) into out[48]. */
void lv_sst_footer_encode(uint64_t metaindex_offset, uint64_t metaindex_size, uint64_t index_offset,
                          uint64_t index_size, uint8_t *out);
/* Footer::decode_from (format.rs:82-103) over src[0..n), n >= 48:
 * handles = {metaindex offset, size, index offset, size}.  LV_ERR_CORRUPTION
 * with "not a sstable (bad magic number)" or "bad handle". */
int lv_sst_footer_decode(const uint8_t *src, size_t n, uint64_t handles[4]);

/* Seal n blocks of a device-resident table being built: for handle i
 * (d_handles[2i] = offset, d_handles[2i+1] = size) write the type byte
 * (d_types ? d_types[i] : 0) at offset+size and the masked crc32c of
 * contents||type at offset+size+1.  Handles must be in range and disjoint. */
int lv_sst_seal_blocks_device(uint8_t *d_file, uint64_t file_bytes, const uint64_t *d_handles,
                              const uint8_t *d_types, size_t n, void *stream);
/* Verify n blocks of a device-resident table: d_status[i] = LV_SST_BLOCK_*
 * (a ReadOptions::verify_checksums read of every block at once).  Optionally
 * d_crc[i] = crc32c(contents || type) (NULL to skip). */
int lv_sst_verify_blocks_device(const uint8_t *d_file, uint64_t file_bytes, const uint64_t *d_handles, size_t n,
                                uint32_t *d_status, uint32_t *d_crc, void *stream);
/* Host-memory variant: copies the table and handles in, verifies, copies
 * the statuses back (end-to-end path). */
int lv_sst_verify_blocks_host(const uint8_t *file, uint64_t file_bytes, const uint64_t *handles, size_t n,
                              uint32_t *status, int device);

#ifdef __cplusplus
}
#endif

#endif /* LVGPU_TABLE_H */
