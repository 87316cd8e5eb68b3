/*
 * lvgpu WAL — batched write-ahead-log encode / verify on MI355X, the callers
 * of the CRC path.  C ABI.
 *
 * Reader side (log_reader.rs): a whole log is scanned on the GPU — every
 * 32 KiB block's physical-record header chain is walked (the framing of
 * read_physical_record, log_reader.rs:271-331) and every [type || payload]
 * CRC unit is checksummed in one batch (log_reader.rs:335-336).  A host
 * reader then replays the reference Reader state machine (fragments, drops,
 * reports, initial offset; log_reader.rs:44-393) taking each record's CRC from
 * the scan instead of computing it.
 *
 * Writer side (log_writer.rs): many logical records are laid out exactly as
 * Writer::add_record does (log_writer.rs:62-110) and every fragment header's
 * masked CRC (log_writer.rs:123-125) comes from one GPU batch.
 */
#ifndef LVGPU_WAL_H
#define LVGPU_WAL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* log_format.rs:22-29, 62-66 */
#define LV_WAL_BLOCK_SIZE 32768u
#define LV_WAL_HEADER_SIZE 7u

/* Physical-record status in lv_wal_scan info (bits 8..15) */
#define LV_WAL_REC_OK 0u          /* header fits its block: CRC computed       */
#define LV_WAL_REC_BAD_LENGTH 1u  /* HEADER_SIZE + length > bytes left in block */
#define LV_WAL_REC_ZERO 2u        /* type ZERO with length 0 (reader skips)      */

typedef struct lv_wal_scan lv_wal_scan;

/* Scan a host-memory log on `device`: copies it in, frames every block on
 * the GPU, CRCs every record and copies the results back.  Returns NULL on
 * error (lv_last_error()).  Records are in log order. */
lv_wal_scan *lv_wal_scan_host(const uint8_t *log, size_t bytes, int device);
/* The same scan, pipelined against its reader: returns at once, while a
 * worker thread scans the log in 32 MiB block-aligned chunks (upload, device
 * scan, results back).  A reader over this scan (lv_wal_reader_new) waits only
 * for the chunk holding the next header it reaches, so replaying chunk k
 * overlaps the scan of chunk k + 1; the accessors below wait for the whole
 * scan.  `log` must stay valid until lv_wal_scan_free.  NULL on an argument
 * error; a scan error surfaces from the reader (< 0) or lv_wal_scan_wait. */
lv_wal_scan *lv_wal_scan_host_pipelined(const uint8_t *log, size_t bytes, int device);
/* Waits for a pipelined scan to finish: 0, or its error (lv_last_error).
 * Immediate for any other scan.  Memory: a pipelined scan keeps its per-chunk
 * arrays (readers over it point into them) and, once this or an accessor below
 * is called, also the flat arrays -- about 16 B per record twice (a 1 GiB log
 * of 178 K records: ~5.7 MB).  A caller that only reads records through
 * lv_wal_reader never pays the second copy. */
int lv_wal_scan_wait(lv_wal_scan *scan);
/* Device-resident scan of a log already in HBM (8-byte aligned), with no
 * host synchronisation: every 32 KiB block's header chain is walked as
 * read_physical_record frames it and every [type || payload] unit is
 * checksummed, in five launches on `stream` (framing, one global length sort,
 * the CRC kernel, the log-order write-back).  Records go to d_hdr_off / d_crc /
 * d_info in log order (the lv_wal_scan arrays below), at most `cap` of them;
 * *d_count (device memory) receives the number of records.  If that number
 * exceeds cap, nothing else is written: call again with a larger capacity.
 * d_workspace: >= lv_wal_scan_workspace_bytes(bytes, cap) bytes, 16-B aligned. */
size_t lv_wal_scan_workspace_bytes(size_t bytes, size_t cap);
int lv_wal_scan_device(const uint8_t *d_log, size_t bytes, uint64_t *d_hdr_off, uint32_t *d_crc, uint32_t *d_info,
                       size_t cap, uint64_t *d_count, void *d_workspace, size_t workspace_bytes, void *stream);
/* Number of physical records reached by the blocks' header chains (a
 * pipelined scan: waits for it; 0 if it failed). */
size_t lv_wal_scan_count(const lv_wal_scan *scan);
/* Header offsets (ascending), value([type||payload]) (0 unless status OK),
 * and info = type | status << 8 | payload_length << 16. */
const uint64_t *lv_wal_scan_offsets(const lv_wal_scan *scan);
const uint32_t *lv_wal_scan_crcs(const lv_wal_scan *scan);
const uint32_t *lv_wal_scan_info(const lv_wal_scan *scan);
/* Build a scan from caller arrays (copied): tests / externally computed CRCs. */
lv_wal_scan *lv_wal_scan_from_arrays(const uint64_t *offsets, const uint32_t *crcs, const uint32_t *info,
                                     size_t n);
void lv_wal_scan_free(lv_wal_scan *scan);

/* Reporter: Reporter::corruption(bytes, reason) (log_reader.rs:37-42). */
typedef void (*lv_wal_reporter_fn)(void *ctx, size_t bytes, const char *reason);

typedef struct lv_wal_reader lv_wal_reader;

/* Reader::new(file, reporter, checksum, initial_offset) (log_reader.rs:75-94)
 * over an in-memory log and its scan (both must outlive the reader).
 * `reporter` may be NULL. */
lv_wal_reader *lv_wal_reader_new(const uint8_t *log, size_t bytes, const lv_wal_scan *scan,
                                 lv_wal_reporter_fn reporter, void *ctx, int checksum,
                                 uint64_t initial_offset);
/* Reader::read_record (log_reader.rs:120-265): 1 and (*data, *len) = the next
 * record (valid until the next call), 0 at end of input, < 0 on error (a
 * header the scan does not cover). */
int lv_wal_reader_read_record(lv_wal_reader *reader, const uint8_t **data, size_t *len);
/* Reader::last_record_offset (log_reader.rs:99). */
uint64_t lv_wal_reader_last_record_offset(const lv_wal_reader *reader);
void lv_wal_reader_free(lv_wal_reader *reader);

/* Writer::add_record for n logical records at once (log_writer.rs:62-134):
 * record i is payload[rec_off[i] .. rec_off[i] + rec_len[i]).  dest_length is
 * the existing log length (Writer::new_with_dest_length, log_writer.rs:48-56).
 * Writes the appended bytes to out (capacity out_cap) and their count to
 * *out_len; header CRCs are one GPU batch on `device`.  If out is NULL or too
 * small, only *out_len is set and LV_ERR_INVALID is returned. */
int lv_wal_encode_host(const uint8_t *payload, const uint64_t *rec_off, const uint64_t *rec_len, size_t n,
                       uint64_t dest_length, uint8_t *out, size_t out_cap, size_t *out_len, int device);

#ifdef __cplusplus
}
#endif

#endif /* LVGPU_WAL_H */
