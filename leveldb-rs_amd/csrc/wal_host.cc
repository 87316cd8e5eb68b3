// Host side of the WAL components: scan accessors, a Reader that replays the
// reference state machine over a GPU scan, and the batched (group-commit)
// writer.  The reader parses headers from host bytes exactly as the reference
// does and takes each record's CRC from the scan (computed by the GPU batch
// kernel); a header the scan does not cover is an error, never a CPU CRC.
#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lvgpu/crc32c.h"
#include "../../include/lvgpu/wal.h"
#include "lv_internal.h"

namespace {

constexpr uint64_t kBlock = LV_WAL_BLOCK_SIZE;
constexpr uint64_t kHeader = LV_WAL_HEADER_SIZE;

// log_format.rs:22-29; log_reader.rs:27-34
enum : int { kZero = 0, kFull = 1, kFirst = 2, kMiddle = 3, kLast = 4, kEof = 5, kBadRecord = 6 };

uint32_t decode_fixed_32(const uint8_t *p) {  // coding.rs:70-77
    return static_cast<uint32_t>(p[0]) | (static_cast<uint32_t>(p[1]) << 8) |
           (static_cast<uint32_t>(p[2]) << 16) | (static_cast<uint32_t>(p[3]) << 24);
}

}  // namespace

// ---------------------------------------------------------------------------
// scan object
// ---------------------------------------------------------------------------
extern "C" {

// (A pipelined scan fills its flat arrays on the first accessor call.)
static const lv_wal_scan *flat(const lv_wal_scan *scan) {
    if (scan && scan->pipe && lvgpu_internal::scan_flatten(const_cast<lv_wal_scan *>(scan))) return nullptr;
    return scan;
}
size_t lv_wal_scan_count(const lv_wal_scan *scan) { return (scan = flat(scan)) ? scan->off.size() : 0; }
const uint64_t *lv_wal_scan_offsets(const lv_wal_scan *scan) { return (scan = flat(scan)) ? scan->off.data() : nullptr; }
const uint32_t *lv_wal_scan_crcs(const lv_wal_scan *scan) { return (scan = flat(scan)) ? scan->crc.data() : nullptr; }
const uint32_t *lv_wal_scan_info(const lv_wal_scan *scan) { return (scan = flat(scan)) ? scan->info.data() : nullptr; }
int lv_wal_scan_wait(lv_wal_scan *scan) { return lvgpu_internal::scan_flatten(scan); }

lv_wal_scan *lv_wal_scan_from_arrays(const uint64_t *offsets, const uint32_t *crcs, const uint32_t *info,
                                     size_t n) {
    if (n && (!offsets || !crcs || !info)) {
        lvgpu_internal::set_error(LV_ERR_INVALID, "null scan array");
        return nullptr;
    }
    for (size_t i = 1; i < n; ++i)
        if (offsets[i] <= offsets[i - 1]) {
            lvgpu_internal::set_error(LV_ERR_INVALID, "scan offsets must ascend");
            return nullptr;
        }
    lv_wal_scan *s = new lv_wal_scan();
    s->off.assign(offsets, offsets + n);
    s->crc.assign(crcs, crcs + n);
    s->info.assign(info, info + n);
    return s;
}

void lv_wal_scan_free(lv_wal_scan *scan) { delete scan; }

}  // extern "C"

// ---------------------------------------------------------------------------
// Reader: restatement of log_reader.rs:44-393 over an in-memory log
// ---------------------------------------------------------------------------
struct lv_wal_reader {
    const uint8_t *log;
    uint64_t size;
    const lv_wal_scan *scan;
    lv_wal_reporter_fn reporter;
    void *ctx;
    bool checksum;
    // the SequentialFile (StringSource-like): read position
    uint64_t fpos = 0;
    // buffer: a view [buf, buf + blen) of the log, like the reference Slice
    uint64_t buf = 0, blen = 0;
    bool eof = false;
    uint64_t last_record_offset = 0;
    uint64_t end_of_buffer_offset = 0;
    uint64_t initial_offset;
    bool resyncing;
    // The scan entries find() searches: the whole scan, or for a pipelined
    // scan the chunk holding the last header asked for (log offsets [ch_lo,
    // ch_hi)); cursor is the last entry found (reads advance monotonically,
    // so the next header is almost always the next entry).
    const uint64_t *ch_off = nullptr;
    const uint32_t *ch_crc = nullptr, *ch_info = nullptr;
    size_t ch_n = 0;
    uint64_t ch_lo = 1, ch_hi = 0;  // (empty: the first find() selects)
    size_t cursor = ~size_t{0};
    // info / crc of a find() result
    uint32_t info_at(long i) const { return ch_info[i]; }
    uint32_t crc_at(long i) const { return ch_crc[i]; }
    bool failed = false;
    std::vector<uint8_t> scratch;

    // log_reader.rs:101-109
    void report_drop(uint64_t bytes, const char *reason) {
        if (reporter && end_of_buffer_offset >= blen + bytes + initial_offset) reporter(ctx, bytes, reason);
    }

    // Makes the entries covering log offset hdr current (waiting for a
    // pipelined scan's chunk); false if there are none.
    bool select(uint64_t hdr) {
        cursor = ~size_t{0};
        if (!scan->pipe) {
            ch_off = scan->off.data();
            ch_crc = scan->crc.data();
            ch_info = scan->info.data();
            ch_n = scan->off.size();
            ch_lo = 0;
            ch_hi = ~uint64_t{0};
            return true;
        }
        lvgpu_internal::ScanPipe &p = *scan->pipe;  // (the chunk arrays stay valid after a flatten)
        const size_t k = static_cast<size_t>(std::upper_bound(p.lo.begin(), p.lo.end(), hdr) - p.lo.begin()) - 1;
        if (hdr >= p.lo.back() || k >= p.chunks.size()) return false;
        if (p.wait(k)) {
            lvgpu_internal::set_error(p.rc, ("WAL scan: " + p.err).c_str());
            return false;
        }
        const lvgpu_internal::ScanChunk &c = p.chunks[k];
        ch_off = c.off.data();
        ch_crc = c.crc.data();
        ch_info = c.info.data();
        ch_n = c.off.size();
        ch_lo = p.lo[k];
        ch_hi = p.lo[k + 1];
        return true;
    }

    // Scan entry for the header at log offset `hdr` (an index into the
    // current entries), or -1.
    long find(uint64_t hdr) {
        if ((hdr < ch_lo || hdr >= ch_hi) && !select(hdr)) return -1;
        const size_t nx = cursor + 1;  // (0 after a select)
        if (nx < ch_n && ch_off[nx] == hdr) {
            cursor = nx;
            return static_cast<long>(nx);
        }
        if (cursor < ch_n && ch_off[cursor] == hdr) return static_cast<long>(cursor);
        const uint64_t *it = std::lower_bound(ch_off, ch_off + ch_n, hdr);
        if (it == ch_off + ch_n || *it != hdr) return -1;
        cursor = static_cast<size_t>(it - ch_off);
        return static_cast<long>(cursor);
    }

    // log_reader.rs:369-392
    bool skip_to_initial_block() {
        const uint64_t offset_in_block = initial_offset % kBlock;
        uint64_t block_start = initial_offset - offset_in_block;
        if (offset_in_block > kBlock - 6) block_start += kBlock;
        end_of_buffer_offset = block_start;
        if (block_start > 0) {
            if (block_start > size - fpos) {  // StringSource::skip past the end
                fpos = size;
                report_drop(block_start, "in-memory file skipped past end");
                return false;
            }
            fpos += block_start;
        }
        return true;
    }

    // log_reader.rs:271-364; returns the record type (or kEof/kBadRecord)
    // and the fragment as [*frag, *frag + *flen).
    int read_physical_record(uint64_t *frag, uint64_t *flen) {
        for (;;) {
            if (blen < kHeader) {
                if (!eof) {
                    blen = 0;  // last read was a full block: skip its trailer
                    const uint64_t n = std::min<uint64_t>(kBlock, size - fpos);
                    buf = fpos;
                    blen = n;
                    fpos += n;
                    end_of_buffer_offset += n;
                    if (n < kBlock) eof = true;
                    continue;
                }
                blen = 0;  // truncated header at end of file: EOF, not corruption
                return kEof;
            }
            const uint8_t *h = log + buf;
            const uint64_t length = static_cast<uint64_t>(h[4]) | (static_cast<uint64_t>(h[5]) << 8);
            const int type = h[6];
            if (kHeader + length > blen) {
                const uint64_t drop = blen;
                blen = 0;
                if (!eof) {
                    report_drop(drop, "bad record length");
                    return kBadRecord;
                }
                return kEof;  // writer died mid-record: not a corruption
            }
            if (type == kZero && length == 0) {
                blen = 0;
                return kBadRecord;
            }
            if (checksum) {
                const long i = find(buf);
                if (i < 0 || ((info_at(i) >> 8) & 0xffu) != LV_WAL_REC_OK) {
                    failed = true;
                    return kEof;
                }
                const uint32_t expected = lv_crc32c_unmask(decode_fixed_32(h));
                if (expected != crc_at(i)) {
                    const uint64_t drop = blen;
                    blen = 0;
                    report_drop(drop, "checksum mismatch");
                    return kBadRecord;
                }
            }
            *frag = buf + kHeader;
            *flen = length;
            buf += kHeader + length;
            blen -= kHeader + length;
            if (end_of_buffer_offset - blen - kHeader - length < initial_offset) return kBadRecord;
            return type;
        }
    }

    // log_reader.rs:120-265; 1 = record in (*out, *out_len), 0 = EOF, -1 = error
    int read_record(const uint8_t **out, size_t *out_len) {
        if (last_record_offset < initial_offset)
            if (!skip_to_initial_block()) return 0;
        scratch.clear();
        bool in_fragmented_record = false;
        uint64_t prospective_record_offset = 0;
        for (;;) {
            uint64_t frag = 0, flen = 0;
            const int rt = read_physical_record(&frag, &flen);
            if (failed) {
                if (!(scan->pipe && scan->pipe->rc))
                    lvgpu_internal::set_error(LV_ERR_INVALID, "WAL scan does not cover a header the reader reached");
                return -1;
            }
            const uint64_t fsize = (rt == kEof || rt == kBadRecord) ? 0 : flen;
            const int64_t physical_record_offset = static_cast<int64_t>(end_of_buffer_offset) -
                                                   static_cast<int64_t>(blen) - static_cast<int64_t>(kHeader) -
                                                   static_cast<int64_t>(fsize);
            if (resyncing) {
                if (rt == kMiddle) continue;
                if (rt == kLast) {
                    resyncing = false;
                    continue;
                }
                resyncing = false;
            }
            if (rt == kEof) {
                if (in_fragmented_record) scratch.clear();
                return 0;
            }
            if (rt == kBadRecord) {
                if (in_fragmented_record) {
                    report_drop(scratch.size(), "error in middle of record");
                    in_fragmented_record = false;
                    scratch.clear();
                }
                continue;
            }
            const uint64_t scratch_size = in_fragmented_record ? scratch.size() : 0;
            switch (rt) {
                case kFull:
                    if (in_fragmented_record) report_drop(scratch.size(), "partial record without end(1)");
                    prospective_record_offset = static_cast<uint64_t>(physical_record_offset);
                    last_record_offset = prospective_record_offset;
                    *out = log + frag;
                    *out_len = flen;
                    return 1;
                case kFirst:
                    if (in_fragmented_record) report_drop(scratch.size(), "partial record without end(2)");
                    prospective_record_offset = static_cast<uint64_t>(physical_record_offset);
                    scratch.assign(log + frag, log + frag + flen);
                    in_fragmented_record = true;
                    break;
                case kMiddle:
                    if (!in_fragmented_record)
                        report_drop(flen, "missing start of fragmented record(1)");
                    else
                        scratch.insert(scratch.end(), log + frag, log + frag + flen);
                    break;
                case kLast:
                    if (!in_fragmented_record) {
                        report_drop(flen, "missing start of fragmented record(2)");
                    } else {
                        scratch.insert(scratch.end(), log + frag, log + frag + flen);
                        last_record_offset = prospective_record_offset;
                        *out = scratch.data();
                        *out_len = scratch.size();
                        return 1;
                    }
                    break;
                case kZero:
                    report_drop(flen + scratch_size, "unexpected record type");
                    in_fragmented_record = false;
                    scratch.clear();
                    break;
                default:
                    report_drop(flen + scratch_size, "unknown record type");
                    in_fragmented_record = false;
                    scratch.clear();
                    break;
            }
        }
    }
};

extern "C" {

lv_wal_reader *lv_wal_reader_new(const uint8_t *log, size_t bytes, const lv_wal_scan *scan,
                                 lv_wal_reporter_fn reporter, void *ctx, int checksum,
                                 uint64_t initial_offset) {
    if ((!log && bytes) || (checksum && !scan)) {
        lvgpu_internal::set_error(LV_ERR_INVALID, "null log or scan");
        return nullptr;
    }
    lv_wal_reader *r = new lv_wal_reader();
    r->log = log;
    r->size = bytes;
    r->scan = scan;
    r->reporter = reporter;
    r->ctx = ctx;
    r->checksum = checksum != 0;
    r->initial_offset = initial_offset;
    r->resyncing = initial_offset > 0;
    return r;
}

int lv_wal_reader_read_record(lv_wal_reader *reader, const uint8_t **data, size_t *len) {
    if (!reader || !data || !len) return lvgpu_internal::set_error(LV_ERR_INVALID, "null argument");
    return reader->read_record(data, len);
}

uint64_t lv_wal_reader_last_record_offset(const lv_wal_reader *reader) {
    return reader ? reader->last_record_offset : 0;
}

void lv_wal_reader_free(lv_wal_reader *reader) { delete reader; }

// ---------------------------------------------------------------------------
// Writer: Writer::add_record for many records, header CRCs in one GPU batch
// ---------------------------------------------------------------------------
int lv_wal_encode_host(const uint8_t *payload, const uint64_t *rec_off, const uint64_t *rec_len, size_t n,
                       uint64_t dest_length, uint8_t *out, size_t out_cap, size_t *out_len, int device) {
    if (!out_len || (n && (!rec_off || !rec_len))) return lvgpu_internal::set_error(LV_ERR_INVALID, "null argument");
    // Pass 1: layout (log_writer.rs:62-110), identical block arithmetic.
    struct Frag {
        uint64_t out_pos;   // header position in `out`
        uint64_t src;       // payload source offset
        uint32_t len;
        uint8_t type;
    };
    std::vector<Frag> frags;
    std::vector<std::pair<uint64_t, uint64_t>> pads;  // (out_pos, bytes) of zero trailers
    uint64_t block_offset = dest_length % kBlock;     // log_writer.rs:48-56
    uint64_t pos = 0;
    for (size_t r = 0; r < n; ++r) {
        uint64_t left = rec_len[r];
        uint64_t src = rec_off[r];
        bool begin = true;
        for (;;) {
            const uint64_t leftover = kBlock - block_offset;
            if (leftover < kHeader) {
                if (leftover > 0) {
                    pads.emplace_back(pos, leftover);
                    pos += leftover;
                }
                block_offset = 0;
            }
            const uint64_t avail = kBlock - block_offset - kHeader;
            const uint64_t frag_len = left < avail ? left : avail;
            const bool end = left == frag_len;
            const uint8_t type = begin && end ? kFull : begin ? kFirst : end ? kLast : kMiddle;
            frags.push_back({pos, src, static_cast<uint32_t>(frag_len), type});
            pos += kHeader + frag_len;
            block_offset += kHeader + frag_len;
            src += frag_len;
            left -= frag_len;
            begin = false;
            if (left == 0) break;
        }
    }
    *out_len = pos;
    if (!out || out_cap < pos) return lvgpu_internal::set_error(LV_ERR_INVALID, "output buffer too small");
    // Pass 2: the fragment CRCs and the bytes, concurrently.  A fragment's CRC
    // covers payload bytes only (crc = mask(extend(type_crc[t], frag)),
    // log_writer.rs:123-125), so the GPU batch runs over the caller's payload
    // buffer -- its upload overlaps the host's layout copy instead of
    // following it.
    for (const auto &p : pads) std::memset(out + p.first, 0, p.second);
    std::vector<uint64_t> off(frags.size());
    std::vector<uint32_t> len(frags.size()), seed(frags.size()), crc(frags.size());
    uint32_t type_crc[5];
    for (uint8_t t = 0; t < 5; ++t) type_crc[t] = lv_crc32c_value(&t, 1);  // log_writer.rs:136-142
    uint64_t pay_end = 0;
    for (size_t i = 0; i < frags.size(); ++i) {
        const Frag &f = frags[i];
        off[i] = f.src;
        len[i] = f.len;
        seed[i] = type_crc[f.type];
        if (f.src + f.len > pay_end) pay_end = f.src + f.len;
    }
    int crc_rc = LV_OK;
    std::thread gpu;
    if (!frags.empty())
        gpu = std::thread([&] {
            static const uint8_t empty = 0;  // all records empty: nothing to read, a valid arena
            crc_rc = lv_crc32c_batch_host(pay_end ? payload : &empty, pay_end, off.data(), len.data(), seed.data(),
                                          crc.data(), frags.size(), LV_CRC_MASK, device);
        });
    // The payload copy is the host's share of the work (the whole log's
    // bytes): split it over up to 8 threads by fragment ranges of equal bytes.
    auto copy_range = [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) {
            const Frag &f = frags[i];
            if (f.len) std::memcpy(out + f.out_pos + kHeader, payload + f.src, f.len);
        }
    };
    unsigned nt = std::thread::hardware_concurrency();
    nt = nt == 0 ? 1 : (nt > 8 ? 8 : nt);
    if (pos < (8u << 20) || nt == 1 || frags.size() < 2 * nt) {
        copy_range(0, frags.size());
    } else {
        std::vector<std::thread> th;
        size_t lo = 0;
        for (unsigned t = 1; t <= nt && lo < frags.size(); ++t) {
            size_t hi = lo;
            const uint64_t until = pos * t / nt;  // fragment i ends near out byte until
            while (hi < frags.size() && (t == nt || frags[hi].out_pos < until)) ++hi;
            if (hi == lo) continue;
            th.emplace_back(copy_range, lo, hi);
            lo = hi;
        }
        if (lo < frags.size()) copy_range(lo, frags.size());
        for (auto &x : th) x.join();
    }
    if (gpu.joinable()) gpu.join();
    if (crc_rc) return crc_rc;
    for (size_t i = 0; i < frags.size(); ++i) {  // log_writer.rs:117-125
        uint8_t *h = out + frags[i].out_pos;
        h[0] = static_cast<uint8_t>(crc[i]);
        h[1] = static_cast<uint8_t>(crc[i] >> 8);
        h[2] = static_cast<uint8_t>(crc[i] >> 16);
        h[3] = static_cast<uint8_t>(crc[i] >> 24);
        h[4] = static_cast<uint8_t>(frags[i].len & 0xffu);
        h[5] = static_cast<uint8_t>(frags[i].len >> 8);
        h[6] = frags[i].type;
    }
    return LV_OK;
}

}  // extern "C"
