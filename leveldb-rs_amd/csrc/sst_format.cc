// Table-format codecs (src/table/format.rs) behind include/lvgpu/table.h.
#include <cstring>

#include "../../include/lvgpu/crc32c.h"
#include "../../include/lvgpu/table.h"
#include "lv_internal.h"

namespace {

// encode_varint_64, coding.rs:144-153
size_t put_varint64(uint8_t *dst, uint64_t v) {
    size_t i = 0;
    while (v & ~0x7full) {
        dst[i++] = static_cast<uint8_t>((v & 0x7f) | 0x80);
        v >>= 7;
    }
    dst[i++] = static_cast<uint8_t>(v);
    return i;
}

// decode_varint_64_limit, coding.rs:223-241: at most 10 bytes (shift <= 63)
bool get_varint64(const uint8_t *src, size_t n, uint64_t *v, size_t *used) {
    uint64_t r = 0;
    size_t i = 0;
    for (unsigned shift = 0; shift <= 63 && i < n; shift += 7) {
        const uint8_t b = src[i++];
        r |= static_cast<uint64_t>(b & 0x7f) << shift;
        if (!(b & 0x80)) {
            *v = r;
            *used = i;
            return true;
        }
    }
    return false;
}

}  // namespace

extern "C" {

size_t lv_sst_block_handle_encode(uint64_t offset, uint64_t size, uint8_t *dst) {
    const size_t a = put_varint64(dst, offset);
    return a + put_varint64(dst + a, size);
}

int lv_sst_block_handle_decode(const uint8_t *src, size_t n, uint64_t *offset, uint64_t *size, size_t *consumed) {
    size_t a = 0, b = 0;
    uint64_t o = 0, s = 0;
    if (!src || !get_varint64(src, n, &o, &a) || !get_varint64(src + a, n - a, &s, &b))
        return lvgpu_internal::set_error(LV_ERR_CORRUPTION, "bad handle");  // format.rs:43-46
    if (offset) *offset = o;
    if (size) *size = s;
    if (consumed) *consumed = a + b;
    return LV_OK;
}

void lv_sst_footer_encode(uint64_t metaindex_offset, uint64_t metaindex_size, uint64_t index_offset,
                          uint64_t index_size, uint8_t *out) {
    std::memset(out, 0, LV_SST_FOOTER_SIZE);
    size_t p = lv_sst_block_handle_encode(metaindex_offset, metaindex_size, out);
    lv_sst_block_handle_encode(index_offset, index_size, out + p);
    for (int i = 0; i < 8; ++i) out[40 + i] = static_cast<uint8_t>(LV_SST_MAGIC >> (8 * i));  // format.rs:77-78
}

int lv_sst_footer_decode(const uint8_t *src, size_t n, uint64_t handles[4]) {
    if (!src || n < LV_SST_FOOTER_SIZE || !handles)
        return lvgpu_internal::set_error(LV_ERR_INVALID, "footer needs 48 bytes");
    uint64_t magic = 0;
    for (int i = 7; i >= 0; --i) magic = (magic << 8) | src[LV_SST_FOOTER_SIZE - 8 + i];
    if (magic != LV_SST_MAGIC)  // format.rs:85-93
        return lvgpu_internal::set_error(LV_ERR_CORRUPTION, "not a sstable (bad magic number)");
    size_t a = 0, b = 0;
    if (int rc = lv_sst_block_handle_decode(src, n, &handles[0], &handles[1], &a)) return rc;
    if (int rc = lv_sst_block_handle_decode(src + a, n - a, &handles[2], &handles[3], &b)) return rc;
    return LV_OK;
}

}  // extern "C"
