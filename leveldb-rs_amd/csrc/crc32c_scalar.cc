// Host scalar drop-ins for the reference's crc32c module (src/util/crc32c.rs).
// These serve single-record callers (the WAL writer emits one record at a
// time, log_writer.rs:112-134) where a kernel launch would cost 100x the
// checksum.  The GPU batch path (crc32c_batch.hip) never calls into here.
#include <nmmintrin.h>

#include <cstring>

#include "../../include/lvgpu/crc32c.h"
#include "crc32c_gf2.h"

namespace {

constexpr uint32_t kMaskDelta = 0xa282ead8u;  // crc32c.rs:23

struct SliceTables {
    uint32_t t[8][256];
    SliceTables() {
        uint32_t base[4][256];
        lvgpu::slice_tables(base);
        std::memcpy(t, base, sizeof(base));
        for (int k = 4; k < 8; ++k)
            for (int e = 0; e < 256; ++e) t[k][e] = (t[k - 1][e] >> 8) ^ t[0][t[k - 1][e] & 0xffu];
    }
};

const SliceTables &tables() {
    static const SliceTables tabs;  // thread-safe once-init (C++11 magic static)
    return tabs;
}

inline uint32_t load32(const uint8_t *p) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return v;  // x86 is little-endian, matching byteorder::LittleEndian
}

inline uint64_t load64(const uint8_t *p) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    return v;
}

bool have_sse42() {
    static const bool ok = __builtin_cpu_supports("sse4.2");
    return ok;
}

}  // namespace

extern "C" {

uint32_t lv_crc32c_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + kMaskDelta; }

uint32_t lv_crc32c_unmask(uint32_t masked_crc) {
    const uint32_t r = masked_crc - kMaskDelta;
    return (r >> 17) | (r << 15);
}

// Slice-by-8: fold 8 bytes per step through eight byte tables.
uint32_t lv_crc32c_extend_sw(uint32_t crc, const uint8_t *data, size_t n) {
    const auto &T = tables().t;
    uint32_t s = ~crc;
    for (; n >= 8; n -= 8, data += 8) {
        const uint32_t lo = s ^ load32(data);
        const uint32_t hi = load32(data + 4);
        s = T[7][lo & 0xff] ^ T[6][(lo >> 8) & 0xff] ^ T[5][(lo >> 16) & 0xff] ^ T[4][lo >> 24] ^
            T[3][hi & 0xff] ^ T[2][(hi >> 8) & 0xff] ^ T[1][(hi >> 16) & 0xff] ^ T[0][hi >> 24];
    }
    while (n--) s = T[0][(s ^ *data++) & 0xff] ^ (s >> 8);
    return ~s;
}

// SSE4.2 crc32 instruction over 8-byte words.  The CRC is independent of
// address alignment, so unlike crc32c.rs:97-102 no byte prologue is needed.
__attribute__((target("sse4.2"))) uint32_t lv_crc32c_extend_hw(uint32_t crc, const uint8_t *data,
                                                                size_t n) {
    uint64_t s = ~crc;
    for (; n >= 8; n -= 8, data += 8) s = _mm_crc32_u64(s, load64(data));
    uint32_t s32 = static_cast<uint32_t>(s);
    if (n >= 4) {
        s32 = _mm_crc32_u32(s32, load32(data));
        data += 4;
        n -= 4;
    }
    while (n--) s32 = _mm_crc32_u8(s32, *data++);
    return ~s32;
}

uint32_t lv_crc32c_extend(uint32_t crc, const uint8_t *data, size_t n) {
    return have_sse42() ? lv_crc32c_extend_hw(crc, data, n) : lv_crc32c_extend_sw(crc, data, n);
}

uint32_t lv_crc32c_value(const uint8_t *data, size_t n) { return lv_crc32c_extend(0, data, n); }

}  // extern "C"
