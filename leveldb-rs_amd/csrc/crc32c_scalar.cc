// Host scalar drop-ins for the reference's crc32c module (src/util/crc32c.rs).
// These serve single-record callers (the WAL writer emits one record at a
// time, log_writer.rs:112-134) where a kernel launch would cost 100x the
// checksum.  The GPU batch path (blocks.hip, classes.hip, ...) never calls into here.
#include <nmmintrin.h>

#include <cstring>

#include "../../include/lvgpu/crc32c.h"
#include "crc32c_gf2.h"

namespace {

constexpr uint32_t kMaskDelta = 0xa282ead8u;  // crc32c.rs:23

// Sixteen byte tables: t[k][e] = R(e, 0^k) — the CRC of byte e followed by
// k zero bytes — so a 16-byte step is sixteen independent lookups.
struct SliceTables {
    uint32_t t[16][256];
    SliceTables() {
        uint32_t base[4][256];
        lvgpu::slice_tables(base);
        std::memcpy(t, base, sizeof(base));
        for (int k = 4; k < 16; ++k)
            for (int e = 0; e < 256; ++e) t[k][e] = (t[k - 1][e] >> 8) ^ t[0][t[k - 1][e] & 0xffu];
    }
};

const SliceTables g_tabs;  // built at load time, read-only afterwards

// Three-stream hardware path: a superblock of 3 x kLane bytes runs three
// independent crc32q chains (the instruction's latency is 3 cycles, its
// throughput 1/cycle) and merges them by linearity,
// R(s, A||B||C) = Shift_2L(R(s, A)) ^ Shift_L(R(0, B)) ^ R(0, C).
constexpr size_t kLane = 512;
struct ShiftPair {
    uint32_t l1[4][256], l2[4][256];  // Shift_kLane, Shift_2kLane as byte tables
    ShiftPair() {
        lvgpu::shift_tables(kLane, l1);
        lvgpu::shift_tables(2 * kLane, l2);
    }
};
const ShiftPair g_shift;

inline uint32_t apply(const uint32_t (&t)[4][256], uint32_t s) {
    return t[0][s & 0xff] ^ t[1][(s >> 8) & 0xff] ^ t[2][(s >> 16) & 0xff] ^ t[3][s >> 24];
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

// extend(s, A||B) = ~R(~s, A||B) = ~(Shift_|B|(R(~s, A)) ^ R(0, B)), and with
// R(~s, A) = ~crc_a, R(0, B) = ~crc_b ^ Shift_|B|(~0) this is
// Shift_|B|(crc_a) ^ crc_b (GF(2)-linear Shift).
uint32_t lv_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
    return lvgpu::shift_matrix(len_b).apply(crc_a) ^ crc_b;
}

// Software path (the twin of crc32c.rs:65-84, same value): slice-by-16, the
// state xored into the first word, the other 12 bytes indexed directly.
uint32_t lv_crc32c_extend_sw(uint32_t crc, const uint8_t *data, size_t n) {
    const uint32_t(*T)[256] = g_tabs.t;
    uint32_t s = ~crc;
    for (; n >= 16; n -= 16, data += 16) {
        const uint32_t w = s ^ load32(data);
        s = T[15][w & 0xff] ^ T[14][(w >> 8) & 0xff] ^ T[13][(w >> 16) & 0xff] ^ T[12][w >> 24] ^
            T[11][data[4]] ^ T[10][data[5]] ^ T[9][data[6]] ^ T[8][data[7]] ^
            T[7][data[8]] ^ T[6][data[9]] ^ T[5][data[10]] ^ T[4][data[11]] ^
            T[3][data[12]] ^ T[2][data[13]] ^ T[1][data[14]] ^ T[0][data[15]];
    }
    while (n--) s = T[0][(s ^ *data++) & 0xff] ^ (s >> 8);
    return ~s;
}

// SSE4.2 crc32 instruction over 8-byte words (the twin of crc32c.rs:86-118,
// same value).  The CRC is independent of address alignment, so no byte
// prologue is needed; long buffers run three chains per superblock.
__attribute__((target("sse4.2"))) uint32_t lv_crc32c_extend_hw(uint32_t crc, const uint8_t *data,
                                                                size_t n) {
    uint64_t s = ~crc;
    for (; n >= 3 * kLane; n -= 3 * kLane, data += 3 * kLane) {
        uint64_t a = s, b = 0, c = 0;
        for (size_t k = 0; k < kLane; k += 8) {
            a = _mm_crc32_u64(a, load64(data + k));
            b = _mm_crc32_u64(b, load64(data + kLane + k));
            c = _mm_crc32_u64(c, load64(data + 2 * kLane + k));
        }
        s = apply(g_shift.l2, static_cast<uint32_t>(a)) ^ apply(g_shift.l1, static_cast<uint32_t>(b)) ^
            static_cast<uint32_t>(c);
    }
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
