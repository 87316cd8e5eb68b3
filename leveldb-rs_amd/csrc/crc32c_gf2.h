// GF(2) algebra for CRC-32C (reflected Castagnoli, poly 0x82f63b78) used to
// build the device lookup tables.  Host-only, header-only.
//
// Notation (DESIGN.md "CRC algebra"):
//   R(s, D)   raw register update over bytes D from state s (no pre/post xor);
//             extend(c, D) = R(c ^ ~0, D) ^ ~0           (crc32c.rs:42-51, :65-84)
//   Shift_n   R(s, 0^n): s * x^(8n) mod P — a GF(2)-linear map on 32 bits
//   T_k[e]    slice table "byte e followed by k zero bytes" (crc32c.rs:25-38)
// Linearity: R(s, A||B) = Shift_|B|(R(s, A)) ^ R(0, B).
#pragma once
#include <array>
#include <cstdint>

namespace lvgpu {

constexpr uint32_t kPoly = 0x82f63b78u;  // crc32c.rs:22

// A 32x32 GF(2) matrix stored as 32 column images: M * v = XOR of col[j]
// over the set bits j of v.
struct Gf2Mat {
    std::array<uint32_t, 32> col{};
    uint32_t apply(uint32_t v) const {
        uint32_t r = 0;
        for (int j = 0; j < 32; ++j)
            if (v >> j & 1u) r ^= col[j];
        return r;
    }
    Gf2Mat then(const Gf2Mat& next) const {  // next ∘ this
        Gf2Mat m;
        for (int j = 0; j < 32; ++j) m.col[j] = next.apply(col[j]);
        return m;
    }
};

// One zero-byte step: s -> (s >> 8) ^ T0[s & 0xff], done bit-serially.
inline uint32_t zero_byte_step(uint32_t s) {
    for (int b = 0; b < 8; ++b) s = (s & 1u) ? (s >> 1) ^ kPoly : (s >> 1);
    return s;
}

inline Gf2Mat shift_matrix(uint64_t nbytes) {
    Gf2Mat one, acc;
    for (int j = 0; j < 32; ++j) {
        one.col[j] = zero_byte_step(1u << j);
        acc.col[j] = 1u << j;  // identity
    }
    while (nbytes) {  // square-and-multiply over the byte count
        if (nbytes & 1u) acc = acc.then(one);
        one = one.then(one);
        nbytes >>= 1;
    }
    return acc;
}

// T_k for k = 0..3: T_0 is the bit-reflected byte table, T_k[e] = Shift_k(T_0[e]).
inline void slice_tables(uint32_t out[4][256]) {
    for (uint32_t e = 0; e < 256; ++e) {
        uint32_t c = e;
        for (int b = 0; b < 8; ++b) c = (c & 1u) ? (c >> 1) ^ kPoly : (c >> 1);
        out[0][e] = c;
    }
    for (int k = 1; k < 4; ++k)
        for (int e = 0; e < 256; ++e)
            out[k][e] = (out[k - 1][e] >> 8) ^ out[0][out[k - 1][e] & 0xffu];
}

// Byte-position tables of a shift: S[j][e] = Shift_n(e << 8j), so that
// Shift_n(v) = S[0][v.b0] ^ S[1][v.b1] ^ S[2][v.b2] ^ S[3][v.b3].
inline void shift_tables(uint64_t nbytes, uint32_t out[4][256]) {
    Gf2Mat m = shift_matrix(nbytes);
    for (int j = 0; j < 4; ++j)
        for (uint32_t e = 0; e < 256; ++e) out[j][e] = m.apply(e << (8 * j));
}

}  // namespace lvgpu
