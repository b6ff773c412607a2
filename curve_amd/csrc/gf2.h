// curve_amd/csrc/gf2.h -- GF(2)[x] / P(x) arithmetic for CRC-32C, shared by the
// CPU primitive (crc32c_cpu.cpp) and the device-table builder (engine.cpp).
//
// Representation: reflected, as the CRC register holds it.  Bit 31 of a word is
// the coefficient of x^0, bit 0 the coefficient of x^31, P = 0x82F63B78 (x^32
// implied).  Feeding n zero bytes into a raw CRC register is multiplication by
// x^(8n) mod P, which is what every combine / shift / device table below uses.
#pragma once
#include <stdint.h>

namespace cc {

constexpr uint32_t kPoly = 0x82F63B78u;
constexpr uint32_t kOne = 0x80000000u;  // the polynomial "1"

// a(x) * b(x) mod P(x).
inline uint32_t mulmod(uint32_t a, uint32_t b) {
    uint32_t prod = 0;
    for (int i = 0; i < 32; i++) {
        if (a & (kOne >> i)) prod ^= b;
        b = (b >> 1) ^ (kPoly & (0u - (b & 1u)));  // b *= x
    }
    return prod;
}

// b(x) / x mod P (inverse of the "b *= x" step: bit 31 of b*x is bit 0 of b
// because P's x^0 coefficient -- bit 31 of kPoly -- is 1).
inline uint32_t div_x(uint32_t b) {
    return (b & 0x80000000u) ? (((b ^ kPoly) << 1) | 1u) : (b << 1);
}

// x^(-8t) mod P.
inline uint32_t div_x8(uint32_t r) {  // r * x^-8
    for (int i = 0; i < 8; i++) r = div_x(r);
    return r;
}
inline uint32_t xinv_bytes(uint32_t t) {
    uint32_t r = kOne;
    for (uint32_t i = 0; i < 8 * t; i++) r = div_x(r);
    return r;
}

// x^(2^k) mod P for k = 0..63, built by repeated squaring.
struct X2kTable {
    uint32_t t[64];
    X2kTable() {
        t[0] = kOne >> 1;  // x^1
        for (int k = 1; k < 64; k++) t[k] = mulmod(t[k - 1], t[k - 1]);
    }
};
inline const X2kTable& x2k() {
    static const X2kTable tab;
    return tab;
}

// x^n mod P.
inline uint32_t xpow(uint64_t n) {
    uint32_t r = kOne;
    const X2kTable& T = x2k();
    for (int k = 0; n; k++, n >>= 1)
        if (n & 1u) r = mulmod(r, T.t[k]);
    return r;
}

// Raw register after feeding nbytes zero bytes.
inline uint32_t shift_bytes(uint32_t reg, uint64_t nbytes) {
    if (reg == 0 || nbytes == 0) return reg;
    // x^(8n): 8n may exceed 2^64 only for absurd n; n < 2^61 here.
    return mulmod(xpow(nbytes << 3), reg);
}

}  // namespace cc
