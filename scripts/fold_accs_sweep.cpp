// Fold-loop accumulator sweep for crc32c_cpu.cpp's fold_update: A zmm accumulators folded
// A*512 bits a step, single thread, at 4 KiB / 64 KiB / 4 MiB per call, beside the library's
// crc32c_value.  Built and run by scripts/cpu_fold_sweep.sh (CPU only).
#include <immintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <chrono>
#include <initializer_list>
extern "C" uint32_t crc32c_value(const void* p, size_t n);
static const uint32_t P = 0x82F63B78u;
static uint32_t mulmod(uint32_t a, uint32_t b) { uint32_t r = 0; for (int i = 0; i < 32; i++) { if (a & (0x80000000u >> i)) r ^= b; b = (b & 1) ? (b >> 1) ^ P : b >> 1; } return r; }
static uint32_t xpow(uint64_t n) { uint32_t r = 0x80000000u, x = 0x40000000u; while (n) { if (n & 1) r = mulmod(r, x); x = mulmod(x, x); n >>= 1; } return r; }
#define T __attribute__((target("avx512f,vpclmulqdq,pclmul,sse4.2")))
T static inline __m512i f5(__m512i x, __m512i k, __m512i d) { return _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(x, k, 0), _mm512_clmulepi64_epi128(x, k, 0x11), d, 0x96); }
T static inline __m512i K5(uint64_t D) { uint64_t lo = xpow(D + 31), hi = xpow(D - 33); return _mm512_set_epi64(hi, lo, hi, lo, hi, lo, hi, lo); }
static uint64_t KX[4][2];
T static inline __m128i f1(__m128i x, int D, __m128i d) { __m128i k = _mm_set_epi64x(KX[D / 128][1], KX[D / 128][0]); return _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x, k, 0), _mm_clmulepi64_si128(x, k, 0x11)), d); }
template <int A> T uint32_t run(uint32_t reg, const unsigned char* p, size_t n) {  // n multiple of 64*A, >= 64*A
    static const __m512i k = K5(512 * A), k1 = K5(512);
    __m512i x[A];
    for (int i = 0; i < A; i++) x[i] = _mm512_loadu_si512(p + 64 * i);
    x[0] = _mm512_xor_si512(x[0], _mm512_castsi128_si512(_mm_cvtsi32_si128((int)reg)));
    p += 64 * A; n -= 64 * A;
    while (n >= 64 * A) {
        for (int i = 0; i < A; i++) x[i] = f5(x[i], k, _mm512_loadu_si512(p + 64 * i));
        p += 64 * A; n -= 64 * A;
    }
    for (int i = 1; i < A; i++) x[i] = f5(x[i - 1], k1, x[i]);
    __m512i z = x[A - 1];
    __m128i v = _mm512_extracti32x4_epi32(z, 3);
    v = f1(_mm512_extracti32x4_epi32(z, 0), 384, v); v = f1(_mm512_extracti32x4_epi32(z, 1), 256, v); v = f1(_mm512_extracti32x4_epi32(z, 2), 128, v);
    uint64_t l = _mm_crc32_u64(0, (uint64_t)_mm_cvtsi128_si64(v)); l = _mm_crc32_u64(l, (uint64_t)_mm_extract_epi64(v, 1));
    return (uint32_t)l;
}
T static inline uint32_t mm(uint32_t a, uint32_t b) {  // a*b mod P, one clmul
    const __m128i p = _mm_clmulepi64_si128(_mm_cvtsi32_si128((int)a), _mm_cvtsi32_si128((int)b), 0x00);
    const uint64_t v = (uint64_t)_mm_cvtsi128_si64(p) << 1;
    return _mm_crc32_u32(0, (uint32_t)v) ^ (uint32_t)(v >> 32);
}
// hybrid: superblocks of M steps; a step folds 512 B (8 zmm) while three crc32q streams take
// 8Q bytes each from the superblock's last third; superblocks chain by one multiply
template <int Q, int M> struct Hy {
    static constexpr size_t C = 8 * Q * M, F = 512 * M, SB = F + 3 * C;
    uint32_t kc1, kc2, kc3, ksb;
    __m512i k, k1;
    T Hy() { kc1 = xpow(8 * C); kc2 = xpow(16 * C); kc3 = xpow(24 * C); ksb = xpow(8 * SB); k = K5(4096); k1 = K5(512); }
    T uint32_t raw0(const unsigned char* p) const {
        __m512i x[8];
        for (int i = 0; i < 8; i++) x[i] = _mm512_loadu_si512(p + 64 * i);
        const unsigned char* s = p + F;
        uint64_t a = 0, b = 0, c = 0;
        for (int q = 0; q < Q; q++) {
            uint64_t u, v, w; memcpy(&u, s + 8 * q, 8); memcpy(&v, s + C + 8 * q, 8); memcpy(&w, s + 2 * C + 8 * q, 8);
            a = _mm_crc32_u64(a, u); b = _mm_crc32_u64(b, v); c = _mm_crc32_u64(c, w);
        }
        s += 8 * Q;
        for (int m = 1; m < M; m++) {
            p += 512;
            for (int i = 0; i < 8; i++) x[i] = f5(x[i], k, _mm512_loadu_si512(p + 64 * i));
            for (int q = 0; q < Q; q++) {
                uint64_t u, v, w; memcpy(&u, s + 8 * q, 8); memcpy(&v, s + C + 8 * q, 8); memcpy(&w, s + 2 * C + 8 * q, 8);
                a = _mm_crc32_u64(a, u); b = _mm_crc32_u64(b, v); c = _mm_crc32_u64(c, w);
            }
            s += 8 * Q;
        }
        for (int i = 1; i < 8; i++) x[i] = f5(x[i - 1], k1, x[i]);
        __m512i z = x[7];
        __m128i v = _mm512_extracti32x4_epi32(z, 3);
        v = f1(_mm512_extracti32x4_epi32(z, 0), 384, v); v = f1(_mm512_extracti32x4_epi32(z, 1), 256, v); v = f1(_mm512_extracti32x4_epi32(z, 2), 128, v);
        uint64_t l = _mm_crc32_u64(0, (uint64_t)_mm_cvtsi128_si64(v)); l = _mm_crc32_u64(l, (uint64_t)_mm_extract_epi64(v, 1));
        return mm(kc3, (uint32_t)l) ^ mm(kc2, (uint32_t)a) ^ mm(kc1, (uint32_t)b) ^ (uint32_t)c;
    }
    T uint32_t run(uint32_t reg, const unsigned char* p, size_t n) const {  // the tail by crc32q
        while (n >= SB) { reg = mm(ksb, reg) ^ raw0(p); p += SB; n -= SB; }
        if (n >= 256) { const size_t f = n / 256 * 256; reg = ::run<4>(reg, p, f); p += f; n -= f; }
        uint64_t l = reg;
        while (n >= 8) { uint64_t u; memcpy(&u, p, 8); l = _mm_crc32_u64(l, u); p += 8; n -= 8; }
        while (n--) l = _mm_crc32_u8((uint32_t)l, *p++);
        return (uint32_t)l;
    }
};
// one region split per call: the fold takes the first 512*M bytes, the streams 8QM each after it,
// M = n / (512 + 24Q); the shift constants computed per call (x^(8*8QM) by squaring)
static uint32_t XT[64];
T static uint32_t xp(uint64_t n) { uint32_t r = 0x80000000u; for (int k = 0; n; k++, n >>= 1) if (n & 1) r = mm(r, XT[k]); return r; }
template <int Q> T uint32_t one(uint32_t reg, const unsigned char* p, size_t n) {
    static const __m512i k = K5(4096), k1 = K5(512);
    const size_t M = n / (512 + 24 * Q);
    if (M < 2) return ::run<4>(reg, p, n / 256 * 256);  // (sweep sizes only)
    const size_t C = 8 * Q * M, F = 512 * M;
    __m512i x[8];
    for (int i = 0; i < 8; i++) x[i] = _mm512_loadu_si512(p + 64 * i);
    x[0] = _mm512_xor_si512(x[0], _mm512_castsi128_si512(_mm_cvtsi32_si128((int)reg)));
    const unsigned char* s = p + F;
    uint64_t a = 0, b = 0, c = 0;
    for (int q = 0; q < Q; q++) {
        uint64_t u, v, w; memcpy(&u, s + 8 * q, 8); memcpy(&v, s + C + 8 * q, 8); memcpy(&w, s + 2 * C + 8 * q, 8);
        a = _mm_crc32_u64(a, u); b = _mm_crc32_u64(b, v); c = _mm_crc32_u64(c, w);
    }
    s += 8 * Q;
    const unsigned char* f = p;
    for (size_t m = 1; m < M; m++) {
        f += 512;
        for (int i = 0; i < 8; i++) x[i] = f5(x[i], k, _mm512_loadu_si512(f + 64 * i));
        for (int q = 0; q < Q; q++) {
            uint64_t u, v, w; memcpy(&u, s + 8 * q, 8); memcpy(&v, s + C + 8 * q, 8); memcpy(&w, s + 2 * C + 8 * q, 8);
            a = _mm_crc32_u64(a, u); b = _mm_crc32_u64(b, v); c = _mm_crc32_u64(c, w);
        }
        s += 8 * Q;
    }
    const uint32_t kc1 = xp(8 * C), kc2 = mm(kc1, kc1), kc3 = mm(kc2, kc1);
    for (int i = 1; i < 8; i++) x[i] = f5(x[i - 1], k1, x[i]);
    __m512i z = x[7];
    __m128i v = _mm512_extracti32x4_epi32(z, 3);
    v = f1(_mm512_extracti32x4_epi32(z, 0), 384, v); v = f1(_mm512_extracti32x4_epi32(z, 1), 256, v); v = f1(_mm512_extracti32x4_epi32(z, 2), 128, v);
    uint64_t l = _mm_crc32_u64(0, (uint64_t)_mm_cvtsi128_si64(v)); l = _mm_crc32_u64(l, (uint64_t)_mm_extract_epi64(v, 1));
    reg = mm(kc3, (uint32_t)l) ^ mm(kc2, (uint32_t)a) ^ mm(kc1, (uint32_t)b) ^ (uint32_t)c;
    p += F + 3 * C; n -= F + 3 * C;
    if (n >= 256) { const size_t t = n / 256 * 256; reg = ::run<4>(reg, p, t); p += t; n -= t; }
    l = reg;
    while (n >= 8) { uint64_t u; memcpy(&u, p, 8); l = _mm_crc32_u64(l, u); p += 8; n -= 8; }
    while (n--) l = _mm_crc32_u8((uint32_t)l, *p++);
    return (uint32_t)l;
}
template <int Q> void obench(const unsigned char* buf) {
    for (size_t n : {4096ul, 16384ul, 65536ul, 4ul << 20}) {
        if (~one<Q>(~0u, buf, n) != crc32c_value(buf, n)) { printf("one Q=%d n=%zu WRONG\n", Q, n); return; }
        long reps = (8l << 30) / n; uint32_t s = 0;
        auto t0 = std::chrono::steady_clock::now();
        for (long r = 0; r < reps; r++) s += one<Q>(r, buf, n);
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        printf("one Q=%2d n=%7zu %6.1f GiB/s (%u)\n", Q, n, reps * (double)n / dt / (1 << 30), s);
    }
}
template <int Q, int M> void hbench(const unsigned char* buf) {
    static const Hy<Q, M> h;
    for (size_t n : {65536ul, 4ul << 20}) {
        if (~h.run(~0u, buf, n) != crc32c_value(buf, n)) { printf("Q=%d M=%d WRONG\n", Q, M); return; }
        long reps = (8l << 30) / n; uint32_t s = 0;
        auto t0 = std::chrono::steady_clock::now();
        for (long r = 0; r < reps; r++) s += h.run(r, buf, n);
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        printf("hybrid Q=%2d M=%2d SB=%6zu n=%7zu %6.1f GiB/s (%u)\n", Q, M, Hy<Q, M>::SB, n, reps * (double)n / dt / (1 << 30), s);
    }
}
template <int A> void bench(const unsigned char* buf) {
    if (~run<A>(~0u, buf, 65536) != crc32c_value(buf, 65536)) { printf("A=%d WRONG\n", A); return; }
    for (size_t n : {4096ul, 65536ul, 4ul << 20}) {
        long reps = (8l << 30) / n; uint32_t s = 0;
        auto t0 = std::chrono::steady_clock::now();
        for (long r = 0; r < reps; r++) s += run<A>(r, buf, n);
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        printf("A=%2d n=%7zu %6.1f GiB/s (%u)\n", A, n, reps * (double)n / dt / (1 << 30), s);
    }
}
int main() {
    for (int i = 1; i < 4; i++) KX[i][0] = xpow(128 * i + 31), KX[i][1] = xpow(128 * i - 33);
    size_t N = 4 << 20; unsigned char* buf = (unsigned char*)aligned_alloc(64, N);
    for (size_t i = 0; i < N; i++) buf[i] = rand();
    XT[0] = 0x40000000u; for (int i = 1; i < 64; i++) XT[i] = mulmod(XT[i - 1], XT[i - 1]);
    bench<8>(buf); obench<10>(buf);
    for (size_t n : {4096ul, 8192ul, 16384ul, 65536ul, 1ul << 20, 4ul << 20}) {
        long reps = (8l << 30) / n; uint32_t s = 0;
        auto t0 = std::chrono::steady_clock::now();
        for (long r = 0; r < reps; r++) s += crc32c_value(buf, n);
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        printf("lib  n=%7zu %6.1f GiB/s (%u)\n", n, reps * (double)n / dt / (1 << 30), s);
    }
}
