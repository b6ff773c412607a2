// curve_amd/csrc/crc32c_cpu.cpp -- the CPU side of the C ABI: the CRC32C
// primitive that replaces curve::common::CRC32 (src/common/crc32.h:40-55) for
// small, latency-bound buffers (metapage header CRC, chunkserver_chunkfile.cpp:86;
// conf-epoch CRC, conf_epoch_file.cpp:148-164; ...) plus the GF(2) combine
// algebra.  Bulk page data goes to the GPU (engine.cpp); this file is not a
// fallback for it.
//
// Large buffers run three independent crc32q streams (the x86 crc32 instruction
// has 3-cycle latency, 1/cycle throughput) and merge them with x^(8n) mod P
// multiplications; results are bit-identical to butil's single stream.  On
// CPUs with VPCLMULQDQ (checked at run time), buffers of 256 bytes and more
// fold instead (fold_update below), ~3x the 3-way loop's rate.
#include <immintrin.h>
#include <nmmintrin.h>
#include <stdlib.h>
#include <string.h>
#include <wmmintrin.h>

#include <algorithm>
#include <vector>

#include "../../include/curve_crc.h"
#include "gf2.h"

namespace {

// Block sizes of the 3-way loop, largest first: a round hashes 3 blocks of b
// bytes as three independent crc32q chains and merges them with two
// shift-by-constant table lookups.  The small sizes make 4 KiB pages (3 x 1360
// + 16) and other short buffers 3-way too.
constexpr size_t kBlocks[] = {4096, 2048, 1360, 1024, 680, 512, 336, 256, 168};
constexpr int kNumBlocks = sizeof(kBlocks) / sizeof(kBlocks[0]);

// x^(8b) and x^(16b) as 4x256 byte tables per block size: shift-by-constant
// in 4 lookups instead of a 32-step multiply.
struct ShiftTables {
    uint32_t t1[kNumBlocks][4][256];  // register * x^(8*b)
    uint32_t t2[kNumBlocks][4][256];  // register * x^(16*b)
    ShiftTables() {
        for (int i = 0; i < kNumBlocks; i++) {
            const uint32_t m1 = cc::xpow(8ull * kBlocks[i]);
            const uint32_t m2 = cc::xpow(16ull * kBlocks[i]);
            for (int k = 0; k < 4; k++)
                for (uint32_t v = 0; v < 256; v++) {
                    t1[i][k][v] = cc::mulmod(m1, v << (8 * k));
                    t2[i][k][v] = cc::mulmod(m2, v << (8 * k));
                }
        }
    }
    static inline uint32_t apply(const uint32_t (&t)[4][256], uint32_t r) {
        return t[0][r & 0xFF] ^ t[1][(r >> 8) & 0xFF] ^ t[2][(r >> 16) & 0xFF] ^ t[3][r >> 24];
    }
};
const ShiftTables& shift_tables() {
    static const ShiftTables s;
    return s;
}

// a * b mod P in the reflected domain with one carry-less multiply: the
// 63-bit product, shifted to 64-bit reflected form, reduced by the crc32
// instruction (low word) and XORed with the high word.  Equal to cc::mulmod
// (the 32-step bitwise multiply, tests/test_cpu_primitive.py), ~40x faster.
inline uint32_t mulmod_clmul(uint32_t a, uint32_t b) {
    const __m128i p = _mm_clmulepi64_si128(_mm_cvtsi32_si128((int)a), _mm_cvtsi32_si128((int)b), 0x00);
    const uint64_t v = (uint64_t)_mm_cvtsi128_si64(p) << 1;
    return _mm_crc32_u32(0, (uint32_t)v) ^ (uint32_t)(v >> 32);
}

// x^n mod P by the x^(2^k) table, multiplied with mulmod_clmul.
inline uint32_t xpow_clmul(uint64_t n) {
    uint32_t r = cc::kOne;
    const cc::X2kTable& T = cc::x2k();
    for (int k = 0; n; k++, n >>= 1)
        if (n & 1u) r = mulmod_clmul(r, T.t[k]);
    return r;
}

inline uint32_t shift_clmul(uint32_t reg, uint64_t nbytes) {
    if (reg == 0 || nbytes == 0) return reg;
    return mulmod_clmul(xpow_clmul(nbytes << 3), reg);
}

inline uint64_t load64(const unsigned char* p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}

template <size_t B>
inline uint64_t three_way(uint64_t l, const unsigned char* p, const ShiftTables& st, int i) {
    uint64_t a = l, b = 0, c = 0;
    for (size_t k = 0; k < B; k += 8) {
        a = _mm_crc32_u64(a, load64(p + k));
        b = _mm_crc32_u64(b, load64(p + B + k));
        c = _mm_crc32_u64(c, load64(p + 2 * B + k));
    }
    return ShiftTables::apply(st.t2[i], static_cast<uint32_t>(a)) ^
           ShiftTables::apply(st.t1[i], static_cast<uint32_t>(b)) ^ static_cast<uint32_t>(c);
}

// Carry-less folding over 512-bit registers (VPCLMULQDQ, AVX-512), for CPUs
// that have it (the MI355X hosts' EPYCs do): the buffer is cut into 16-byte
// lanes; a lane's bits are moved forward by D bits with two 64x64 carry-less
// multiplies by x^(D+31) (low qword) and x^(D-33) (high qword) -- the reflected
// domain's offsets, found by exhaustive search against the bitwise CRC and
// pinned by tests/test_cpu_primitive.py -- and XORed onto the lane D bits later.
// Eight accumulators fold 512 bytes a step; at the end the accumulators fold
// into one 16-byte lane, whose CRC (register 0) is the register of the whole.
// The fold issues two 512-bit carry-less multiplies per 64 bytes, and on the
// hosts measured that port, not the loads, sets the rate (4, 8 and 16
// accumulators all ran at ~74 GiB/s, scripts/fold_accs_sweep.cpp).  The crc32
// instruction runs on another port, so a split runs both: of M steps of
// kStep bytes, the fold takes the first 512*M bytes and three crc32q streams
// take kStreamQ qwords a step each from the three stretches after them; the
// four registers are joined by x^(8*stretch) multiplies.  kStreamQ = 10 was the
// best of 6..16 on the MI355X host (EPYC 9575F): 98 vs 60-74 GiB/s at 64 KiB.
// Splits of kSplitMinSteps..kSplitMaxSteps steps take precomputed constants.
constexpr int kStreamQ = 10;
constexpr size_t kStep = 512 + 3 * 8 * kStreamQ;
constexpr size_t kSplitMinSteps = 8, kSplitMaxSteps = 64;

struct FoldKeys {
    uint64_t k[5][2];  // distances 4096, 2048, 512, 384, 256 bits; 128 below
    uint64_t k128[2];
    uint32_t split[kSplitMaxSteps + 1][3];  // x^(8*s), x^(16*s), x^(24*s) for the stretch s of M steps
    FoldKeys() {
        const uint64_t d[5] = {4096, 2048, 512, 384, 256};
        for (int i = 0; i < 5; i++) k[i][0] = cc::xpow(d[i] + 31), k[i][1] = cc::xpow(d[i] - 33);
        k128[0] = cc::xpow(128 + 31), k128[1] = cc::xpow(128 - 33);
        for (size_t m = 0; m <= kSplitMaxSteps; m++)
            for (int j = 0; j < 3; j++) split[m][j] = cc::xpow(64ull * kStreamQ * m * (j + 1));
    }
};
const FoldKeys& fold_keys() {
    static const FoldKeys s;
    return s;
}

constexpr size_t kFoldMin = 256;  // below this the crc32q paths are as fast

#define CC_FOLD_TARGET __attribute__((target("avx512f,vpclmulqdq,pclmul,sse4.2")))

CC_FOLD_TARGET inline __m512i fold512(__m512i x, __m512i k, __m512i next) {
    // (x.lo * k.lo) ^ (x.hi * k.hi) ^ next, per 128-bit lane
    return _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(x, k, 0x00), _mm512_clmulepi64_epi128(x, k, 0x11), next,
                                     0x96);
}

CC_FOLD_TARGET inline __m128i fold128(__m128i x, const uint64_t (&k)[2], __m128i next) {
    const __m128i kk = _mm_set_epi64x((long long)k[1], (long long)k[0]);
    return _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x, kk, 0x00), _mm_clmulepi64_si128(x, kk, 0x11)), next);
}

CC_FOLD_TARGET inline __m512i keys512(const uint64_t (&k)[2]) {
    return _mm512_set_epi64((long long)k[1], (long long)k[0], (long long)k[1], (long long)k[0], (long long)k[1],
                            (long long)k[0], (long long)k[1], (long long)k[0]);
}

CC_FOLD_TARGET inline uint32_t reduce8(__m512i (&x)[8], const FoldKeys& fk) {
    // eight accumulators (x[7] the last 64 bytes) to one register: fold each onto
    // the next, then the last zmm's four lanes onto its top lane
    const __m512i k512 = keys512(fk.k[2]);
    for (int i = 1; i < 8; i++) x[i] = fold512(x[i - 1], k512, x[i]);
    __m128i v = _mm512_extracti32x4_epi32(x[7], 3);
    v = fold128(_mm512_extracti32x4_epi32(x[7], 0), fk.k[3], v);
    v = fold128(_mm512_extracti32x4_epi32(x[7], 1), fk.k[4], v);
    v = fold128(_mm512_extracti32x4_epi32(x[7], 2), fk.k128, v);
    const uint64_t l = _mm_crc32_u64(0, (uint64_t)_mm_cvtsi128_si64(v));
    return static_cast<uint32_t>(_mm_crc32_u64(l, (uint64_t)_mm_extract_epi64(v, 1)));
}

// raw register update over [p, p + M*kStep), M >= kSplitMinSteps
CC_FOLD_TARGET uint32_t fold_split(uint32_t reg, const unsigned char* p, size_t M) {
    const FoldKeys& fk = fold_keys();
    const size_t C = 8 * kStreamQ * M;  // one stream's stretch
    const unsigned char* s = p + 512 * M;
    __m512i x[8];
    for (int i = 0; i < 8; i++) x[i] = _mm512_loadu_si512(p + 64 * i);
    x[0] = _mm512_xor_si512(x[0], _mm512_castsi128_si512(_mm_cvtsi32_si128((int)reg)));
    uint64_t a = 0, b = 0, c = 0;
    const __m512i k4096 = keys512(fk.k[0]);
    for (size_t m = 0;;) {
        for (int q = 0; q < kStreamQ; q++) {
            a = _mm_crc32_u64(a, load64(s + 8 * q));
            b = _mm_crc32_u64(b, load64(s + C + 8 * q));
            c = _mm_crc32_u64(c, load64(s + 2 * C + 8 * q));
        }
        s += 8 * kStreamQ;
        if (++m == M) break;
        p += 512;
        for (int i = 0; i < 8; i++) x[i] = fold512(x[i], k4096, _mm512_loadu_si512(p + 64 * i));
    }
    uint32_t k[3];
    if (M <= kSplitMaxSteps) {
        k[0] = fk.split[M][0], k[1] = fk.split[M][1], k[2] = fk.split[M][2];
    } else {  // ~20 multiplies, against >= 48 KiB of data
        k[0] = xpow_clmul(8 * C), k[1] = mulmod_clmul(k[0], k[0]), k[2] = mulmod_clmul(k[1], k[0]);
    }
    return mulmod_clmul(k[2], reduce8(x, fk)) ^ mulmod_clmul(k[1], static_cast<uint32_t>(a)) ^
           mulmod_clmul(k[0], static_cast<uint32_t>(b)) ^ static_cast<uint32_t>(c);
}

// The split pays where crc32 and the carry-less multiply issue on different
// pipes (AMD Zen: +30 % at 64 KiB on the EPYC 9575F); on the Intel Xeon of the
// build container the split ran slower than the fold alone, so it stays off there.
// CURVE_CRC_FOLD_SPLIT=1 / =0 forces it on / off (tests run every path on any host).
bool split_pays() {
    static const bool on = [] {
        const char* f = getenv("CURVE_CRC_FOLD_SPLIT");
        if (f && f[0]) return f[0] != '0';
        __builtin_cpu_init();
        return __builtin_cpu_is("amd") != 0;
    }();
    return on;
}

// raw register update over [p, p+n), n >= kFoldMin; leaves n % 256 bytes to crc32q
CC_FOLD_TARGET uint32_t fold_update(uint32_t reg, const unsigned char* p, size_t n) {
    if (n / kStep >= kSplitMinSteps && split_pays()) {
        // one split for the whole buffer: four long streams, which the hardware
        // prefetchers follow (48 KiB splits chained ran 73 vs 97 GiB/s at 4 MiB)
        const size_t M = n / kStep;
        reg = fold_split(reg, p, M);
        p += M * kStep;
        n -= M * kStep;
        if (n < kFoldMin) {
            uint64_t l = reg;
            while (n >= 8) {
                l = _mm_crc32_u64(l, load64(p));
                p += 8;
                n -= 8;
            }
            while (n--) l = _mm_crc32_u8(static_cast<uint32_t>(l), *p++);
            return static_cast<uint32_t>(l);
        }
    }
    const FoldKeys& fk = fold_keys();
    __m512i x0 = _mm512_loadu_si512(p), x1 = _mm512_loadu_si512(p + 64), x2 = _mm512_loadu_si512(p + 128),
            x3 = _mm512_loadu_si512(p + 192);
    x0 = _mm512_xor_si512(x0, _mm512_castsi128_si512(_mm_cvtsi32_si128((int)reg)));  // the register enters as the first 4 bytes
    p += 256;
    n -= 256;
    const __m512i k2048 = keys512(fk.k[1]);
    if (n >= 512) {
        const __m512i k4096 = keys512(fk.k[0]);
        __m512i y0 = _mm512_loadu_si512(p), y1 = _mm512_loadu_si512(p + 64), y2 = _mm512_loadu_si512(p + 128),
                y3 = _mm512_loadu_si512(p + 192);
        p += 256;
        n -= 256;
        while (n >= 512) {
            x0 = fold512(x0, k4096, _mm512_loadu_si512(p));
            x1 = fold512(x1, k4096, _mm512_loadu_si512(p + 64));
            x2 = fold512(x2, k4096, _mm512_loadu_si512(p + 128));
            x3 = fold512(x3, k4096, _mm512_loadu_si512(p + 192));
            y0 = fold512(y0, k4096, _mm512_loadu_si512(p + 256));
            y1 = fold512(y1, k4096, _mm512_loadu_si512(p + 320));
            y2 = fold512(y2, k4096, _mm512_loadu_si512(p + 384));
            y3 = fold512(y3, k4096, _mm512_loadu_si512(p + 448));
            p += 512;
            n -= 512;
        }
        x0 = fold512(x0, k2048, y0);
        x1 = fold512(x1, k2048, y1);
        x2 = fold512(x2, k2048, y2);
        x3 = fold512(x3, k2048, y3);
    }
    if (n >= 256) {
        x0 = fold512(x0, k2048, _mm512_loadu_si512(p));
        x1 = fold512(x1, k2048, _mm512_loadu_si512(p + 64));
        x2 = fold512(x2, k2048, _mm512_loadu_si512(p + 128));
        x3 = fold512(x3, k2048, _mm512_loadu_si512(p + 192));
        p += 256;
        n -= 256;
    }
    const __m512i k512 = keys512(fk.k[2]);
    x1 = fold512(x0, k512, x1);
    x2 = fold512(x1, k512, x2);
    x3 = fold512(x2, k512, x3);
    __m128i v = _mm512_extracti32x4_epi32(x3, 3);
    v = fold128(_mm512_extracti32x4_epi32(x3, 0), fk.k[3], v);
    v = fold128(_mm512_extracti32x4_epi32(x3, 1), fk.k[4], v);
    v = fold128(_mm512_extracti32x4_epi32(x3, 2), fk.k128, v);
    uint64_t l = _mm_crc32_u64(0, (uint64_t)_mm_cvtsi128_si64(v));
    l = _mm_crc32_u64(l, (uint64_t)_mm_extract_epi64(v, 1));
    while (n >= 8) {
        l = _mm_crc32_u64(l, load64(p));
        p += 8;
        n -= 8;
    }
    while (n--) l = _mm_crc32_u8(static_cast<uint32_t>(l), *p++);
    return static_cast<uint32_t>(l);
}

// CURVE_CRC_NO_FOLD=1 keeps the crc32q paths (tests compare the two)
bool have_fold() {
    static const bool ok = [] {
        const char* off = getenv("CURVE_CRC_NO_FOLD");
        if (off && off[0] && off[0] != '0') return false;
        __builtin_cpu_init();
        return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("vpclmulqdq") &&
               __builtin_cpu_supports("pclmul");
    }();
    return ok;
}

// raw register update over [p, p+n)
uint32_t raw_update(uint32_t reg, const unsigned char* p, size_t n) {
    if (n >= kFoldMin && have_fold()) return fold_update(reg, p, n);
    uint64_t l = reg;
    // no alignment prologue: unaligned 8-byte loads cost nothing extra here, and
    // the byte steps did (64 B: 21 -> 15 ns, 128 B: 28 -> 21 ns a call)
    if (n >= 3 * kBlocks[kNumBlocks - 1]) {
        const ShiftTables& st = shift_tables();
        int i = 0;
        while (n >= 3 * kBlocks[kNumBlocks - 1]) {
            while (3 * kBlocks[i] > n) i++;  // sizes only shrink as n does
            switch (i) {  // compile-time trip counts
                case 0: l = three_way<4096>(l, p, st, 0); break;
                case 1: l = three_way<2048>(l, p, st, 1); break;
                case 2: l = three_way<1360>(l, p, st, 2); break;
                case 3: l = three_way<1024>(l, p, st, 3); break;
                case 4: l = three_way<680>(l, p, st, 4); break;
                case 5: l = three_way<512>(l, p, st, 5); break;
                case 6: l = three_way<336>(l, p, st, 6); break;
                case 7: l = three_way<256>(l, p, st, 7); break;
                default: l = three_way<168>(l, p, st, 8); break;
            }
            p += 3 * kBlocks[i];
            n -= 3 * kBlocks[i];
        }
    }
    while (n >= 8) {
        l = _mm_crc32_u64(l, load64(p));
        p += 8;
        n -= 8;
    }
    while (n--) l = _mm_crc32_u8(static_cast<uint32_t>(l), *p++);
    return static_cast<uint32_t>(l);
}

}  // namespace

extern "C" {

uint32_t crc32c_extend(uint32_t crc, const void* p, size_t n) {
    return ~raw_update(~crc, static_cast<const unsigned char*>(p), n);
}

uint32_t crc32c_value(const void* p, size_t n) { return crc32c_extend(0, p, n); }

uint32_t crc32c_shift(uint32_t crc, uint64_t nbytes) { return shift_clmul(crc, nbytes); }

uint32_t crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) { return shift_clmul(crc_a, len_b) ^ crc_b; }

uint32_t crc32c_zeros(uint64_t nbytes) {
    // V(0^n) = ~shift(~0, n)
    return ~shift_clmul(0xFFFFFFFFu, nbytes);
}

uint32_t crc32c_extend_iov(uint32_t crc, const struct iovec* iov, size_t n) {
    // one raw register carried across the fragments: the same value as
    // extending fragment by fragment, without the per-fragment ~ in and out
    uint32_t reg = ~crc;
    for (size_t i = 0; i < n; i++)
        if (iov[i].iov_len) reg = raw_update(reg, static_cast<const unsigned char*>(iov[i].iov_base), iov[i].iov_len);
    return ~reg;
}

uint32_t cc_fold_host(const uint32_t* page_crcs, uint64_t n, uint64_t page_bytes) {
    if (n == 0) return 0;
    // Horner with the constant m = x^(8*page_bytes), four interleaved chains
    // (pages i = j mod 4 folded with m^4, then merged): the clmul latency is
    // paid once per four pages.  The 4 KiB-page fold of a 4 MiB scan slice
    // (1024 CRCs) was ~35 us with the bitwise multiply, now ~1 us.
    const uint32_t m = xpow_clmul(page_bytes << 3);
    if (n < 8) {
        uint32_t acc = page_crcs[0];
        for (uint64_t i = 1; i < n; i++) acc = mulmod_clmul(m, acc) ^ page_crcs[i];
        return acc;
    }
    const uint32_t m4 = mulmod_clmul(mulmod_clmul(m, m), mulmod_clmul(m, m));
    uint32_t a[4] = {page_crcs[0], page_crcs[1], page_crcs[2], page_crcs[3]};
    const uint64_t full = n / 4 * 4;
    for (uint64_t i = 4; i < full; i += 4)
        for (int j = 0; j < 4; j++) a[j] = mulmod_clmul(m4, a[j]) ^ page_crcs[i + j];
    // chain j holds sum_k c[4k+j] m^(4(K-1-k)); the whole = sum_j chain_j * m^(3-j)
    const uint32_t m2 = mulmod_clmul(m, m), m3 = mulmod_clmul(m2, m);
    uint32_t acc = mulmod_clmul(m3, a[0]) ^ mulmod_clmul(m2, a[1]) ^ mulmod_clmul(m, a[2]) ^ a[3];
    for (uint64_t i = full; i < n; i++) acc = mulmod_clmul(m, acc) ^ page_crcs[i];
    return acc;
}

int cc_slice_fold(const uint32_t* page_crcs, uint64_t n_pages, uint32_t pages_per_slice, uint32_t page_bytes,
                  uint32_t* out) {
    if (n_pages == 0) return CC_OK;
    if (!page_crcs || !out || pages_per_slice == 0 || page_bytes == 0 || n_pages % pages_per_slice) return CC_EINVAL;
    for (uint64_t s = 0; s < n_pages / pages_per_slice; s++)
        out[s] = cc_fold_host(page_crcs + s * pages_per_slice, pages_per_slice, page_bytes);
    return CC_OK;
}

}  // extern "C"

