// crc32c_cpu.cpp's loops (3-way crc32q, the VPCLMULQDQ fold, the fold + crc32q
// split) on buffers allocated to their exact size, built with ASan/UBSan by
// tests/test_sanitize.py: any load past a buffer's end is reported.  The mode
// comes from the environment (CURVE_CRC_NO_FOLD / CURVE_CRC_FOLD_SPLIT), read
// once by the library.  Values checked against a bitwise CRC32C.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <initializer_list>

extern "C" uint32_t crc32c_value(const void* p, size_t n);

static uint32_t bitwise(const unsigned char* p, size_t n) {
    uint32_t c = ~0u;
    for (size_t i = 0; i < n; i++) {
        c ^= p[i];
        for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    }
    return ~c;
}

int main() {
    int bad = 0;
    for (size_t n : {0ul, 1ul, 7ul, 63ul, 255ul, 256ul, 300ul, 511ul, 512ul, 767ul, 4096ul, 6015ul, 6016ul, 6017ul,
                     9999ul, 48129ul, 100000ul, 1048577ul}) {
        for (size_t off = 0; off < 3; off++) {
            unsigned char* b = static_cast<unsigned char*>(malloc(n + off));
            for (size_t i = 0; i < n + off; i++) b[i] = static_cast<unsigned char>(i * 131u + off);
            if (crc32c_value(b + off, n) != bitwise(b + off, n)) {
                printf("mismatch n=%zu off=%zu\n", n, off);
                bad++;
            }
            free(b);
        }
    }
    if (!bad) printf("crc_cpu_bounds: ok\n");
    return bad ? 1 : 0;
}
