/* examples/abi_demo.c -- a plain-C consumer of libcurvecrc's ABI (no Python,
 * no torch): the shape a chunkserver call site takes.
 *
 *   build: gcc -O2 -std=c11 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude examples/abi_demo.c \
 *          -Lcurve_amd -lcurvecrc -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$ORIGIN/../curve_amd' -o build/abi_demo
 *   run:   build/abi_demo            (exit 0 = every check passed)
 *
 * Checks, per reference surface:
 *   1. CRC32(p, n) / CRC32(crc, p, n) known answers (test/common/crc32_test.cpp:49-93)
 *   2. device page CRCs of a 16 MiB chunk == CRC32(page, 4096) per page (CPU primitive)
 *   3. the 4 x 4 MiB ScanMap slice CRCs from cc_fold_dev == CRC32(slice)
 *   4. host path cc_page_crc_host and streaming cc_scan_host agree
 *   5. verify flags a corrupted page exactly
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "curve_crc.h"

#define CHECK(c, msg)                                  \
    do {                                               \
        if (!(c)) {                                    \
            fprintf(stderr, "FAIL: %s (line %d)\n", msg, __LINE__); \
            return 1;                                  \
        }                                              \
    } while (0)

int main(void) {
    /* 1. primitive */
    unsigned char z[32] = {0}, inc[32];
    for (int i = 0; i < 32; i++) inc[i] = (unsigned char)i;
    CHECK(crc32c_value(z, 32) == 0x8a9136aau, "RFC 3720 zeros");
    CHECK(crc32c_value(inc, 32) == 0x46dd794eu, "RFC 3720 incrementing");
    CHECK(crc32c_value("hello world", 11) == crc32c_extend(crc32c_value("hello ", 6), "world", 5), "Extend");
    CHECK(crc32c_zeros(4096) == 0x98F94189u, "zero page");
    if (cc_device_count() <= 0) {
        printf("no GPU: CPU checks passed, device checks skipped\n");
        return 0;
    }
    CHECK(cc_engine_init(NULL) == CC_OK, "engine init");

    const size_t chunk = 16u << 20, page = 4096, n_pages = chunk / page;
    unsigned char* h = (unsigned char*)malloc(chunk);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (size_t i = 0; i < chunk; i++) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = (unsigned char)x; }

    void* d = NULL;
    uint32_t *dcrc = NULL, *dslice = NULL;
    uint64_t* dcnt = NULL;
    CHECK(hipMalloc(&d, chunk) == hipSuccess && hipMalloc((void**)&dcrc, n_pages * 4) == hipSuccess &&
              hipMalloc((void**)&dslice, 16) == hipSuccess && hipMalloc((void**)&dcnt, 16) == hipSuccess,
          "hipMalloc");
    CHECK(hipMemcpy(d, h, chunk, hipMemcpyHostToDevice) == hipSuccess, "H2D");

    /* 2. page CRCs */
    CHECK(cc_page_crc_dev(d, n_pages, page, dcrc, NULL) == CC_OK, "cc_page_crc_dev");
    uint32_t* crcs = (uint32_t*)malloc(n_pages * 4);
    CHECK(hipMemcpy(crcs, dcrc, n_pages * 4, hipMemcpyDeviceToHost) == hipSuccess, "D2H");
    for (size_t i = 0; i < n_pages; i++) CHECK(crcs[i] == crc32c_value(h + i * page, page), "page CRC");

    /* 3. ScanMap slices: 1024 pages -> one 4 MiB slice CRC */
    uint32_t slices[4];
    CHECK(cc_fold_dev(dcrc, 4, 1024, page, dslice, NULL) == CC_OK, "cc_fold_dev");
    CHECK(hipMemcpy(slices, dslice, 16, hipMemcpyDeviceToHost) == hipSuccess, "D2H slices");
    for (int k = 0; k < 4; k++) CHECK(slices[k] == crc32c_value(h + (size_t)k * (4u << 20), 4u << 20), "slice CRC");

    /* 4. host paths */
    uint32_t* hc = (uint32_t*)malloc(n_pages * 4);
    CHECK(cc_page_crc_host(h, n_pages, page, hc) == CC_OK, "cc_page_crc_host");
    CHECK(memcmp(hc, crcs, n_pages * 4) == 0, "host == device");
    unsigned char meta[4096] = {2};
    cc_chunk_src src = {meta, h};
    uint32_t mc, sc[4], fc;
    CHECK(cc_scan_host(&src, 1, chunk, 4096, page, 4u << 20, &mc, sc, &fc) == CC_OK, "cc_scan_host");
    CHECK(memcmp(sc, slices, 16) == 0 && mc == crc32c_value(meta, 4096), "scan slices / metapage");
    CHECK(fc == crc32c_extend(crc32c_value(meta, 4096), h, chunk), "file CRC == CRC32 chain over metapage||data");

    /* 5. verify */
    uint64_t init[2] = {0, ~0ull}, got[2];
    unsigned char one = h[123 * page + 9] ^ 0x80;
    CHECK(hipMemcpy((unsigned char*)d + 123 * page + 9, &one, 1, hipMemcpyHostToDevice) == hipSuccess, "poke");
    CHECK(hipMemcpy(dcnt, init, 16, hipMemcpyHostToDevice) == hipSuccess, "init counters");
    CHECK(cc_page_verify_dev(d, n_pages, page, dcrc, dcnt, dcnt + 1, NULL) == CC_OK, "verify");
    CHECK(hipMemcpy(got, dcnt, 16, hipMemcpyDeviceToHost) == hipSuccess, "D2H counters");
    CHECK(got[0] == 1 && got[1] == 123, "verify finds page 123 only");

    hipFree(d); hipFree(dcrc); hipFree(dslice); hipFree(dcnt);
    free(h); free(crcs); free(hc);
    cc_engine_fini();
    printf("abi_demo: all checks passed (%s)\n", cc_version());
    return 0;
}
