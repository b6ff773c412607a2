/*
 * oracle/crc32c_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's CRC32C arithmetic, used exclusively as the
 * checker in tests/, in __graft_entry__.smoke() and as bench.py's cpu_baseline
 * leg.  The product (curve_amd/libcurvecrc.so) never links, loads or calls this.
 *
 * What it restates
 *   curve::common::CRC32(p, n)      -> butil::crc32c::Value   (src/common/crc32.h:40-42)
 *   curve::common::CRC32(c, p, n)   -> butil::crc32c::Extend  (src/common/crc32.h:53-55)
 * butil (brpc @ 1b9e00641cbec1c8803da6a1f7f555398c954cb0, WORKSPACE:138-153) is not
 * vendored in /root/reference, so the arithmetic is restated from its published
 * algorithm: CRC-32C (Castagnoli), reflected polynomial 0x82F63B78,
 * Extend(c, buf) = ~update(~c, buf), Value(buf) = Extend(0, buf).  The reference
 * builds butil with -msse4.2 -DHAVE_SSE42 (copts.bzl:35,38), i.e. a single-stream
 * hardware crc32 loop: that is what oc_crc32c_sse42() restates and what bench.py
 * times as the CPU baseline ("port").
 *
 * Parity is PINNED by the reference's own known answers (tests/test_oracle.py):
 *   test/common/crc32_test.cpp:49-84     RFC 3720 B.4 vectors
 *   test/common/crc32_test.cpp:90-93     Extend identity
 *   test/chunkserver/copyset_node_test.cpp:811-835   copyset hash 1355371765
 *   test/chunkserver/conf_epoch_file_test.cpp:103-106 chained CRC 599727352
 *
 * Three independent formulations are kept so they check each other:
 *   bitwise (one polynomial step per bit), Sarwate byte table, SSE4.2 crc32q.
 * The GF(2) shift/combine uses the 32x32 matrix-squaring formulation (the
 * classic zlib crc32_combine construction) -- deliberately a different method
 * from the product's polynomial exponentiation.
 */
#define _POSIX_C_SOURCE 200809L
#include <stdint.h>
#include <stddef.h>
#include <time.h>
#include <string.h>
#include <pthread.h>
#include <nmmintrin.h>

#define OC_POLY 0x82F63B78u

/* ---- bitwise ---------------------------------------------------------- */
uint32_t oc_crc32c_bitwise(uint32_t crc, const void *buf, size_t n) {
    const unsigned char *p = (const unsigned char *)buf;
    uint32_t l = crc ^ 0xFFFFFFFFu;
    for (size_t i = 0; i < n; i++) {
        l ^= p[i];
        for (int k = 0; k < 8; k++) l = (l >> 1) ^ (OC_POLY & (0u - (l & 1u)));
    }
    return l ^ 0xFFFFFFFFu;
}

/* ---- Sarwate byte table ---------------------------------------------- */
static uint32_t oc_table[256];
static pthread_once_t oc_table_once = PTHREAD_ONCE_INIT;
static void oc_table_init(void) {
    for (uint32_t b = 0; b < 256; b++) {
        uint32_t c = b;
        for (int k = 0; k < 8; k++) c = (c >> 1) ^ (OC_POLY & (0u - (c & 1u)));
        oc_table[b] = c;
    }
}

uint32_t oc_crc32c_table(uint32_t crc, const void *buf, size_t n) {
    pthread_once(&oc_table_once, oc_table_init);
    const unsigned char *p = (const unsigned char *)buf;
    uint32_t l = crc ^ 0xFFFFFFFFu;
    for (size_t i = 0; i < n; i++) l = oc_table[(l ^ p[i]) & 0xFFu] ^ (l >> 8);
    return l ^ 0xFFFFFFFFu;
}

/* ---- SSE4.2 single stream (butil Fast_CRC32 shape) -------------------- */
/* Byte steps up to 8-byte alignment, 8-byte crc32q steps, byte tail. */
uint32_t oc_crc32c_sse42(uint32_t crc, const void *buf, size_t n) {
    const unsigned char *p = (const unsigned char *)buf;
    const unsigned char *e = p + n;
    uint64_t l = (uint64_t)(crc ^ 0xFFFFFFFFu);
    while (p < e && ((uintptr_t)p & 7u)) l = _mm_crc32_u8((uint32_t)l, *p++);
    while (e - p >= 16) {
        uint64_t a, b;
        memcpy(&a, p, 8);
        memcpy(&b, p + 8, 8);
        l = _mm_crc32_u64(l, a);
        l = _mm_crc32_u64(l, b);
        p += 16;
    }
    while (e - p >= 8) {
        uint64_t a;
        memcpy(&a, p, 8);
        l = _mm_crc32_u64(l, a);
        p += 8;
    }
    while (p < e) l = _mm_crc32_u8((uint32_t)l, *p++);
    return ((uint32_t)l) ^ 0xFFFFFFFFu;
}

uint32_t oc_crc32c_value(const void *buf, size_t n) { return oc_crc32c_sse42(0, buf, n); }

/* ---- GF(2) matrix formulation of shift/combine ------------------------ */
static uint32_t gf2_times(const uint32_t *mat, uint32_t vec) {
    uint32_t sum = 0;
    while (vec) {
        if (vec & 1u) sum ^= *mat;
        vec >>= 1;
        mat++;
    }
    return sum;
}
static void gf2_square(uint32_t *sq, const uint32_t *mat) {
    for (int i = 0; i < 32; i++) sq[i] = gf2_times(mat, mat[i]);
}

/* Raw-register shift: the state after feeding nbytes zero bytes into a raw
 * (no pre/post inversion) CRC register holding `reg`. */
uint32_t oc_raw_shift(uint32_t reg, uint64_t nbytes) {
    uint32_t odd[32], even[32];
    if (nbytes == 0 || reg == 0) return reg;
    odd[0] = OC_POLY; /* operator for one zero bit */
    uint32_t row = 1;
    for (int i = 1; i < 32; i++) { odd[i] = row; row <<= 1; }
    gf2_square(even, odd); /* 2 bits */
    gf2_square(odd, even); /* 4 bits */
    /* apply len zero bytes (each step squares: 1 byte, 2 bytes, 4 bytes...) */
    do {
        gf2_square(even, odd);
        if (nbytes & 1u) reg = gf2_times(even, reg);
        nbytes >>= 1;
        if (nbytes == 0) break;
        gf2_square(odd, even);
        if (nbytes & 1u) reg = gf2_times(odd, reg);
        nbytes >>= 1;
    } while (nbytes != 0);
    return reg;
}

/* V(A||B) from V(A), V(B), |B|  (zlib crc32_combine identity). */
uint32_t oc_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
    return oc_raw_shift(crc_a, len_b) ^ crc_b;
}

/* ---- batched page CRCs (the CPU baseline of the hot path) -------------- */
/* Reference shape: one CRC32(page, page_bytes) call per page, as a caller of
 * src/common/crc32.h would issue them (op_request.cpp:794 for a scan slice). */
void oc_page_crcs(const void *pages, uint64_t n_pages, uint32_t page_bytes, uint32_t *out) {
    const unsigned char *p = (const unsigned char *)pages;
    for (uint64_t i = 0; i < n_pages; i++)
        out[i] = oc_crc32c_sse42(0, p + i * (uint64_t)page_bytes, page_bytes);
}

typedef struct {
    const unsigned char *p;
    uint64_t first, count;
    uint32_t page_bytes;
    uint32_t *out;
} oc_job;

static void *oc_worker(void *arg) {
    oc_job *j = (oc_job *)arg;
    oc_page_crcs(j->p + j->first * (uint64_t)j->page_bytes, j->count, j->page_bytes, j->out + j->first);
    return NULL;
}

/* Page-partitioned across `threads` POSIX threads. */
int oc_page_crcs_mt(const void *pages, uint64_t n_pages, uint32_t page_bytes, uint32_t *out, int threads) {
    if (threads <= 1) { oc_page_crcs(pages, n_pages, page_bytes, out); return 1; }
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    oc_job jobs[256];
    uint64_t per = (n_pages + (uint64_t)threads - 1) / (uint64_t)threads;
    int started = 0;
    for (int t = 0; t < threads; t++) {
        uint64_t first = per * (uint64_t)t;
        if (first >= n_pages) break;
        uint64_t cnt = n_pages - first < per ? n_pages - first : per;
        jobs[t].p = (const unsigned char *)pages;
        jobs[t].first = first;
        jobs[t].count = cnt;
        jobs[t].page_bytes = page_bytes;
        jobs[t].out = out;
        if (pthread_create(&tid[t], NULL, oc_worker, &jobs[t]) != 0) break;
        started++;
    }
    for (int t = 0; t < started; t++) pthread_join(tid[t], NULL);
    /* any range whose thread failed to start is done inline */
    for (int t = started; t < threads; t++) {
        uint64_t first = per * (uint64_t)t;
        if (first >= n_pages) break;
        uint64_t cnt = n_pages - first < per ? n_pages - first : per;
        oc_page_crcs((const unsigned char *)pages + first * (uint64_t)page_bytes, cnt, page_bytes, out + first);
    }
    return started;
}

/* ---- timing helper (bench.py cpu_baseline leg) -------------------------- */
/* Calls fn(crc, buf, n) `iters` times back to back, each call seeded with the
 * previous result (a dependency chain, so the calls cannot overlap), and
 * returns the elapsed seconds.  fn is any CRC with butil Extend's signature:
 * oc_crc32c_sse42 here, or libcurvecrc's crc32c_extend passed in by address --
 * a C loop, so a 4 KiB call is timed without any Python per-call overhead. */
typedef uint32_t (*oc_crc_fn)(uint32_t, const void *, size_t);
double oc_time_calls(oc_crc_fn fn, const void *buf, size_t n, uint64_t iters, uint32_t *sink) {
    struct timespec a, b;
    uint32_t c = 0;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (uint64_t i = 0; i < iters; i++) c = fn(c, buf, n);
    clock_gettime(CLOCK_MONOTONIC, &b);
    if (sink) *sink = c;
    return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}
