// tests/native/parser_fuzz.cpp -- hostile inputs for the CPU parsers that read
// untrusted bytes (test infrastructure):
//   * the per-page CRC sidecar: cc_pcrc_decode, cc_pcrc_load (include/curve_crc.h);
//   * the chunk metapage: cc_chunk_meta_sn and cchost::ChunkFileMetaPage::decode
//     (the reference's ChunkFileMetaPage::decode, chunkserver_chunkfile.cpp:90-130,
//     trusts loc_size and the bitmap bit count; these must not).
// Deterministic mutations: every truncation, extensions, every header bit
// flipped, forged headers whose own CRC checks, random byte storms.  Every
// input lives in a heap buffer of exactly its length, so an over-read is an
// AddressSanitizer report in the sanitized build (scripts/sanitize.sh) and at
// worst a wrong verdict in the plain one (tests/test_sanitize.py runs both).
// Exit status 0 = every verdict was the expected one.
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "../../curve_amd/host/chunkserver_host.h"
#include "../../include/curve_crc.h"

namespace {

int g_fail = 0;
#define EXPECT(c)                                                             \
    do {                                                                      \
        if (!(c)) {                                                           \
            fprintf(stderr, "%s:%d: EXPECT(%s) failed\n", __FILE__, __LINE__, #c); \
            g_fail++;                                                         \
        }                                                                     \
    } while (0)

uint64_t g_rng = 0x9E3779B97F4A7C15ull;
uint64_t rnd() {  // xorshift64*
    g_rng ^= g_rng >> 12;
    g_rng ^= g_rng << 25;
    g_rng ^= g_rng >> 27;
    return g_rng * 0x2545F4914F6CDD1Dull;
}

// a heap copy of exactly n bytes (ASan sees any read past it)
struct Exact {
    unsigned char* p;
    size_t n;
    Exact(const void* src, size_t len) : p(static_cast<unsigned char*>(malloc(len ? len : 1))), n(len) {
        if (len) memcpy(p, src, len);
    }
    ~Exact() { free(p); }
};

std::vector<unsigned char> table(uint32_t n_pages) {
    std::vector<uint32_t> pcs(n_pages);
    for (auto& x : pcs) x = (uint32_t)rnd();
    cc_pcrc_header h = {4096, n_pages, 7, 1234567890123ll, 4096ull + 4096ull * n_pages, 1234567999999ll};
    std::vector<unsigned char> buf(cc_pcrc_encoded_bytes(n_pages));
    EXPECT(cc_pcrc_encode(&h, pcs.data(), buf.data(), buf.size()) == CC_OK);
    return buf;
}

int decode(const std::vector<unsigned char>& b, size_t len, uint32_t max_pages) {
    Exact e(b.data(), len);
    cc_pcrc_header h;
    std::vector<uint32_t> out(max_pages + 1);
    const uint32_t canary = 0xC0DEC0DE;
    out[max_pages] = canary;
    const int rc = cc_pcrc_decode(e.p, e.n, &h, max_pages ? out.data() : nullptr, max_pages);
    EXPECT(out[max_pages] == canary);  // never writes past max_pages
    return rc;
}

// the header's own CRC recomputed after a forgery, so decode gets past it
void reseal(std::vector<unsigned char>& b) {
    const uint32_t c = crc32c_value(b.data(), 56);
    memcpy(b.data() + 56, &c, 4);
}

void fuzz_sidecar() {
    for (uint32_t n : {0u, 1u, 7u, 300u, 4096u}) {
        auto b = table(n);
        EXPECT(decode(b, b.size(), n) == CC_OK);
        EXPECT(decode(b, b.size(), 0) == CC_OK);  // header only
        if (n > 1) EXPECT(decode(b, b.size(), n - 1) == CC_EINVAL);  // caller's buffer too small
        // every truncation (sampled for the big table), and extensions
        const size_t step = b.size() > 2048 ? 97 : 1;
        for (size_t L = 0; L < b.size(); L += step) EXPECT(decode(b, L, n) == CC_ECORRUPT);
        for (size_t x = 1; x <= 64; x += 7) {
            auto c = b;
            c.resize(b.size() + x, 0xAB);
            EXPECT(decode(c, c.size(), n + 32) == CC_ECORRUPT);
        }
        // every bit of the header, 256 random bits of the table
        for (size_t bit = 0; bit < 64 * 8; bit++) {
            auto c = b;
            c[bit / 8] ^= (unsigned char)(1u << (bit % 8));
            EXPECT(decode(c, c.size(), n) == CC_ECORRUPT);
        }
        for (int k = 0; n && k < 256; k++) {
            auto c = b;
            const size_t at = 64 + rnd() % (4ull * n);
            c[at] ^= (unsigned char)(1u << (rnd() % 8));
            EXPECT(decode(c, c.size(), n) == CC_ECORRUPT);
        }
        // forged page counts whose header CRC checks: the length no longer matches
        for (uint32_t f : {n + 1, n ? n - 1 : 5u, 0x3FFFFFFFu, 0x40000000u, 0xFFFFFFFFu}) {
            auto c = b;
            memcpy(c.data() + 16, &f, 4);
            reseal(c);
            EXPECT(decode(c, c.size(), n) == CC_ECORRUPT);
            EXPECT(decode(c, c.size(), 0) == CC_ECORRUPT);
        }
    }
    // byte storms: a valid magic + version half the time, a resealed header half of those
    for (int k = 0; k < 20000; k++) {
        std::vector<unsigned char> c(rnd() % 400);
        for (auto& x : c) x = (unsigned char)rnd();
        if (c.size() >= 64 && (k & 1)) {
            memcpy(c.data(), "CVPCRC02", 8);
            const uint32_t v = 2;
            memcpy(c.data() + 8, &v, 4);
            if (k & 2) {
                const uint32_t np = (uint32_t)(rnd() % 96);
                memcpy(c.data() + 16, &np, 4);
                reseal(c);
            }
        }
        const int rc = decode(c, c.size(), 96);
        EXPECT(rc == CC_OK || rc == CC_ECORRUPT || rc == CC_EINVAL);
        if (rc == CC_OK) EXPECT(c.size() >= 64 && (c.size() - 64) % 4 == 0);
    }
}

void fuzz_sidecar_files(const std::string& dir) {
    auto b = table(64);
    const std::string p = dir + "/t.pcrc";
    auto put = [&](const std::vector<unsigned char>& c, off_t truncate_to) {
        const int fd = open(p.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
        EXPECT(fd >= 0 && write(fd, c.data(), c.size()) == (ssize_t)c.size());
        if (truncate_to >= 0) EXPECT(ftruncate(fd, truncate_to) == 0);
        close(fd);
    };
    cc_pcrc_header h;
    std::vector<uint32_t> out(64);
    put(b, -1);
    EXPECT(cc_pcrc_load(p.c_str(), &h, out.data(), 64) == CC_OK && h.n_pages == 64);
    EXPECT(cc_pcrc_load(p.c_str(), &h, nullptr, 0) == CC_OK);
    EXPECT(cc_pcrc_load(p.c_str(), &h, out.data(), 63) == CC_ECORRUPT);  // larger than the caller's table
    for (off_t L : {(off_t)0, (off_t)10, (off_t)63, (off_t)64, (off_t)65, (off_t)(b.size() - 1)}) {
        put(b, L);
        EXPECT(cc_pcrc_load(p.c_str(), &h, out.data(), 64) != CC_OK);
        EXPECT(cc_pcrc_load(p.c_str(), &h, nullptr, 0) != CC_OK);
    }
    put(b, (off_t)8 << 30);  // 8 GiB sparse: refused before any allocation
    EXPECT(cc_pcrc_load(p.c_str(), &h, out.data(), 64) == CC_ECORRUPT);
    EXPECT(cc_pcrc_load(p.c_str(), &h, nullptr, 0) == CC_ECORRUPT);
    unlink(p.c_str());
    EXPECT(cc_pcrc_load(p.c_str(), &h, out.data(), 64) == -2);  // -ENOENT
}

std::vector<unsigned char> metapage(size_t size, bool clone, uint32_t bits) {
    std::vector<unsigned char> m(size, 0);
    cchost::ChunkFileMetaPage mp;
    mp.sn = 99;
    mp.correctedSn = 3;
    if (clone) {
        mp.location = "s3://bucket/object@7";
        mp.bitmapBits = bits;
        mp.bitmap.assign((bits + 7) / 8, 0x5A);
    }
    mp.encode(reinterpret_cast<char*>(m.data()));
    return m;
}

void check_meta(const std::vector<unsigned char>& m, size_t size, bool want_ok) {
    Exact e(m.data(), size);
    uint64_t sn = 0;
    const int rc = cc_chunk_meta_sn(e.p, (uint32_t)e.n, &sn);
    cchost::ChunkFileMetaPage mp;
    const cchost::CSErrorCode dc = mp.decode(reinterpret_cast<const char*>(e.p), e.n);
    if (want_ok) {
        EXPECT(rc == CC_OK && sn == 99);
        EXPECT(dc == cchost::Success && mp.sn == 99);
    } else {
        EXPECT(rc == CC_ECORRUPT);
        EXPECT(dc == cchost::CrcCheckError || dc == cchost::IncompatibleError);
    }
}

void fuzz_metapage() {
    for (size_t size : {(size_t)4096, (size_t)8192, (size_t)512}) {
        for (int clone = 0; clone < 2; clone++) {
            const uint32_t bits = clone ? (uint32_t)(size * 8 - 512) : 0;  // the bitmap nearly fills the page
            auto m = metapage(size, clone, bits);
            check_meta(m, size, true);
            const size_t hdr = clone ? 25 + 20 + 4 + (bits + 7) / 8 + 4 : 29;
            for (size_t L = 0; L < hdr; L++) check_meta(m, L, false);  // every truncation into the header
            for (size_t bit = 0; bit < hdr * 8; bit += clone ? 13 : 1) {
                auto c = m;
                c[bit / 8] ^= (unsigned char)(1u << (bit % 8));
                check_meta(c, size, false);
            }
        }
        // forged location sizes / bitmap bit counts, whether or not the CRC would check
        const uint64_t locs[] = {1, 8, size - 33, size - 29, size - 25, size, size + 1, 1ull << 32,
                                 (1ull << 63), ~0ull, ~0ull - 24};
        for (uint64_t loc : locs) {
            for (uint32_t bits : {0u, 1u, 0x7FFFFFFFu, 0xFFFFFFFFu, (uint32_t)(size * 8)}) {
                std::vector<unsigned char> c(size, 0);
                c[0] = 2;
                memcpy(c.data() + 17, &loc, 8);
                if (loc < size - 29) memcpy(c.data() + 25 + loc, &bits, 4);
                Exact e(c.data(), size);
                uint64_t sn;
                EXPECT(cc_chunk_meta_sn(e.p, (uint32_t)size, &sn) == CC_ECORRUPT);
                cchost::ChunkFileMetaPage mp;
                EXPECT(mp.decode(reinterpret_cast<const char*>(e.p), size) != cchost::Success);
            }
        }
    }
    for (int k = 0; k < 20000; k++) {  // storms
        const size_t size = 29 + rnd() % 200;
        std::vector<unsigned char> c(size);
        for (auto& x : c) x = (unsigned char)rnd();
        if (k & 1) {  // a small plausible loc_size
            const uint64_t loc = rnd() % 64;
            memcpy(c.data() + 17, &loc, 8);
        }
        Exact e(c.data(), size);
        uint64_t sn;
        const int rc = cc_chunk_meta_sn(e.p, (uint32_t)size, &sn);
        EXPECT(rc == CC_OK || rc == CC_ECORRUPT);
        cchost::ChunkFileMetaPage mp;
        (void)mp.decode(reinterpret_cast<const char*>(e.p), size);
    }
}

}  // namespace

int main(int argc, char** argv) {
    char tmpl[] = "/tmp/ccfuzz_XXXXXX";
    const char* dir = argc > 1 ? argv[1] : mkdtemp(tmpl);
    if (!dir) return 2;
    fuzz_sidecar();
    fuzz_sidecar_files(dir);
    fuzz_metapage();
    if (argc <= 1) rmdir(dir);
    printf("parser_fuzz: %s (%d failed expectations)\n", g_fail ? "FAIL" : "ok", g_fail);
    return g_fail ? 1 : 0;
}
