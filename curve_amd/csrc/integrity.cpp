// curve_amd/csrc/integrity.cpp -- per-page CRC persistence:
// the sidecar table codec, its atomic store, and the check of a batch of chunk
// files against their tables (the body of an IntegrityService job,
// proto/integrity.proto:55-61 -- declared in the reference, never implemented).
//
// The reference keeps no per-page data CRC anywhere: the chunk metapage holds
// version / sn / correctedSn / location / bitmap and a CRC of that header only
// (src/chunkserver/datastore/chunkserver_chunkfile.cpp:64-130).  So the table is
// a NEW artefact, kept outside the copyset data directory (CopysetNode::GetHash
// chains every file listed there, copyset_node.cpp:931-970, and a sidecar in it
// would change the copyset hash).
//
// Sidecar layout (little-endian, 64-byte header):
//    0  magic "CVPCRC02"
//    8  version u32 (= 2) | page_bytes u32 | n_pages u32 | reserved u32
//   24  chunk_sn u64          metapage sn of the chunk when the table was written
//   32  data_mtime_ns i64     the chunk FILE's st_mtim then
//   40  data_size u64         the chunk file's size then
//   48  stamp_ns i64          CLOCK_REALTIME when the CRCs' bytes were known current
//                             (racy-table rule, include/curve_crc.h cc_pcrc_is_racy)
//   56  header_crc u32        CRC32C of bytes [0, 56)
//   60  table_crc u32         CRC32C of the page-CRC array
//   64  page CRCs, n_pages x u32 (CRC32 of each data page, the file's bytes
//       [meta_bytes + i * page_bytes, +page_bytes))
// A table is only ever used to condemn data when it provably describes the
// chunk's current bytes: both CRCs check, the geometry matches, the chunk's
// sn, mtime and size are the ones recorded, and the table is not racy (its
// stamp is at least one coarse-clock tick after the recorded mtime, so no
// write can have kept that mtime after the CRCs were taken).  Otherwise it is
// reported (corrupt / stale) and, by policy, rebuilt -- never turned into bad
// pages.
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <string>
#include <thread>
#include <vector>

#include "../../include/curve_crc.h"

namespace {

constexpr char kMagic[8] = {'C', 'V', 'P', 'C', 'R', 'C', '0', '2'};
constexpr uint32_t kVersion = 2;

inline void put32(unsigned char* p, uint32_t v) { memcpy(p, &v, 4); }
inline void put64(unsigned char* p, uint64_t v) { memcpy(p, &v, 8); }
inline uint32_t get32(const unsigned char* p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
inline uint64_t get64(const unsigned char* p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}

int read_full(int fd, void* dst, size_t n, off_t off) {
    char* p = static_cast<char*>(dst);
    size_t got = 0;
    while (got < n) {
        const ssize_t r = pread(fd, p + got, n - got, off + (off_t)got);
        if (r < 0) {
            if (errno == EINTR) continue;
            return -errno;
        }
        if (r == 0) return CC_EIO;  // short file
        got += (size_t)r;
    }
    return 0;
}

int write_full(int fd, const void* src, size_t n) {
    const char* p = static_cast<const char*>(src);
    size_t put = 0;
    while (put < n) {
        const ssize_t r = write(fd, p + put, n - put);
        if (r < 0) {
            if (errno == EINTR) continue;
            return -errno;
        }
        put += (size_t)r;
    }
    return 0;
}

int64_t mtime_ns(const struct stat& sb) { return (int64_t)sb.st_mtim.tv_sec * 1000000000ll + sb.st_mtim.tv_nsec; }

int64_t now_ns() {
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    return (int64_t)ts.tv_sec * 1000000000ll + ts.tv_nsec;
}

// One tick of the clock file timestamps come from (the kernel's coarse
// realtime clock: a jiffy, 1-10 ms); at least 1 ms, at most 1 s.
int64_t coarse_tick_ns() {
    static const int64_t tick = [] {
        struct timespec r;
        int64_t t = 0;
        if (clock_getres(CLOCK_REALTIME_COARSE, &r) == 0) t = (int64_t)r.tv_sec * 1000000000ll + r.tv_nsec;
        return t < 1000000 ? 1000000 : (t > 1000000000 ? 1000000000 : t);
    }();
    return tick;
}

// The granularity a recorded mtime may have been truncated to.  A filesystem
// that keeps whole seconds (ext4 with 128-byte inodes, many NFS / FUSE mounts)
// or FAT's 2 s records an mtime with no sub-second part: a same-size rewrite
// within that second keeps it, so such a table stays racy for 1 s (2 s when the
// second is even) after its mtime, not for one coarse-clock tick.
int64_t mtime_granule_ns(int64_t mtime) {
    const int64_t tick = coarse_tick_ns();
    if (mtime % 1000000000ll != 0) return tick;
    const int64_t g = mtime % 2000000000ll == 0 ? 2000000000ll : 1000000000ll;
    return g > tick ? g : tick;
}

// Chunk file identity for staleness: sn from the metapage, mtime + size from stat.
struct ChunkId {
    uint64_t sn = 0;
    int64_t mtime = 0;
    uint64_t size = 0;
};

// file_bytes != 0: the chunk geometry's file size; any other size is
// CC_EFORMAT before the metapage is read, as CSChunkFile::Open checks the size
// first (chunkserver_chunkfile.cpp:233-238, FileFormatError)
int chunk_identity(const char* path, uint32_t meta_bytes, ChunkId* id, uint64_t file_bytes = 0) {
    const int fd = open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return -errno;
    struct stat sb;
    int rc = fstat(fd, &sb) == 0 ? 0 : -errno;
    if (!rc && file_bytes && (uint64_t)sb.st_size != file_bytes) rc = CC_EFORMAT;
    std::vector<unsigned char> mp(meta_bytes);
    if (!rc) rc = read_full(fd, mp.data(), meta_bytes, 0);
    close(fd);
    if (rc) return rc;
    if ((rc = cc_chunk_meta_sn(mp.data(), meta_bytes, &id->sn))) return rc;
    id->mtime = mtime_ns(sb);
    id->size = (uint64_t)sb.st_size;
    return 0;
}

int stat_identity(const char* path, ChunkId* id) {
    struct stat sb;
    if (stat(path, &sb) != 0) return -errno;
    id->mtime = mtime_ns(sb);
    id->size = (uint64_t)sb.st_size;
    return 0;
}

}  // namespace

extern "C" {

uint64_t cc_pcrc_encoded_bytes(uint32_t n_pages) { return CC_PCRC_HEADER_BYTES + 4ull * n_pages; }

int cc_pcrc_encode(const cc_pcrc_header* h, const uint32_t* page_crcs, void* out, uint64_t out_bytes) {
    if (!h || !out || (h->n_pages && !page_crcs) || h->page_bytes == 0) return CC_EINVAL;
    if (out_bytes < cc_pcrc_encoded_bytes(h->n_pages)) return CC_EINVAL;
    unsigned char* p = static_cast<unsigned char*>(out);
    memset(p, 0, CC_PCRC_HEADER_BYTES);
    memcpy(p, kMagic, 8);
    put32(p + 8, kVersion);
    put32(p + 12, h->page_bytes);
    put32(p + 16, h->n_pages);
    put64(p + 24, h->chunk_sn);
    put64(p + 32, (uint64_t)h->data_mtime_ns);
    put64(p + 40, h->data_size);
    put64(p + 48, (uint64_t)h->stamp_ns);
    if (h->n_pages) memcpy(p + CC_PCRC_HEADER_BYTES, page_crcs, 4ull * h->n_pages);  // page_crcs may be null at 0
    put32(p + 56, crc32c_value(p, 56));
    put32(p + 60, crc32c_value(p + CC_PCRC_HEADER_BYTES, 4ull * h->n_pages));
    return CC_OK;
}

int cc_pcrc_decode(const void* buf, uint64_t bytes, cc_pcrc_header* h, uint32_t* page_crcs, uint32_t max_pages) {
    if (!buf || !h) return CC_EINVAL;
    const unsigned char* p = static_cast<const unsigned char*>(buf);
    if (bytes < CC_PCRC_HEADER_BYTES || memcmp(p, kMagic, 8) != 0) return CC_ECORRUPT;
    if (crc32c_value(p, 56) != get32(p + 56) || get32(p + 8) != kVersion) return CC_ECORRUPT;
    const uint32_t n = get32(p + 16);
    if (bytes != cc_pcrc_encoded_bytes(n)) return CC_ECORRUPT;
    if (crc32c_value(p + CC_PCRC_HEADER_BYTES, 4ull * n) != get32(p + 60)) return CC_ECORRUPT;
    h->page_bytes = get32(p + 12);
    h->n_pages = n;
    h->chunk_sn = get64(p + 24);
    h->data_mtime_ns = (int64_t)get64(p + 32);
    h->data_size = get64(p + 40);
    h->stamp_ns = (int64_t)get64(p + 48);
    if (page_crcs) {
        if (n > max_pages) return CC_EINVAL;
        memcpy(page_crcs, p + CC_PCRC_HEADER_BYTES, 4ull * n);
    }
    return CC_OK;
}

int cc_chunk_meta_sn(const void* metapage, uint32_t bytes, uint64_t* sn) {
    // ChunkFileMetaPage::decode (chunkserver_chunkfile.cpp:90-130): version u8 |
    // sn u64 | correctedSn u64 | loc_size u64 [| location | bits u32 | bitmap]
    // | CRC32 of the above; bounds-checked (a header that cannot fit is corrupt)
    if (!metapage || !sn) return CC_EINVAL;
    const unsigned char* p = static_cast<const unsigned char*>(metapage);
    if (bytes < 29) return CC_ECORRUPT;
    uint64_t len = 25;
    const uint64_t loc = get64(p + 17);
    if (loc) {
        if (loc > bytes || len + loc + 4 + 4 > bytes) return CC_ECORRUPT;
        len += loc;
        const uint64_t bits = get32(p + len);
        len += 4;
        const uint64_t nb = (bits + 7) >> 3;
        if (nb > bytes - len - 4) return CC_ECORRUPT;
        len += nb;
    }
    if (crc32c_value(p, len) != get32(p + len)) return CC_ECORRUPT;
    if (p[0] != 1 && p[0] != 2) return CC_ECORRUPT;  // FORMAT_VERSION / _V2 (datastore/define.h:39-40)
    *sn = get64(p + 1);
    return CC_OK;
}

int cc_pcrc_is_racy(const cc_pcrc_header* h) {
    if (!h) return CC_EINVAL;
    // closed boundary (git's >=): the coarse clock may lag a write by a full tick
    return h->data_mtime_ns + mtime_granule_ns(h->data_mtime_ns) >= h->stamp_ns ? 1 : 0;
}

int cc_pcrc_load(const char* table_path, cc_pcrc_header* h, uint32_t* page_crcs, uint32_t max_pages) {
    if (!table_path || !h) return CC_EINVAL;
    const int fd = open(table_path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return -errno;
    struct stat sb;
    if (fstat(fd, &sb) != 0) {
        const int e = -errno;
        close(fd);
        return e;
    }
    // never allocate what a valid table for this caller cannot need: a corrupt
    // or hostile sidecar must not make a job step read gigabytes
    const uint64_t cap = page_crcs ? cc_pcrc_encoded_bytes(max_pages) : CC_PCRC_HEADER_BYTES;
    if (page_crcs && (uint64_t)sb.st_size > cap) {
        close(fd);
        return CC_ECORRUPT;
    }
    if ((uint64_t)sb.st_size < CC_PCRC_HEADER_BYTES || sb.st_size > (off_t)cc_pcrc_encoded_bytes(0xFFFFFFFFu)) {
        close(fd);
        return CC_ECORRUPT;
    }
    std::vector<unsigned char> buf(page_crcs ? (size_t)sb.st_size : (size_t)CC_PCRC_HEADER_BYTES);
    const int rc = read_full(fd, buf.data(), buf.size(), 0);
    close(fd);
    if (rc) return rc;
    if (page_crcs) return cc_pcrc_decode(buf.data(), buf.size(), h, page_crcs, max_pages);
    // header only: its own CRC, and a length that matches the file
    unsigned char* p = buf.data();
    if (memcmp(p, kMagic, 8) != 0 || crc32c_value(p, 56) != get32(p + 56) || get32(p + 8) != kVersion ||
        (uint64_t)sb.st_size != cc_pcrc_encoded_bytes(get32(p + 16)))
        return CC_ECORRUPT;
    h->page_bytes = get32(p + 12);
    h->n_pages = get32(p + 16);
    h->chunk_sn = get64(p + 24);
    h->data_mtime_ns = (int64_t)get64(p + 32);
    h->data_size = get64(p + 40);
    h->stamp_ns = (int64_t)get64(p + 48);
    return CC_OK;
}

}  // extern "C"

namespace {
// The store behind cc_pcrc_store.  With `expect`, the chunk's identity read here
// must still be the one the CRCs were computed under (else CC_ESTALE, nothing
// written): a write landing between a job's read and its table refresh must not
// get a table of the bytes before it.  `stamp` is when those bytes were known
// current (0 = now: only for a caller holding the chunk's write lock, so no
// write can land between the bytes it describes and this call).
int store_table(const char* chunk_path, uint32_t meta_bytes, const char* table_path, const uint32_t* page_crcs,
                uint32_t n_pages, uint32_t page_bytes, const ChunkId* expect, int64_t stamp = 0) {
    if (!chunk_path || !table_path || (n_pages && !page_crcs) || page_bytes == 0 || meta_bytes == 0)
        return CC_EINVAL;
    ChunkId id;
    int rc = chunk_identity(chunk_path, meta_bytes, &id);
    if (rc) return rc;
    if (id.size != (uint64_t)meta_bytes + (uint64_t)n_pages * page_bytes) return CC_EFORMAT;  // FileFormatError
    if (expect && (id.sn != expect->sn || id.mtime != expect->mtime || id.size != expect->size)) return CC_ESTALE;
    cc_pcrc_header h = {page_bytes, n_pages, id.sn, id.mtime, id.size, stamp ? stamp : now_ns()};
    std::vector<unsigned char> buf(cc_pcrc_encoded_bytes(n_pages));
    if ((rc = cc_pcrc_encode(&h, page_crcs, buf.data(), buf.size()))) return rc;
    // atomic replace: a reader sees the old table or the new one, never a torn one
    std::string tmp = std::string(table_path) + ".tmp." + std::to_string(getpid()) + "." +
                      std::to_string(std::hash<std::thread::id>()(std::this_thread::get_id()));
    const int fd = open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0) return -errno;
    rc = write_full(fd, buf.data(), buf.size());
    if (!rc && fsync(fd) != 0) rc = -errno;
    if (close(fd) != 0 && !rc) rc = -errno;
    if (!rc && rename(tmp.c_str(), table_path) != 0) rc = -errno;
    if (rc) unlink(tmp.c_str());
    return rc;
}
}  // namespace

extern "C" {

int cc_pcrc_store(const char* chunk_path, uint32_t meta_bytes, const char* table_path, const uint32_t* page_crcs,
                  uint32_t n_pages, uint32_t page_bytes) {
    return store_table(chunk_path, meta_bytes, table_path, page_crcs, n_pages, page_bytes, nullptr);
}

int cc_pcrc_store_expect(const char* chunk_path, uint32_t meta_bytes, const char* table_path,
                         const uint32_t* page_crcs, uint32_t n_pages, uint32_t page_bytes,
                         const cc_pcrc_header* expect) {
    if (!expect) return CC_EINVAL;
    ChunkId e;
    e.sn = expect->chunk_sn;
    e.mtime = expect->data_mtime_ns;
    e.size = expect->data_size;
    // never the store's own clock: a second same-size write in the mtime's tick
    // keeps the identity, and a table stamped later than that would not be racy
    // and would condemn the newer bytes.  The caller's stamp (taken before its
    // pwrite), else the mtime itself -- racy until a check re-stamps the table.
    const int64_t stamp = expect->stamp_ns ? expect->stamp_ns : expect->data_mtime_ns;
    return store_table(chunk_path, meta_bytes, table_path, page_crcs, n_pages, page_bytes, &e, stamp);
}

int cc_integrity_check(const char* const* chunk_paths, const char* const* table_paths, uint64_t n,
                       const cc_integrity_opts* o, cc_integrity_result* res, uint64_t* bad_list, uint64_t bad_cap,
                       uint64_t* n_bad) {
    if (n_bad) *n_bad = 0;
    if (n == 0) return CC_OK;
    if (!chunk_paths || !table_paths || !o || !res || (bad_cap && !bad_list)) return CC_EINVAL;
    if (o->page_bytes == 0 || o->chunk_bytes == 0 || o->meta_bytes == 0 || o->chunk_bytes % o->page_bytes)
        return CC_EINVAL;
    const uint32_t n_pages = o->chunk_bytes / o->page_bytes;
    // 1. identity BEFORE the read: sn from the metapage, mtime + size; and the
    //    stamp a table rewritten from this read will carry (taken first: every
    //    byte read below is at least this current)
    const int64_t stamp = now_ns();
    std::vector<ChunkId> before(n);
    for (uint64_t i = 0; i < n; i++) {
        res[i] = cc_integrity_result{0, CC_TABLE_OK, n_pages, 0, -1};
        if (!chunk_paths[i] || !table_paths[i]) {
            res[i].status = CC_EINVAL;
            continue;
        }
        res[i].status = chunk_identity(chunk_paths[i], o->meta_bytes, &before[i],
                                       (uint64_t)o->meta_bytes + o->chunk_bytes);
    }
    // 2. page CRCs of every chunk's data on the device (slice = page: the
    //    per-slice CRCs of cc_scan_files ARE the page CRCs)
    std::vector<uint32_t> pcs((size_t)n * n_pages);
    std::vector<cc_file_result> fr(n);
    int rc = cc_scan_files(chunk_paths, n, o->chunk_bytes, o->meta_bytes, o->page_bytes, o->page_bytes,
                           o->io_threads, pcs.data(), fr.data());
    if (rc) return rc;
    std::vector<uint32_t> want(n_pages);
    uint64_t nb = 0;
    for (uint64_t i = 0; i < n; i++) {
        cc_integrity_result& r = res[i];
        if (r.status) continue;
        if (fr[i].status) {
            r.status = fr[i].status;
            continue;
        }
        const uint32_t* got = pcs.data() + i * n_pages;
        // 3. the file must not have changed while it was read
        ChunkId after;
        if ((r.status = stat_identity(chunk_paths[i], &after))) continue;
        const bool moved = after.mtime != before[i].mtime || after.size != before[i].size;
        cc_pcrc_header h;
        const int lr = cc_pcrc_load(table_paths[i], &h, want.data(), n_pages);
        auto rebuild = [&](uint32_t state_ok) {
            if (moved) {  // bytes of a moving target: nothing to record
                r.table_state = CC_TABLE_STALE;
                return;
            }
            // the chunk must still be the one read in step 2 (identity before)
            const int s = store_table(chunk_paths[i], o->meta_bytes, table_paths[i], got, n_pages, o->page_bytes,
                                      &before[i], stamp);
            if (s == CC_ESTALE) {
                r.table_state = CC_TABLE_STALE;
                return;
            }
            if (s) r.status = s;
            r.table_state = state_ok;
        };
        if (lr == -ENOENT) {
            r.table_state = CC_TABLE_MISSING;
            if (o->create_missing) rebuild(CC_TABLE_CREATED);
            continue;
        }
        if (lr == CC_ECORRUPT || (lr == CC_OK && (h.page_bytes != o->page_bytes || h.n_pages != n_pages)) ||
            lr == CC_EINVAL) {
            r.table_state = CC_TABLE_CORRUPT;
            if (o->refresh_stale) rebuild(CC_TABLE_REBUILT);
            continue;
        }
        if (lr) {
            r.status = lr;
            continue;
        }
        if (moved || h.chunk_sn != before[i].sn || h.data_mtime_ns != before[i].mtime ||
            h.data_size != before[i].size) {
            // the chunk changed after its table was written (a write that did
            // not persist its CRCs, or a snapshot): stale, never bad pages
            r.table_state = CC_TABLE_STALE;
            if (o->refresh_stale) rebuild(CC_TABLE_REFRESHED);
            continue;
        }
        if (cc_pcrc_is_racy(&h)) {
            // the table was written within a clock tick of the chunk's last
            // write: a later write may have kept the mtime, so a mismatch
            // proves nothing -- stale; a match re-stamps the table (rewritten
            // with this check's stamp, one tick or more after the mtime)
            const bool same = memcmp(got, want.data(), 4ull * n_pages) == 0;
            if (!same) {
                r.table_state = CC_TABLE_STALE;
                if (o->refresh_stale) rebuild(CC_TABLE_REFRESHED);
            } else {
                rebuild(CC_TABLE_OK);
            }
            continue;
        }
        for (uint32_t p = 0; p < n_pages; p++) {
            if (got[p] == want[p]) continue;
            if (r.first_bad < 0) r.first_bad = p;
            r.bad_pages++;
            if (nb < bad_cap) bad_list[nb] = (i << 32) | p;
            nb++;
        }
    }
    if (n_bad) *n_bad = nb;
    return CC_OK;
}

}  // extern "C"
