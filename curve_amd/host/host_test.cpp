// curve_amd/host/host_test.cpp -- parity tests of the C++ host layer
// (chunkserver_host.h) in the shape of the reference's own gtest cases, run
// as one binary (no gtest in this image).  TEST ONLY: links the CPU oracle
// (oracle/crc32c_oracle.c) as the checker.
//
//   host_test            run every case; GPU cases are SKIPPED when no device
//   host_test --gpu      fail if no device (GPU box)
// Exit status 0 iff every case that ran passed.  Prints one line per case.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <functional>
#include <random>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "../../include/curve_crc.h"
#include "../../include/curve_crc32_compat.h"
#include "chunkserver_host.h"
#include "integrity_service.h"

extern "C" uint32_t oc_crc32c_sse42(uint32_t crc, const void* buf, size_t n);  // oracle (test only)

using namespace cchost;

namespace {

int g_fail = 0;
#define EXPECT(c)                                                             \
    do {                                                                      \
        if (!(c)) {                                                           \
            fprintf(stderr, "  %s:%d: EXPECT(%s) failed\n", __FILE__, __LINE__, #c); \
            g_fail++;                                                         \
        }                                                                     \
    } while (0)

std::string g_tmp;

std::string MakeDir(const std::string& name) {
    std::string d = g_tmp + "/" + name;
    mkdir(d.c_str(), 0755);
    return d;
}

void WriteFile(const std::string& path, const std::string& bytes) {
    FILE* f = fopen(path.c_str(), "wb");
    if (!f) {
        perror(path.c_str());
        abort();
    }
    fwrite(bytes.data(), 1, bytes.size(), f);
    fclose(f);
}

std::string MetaPage(uint64_t sn, uint8_t version = FORMAT_VERSION_V2, uint32_t page = 4096) {
    std::string buf(page, '\0');
    ChunkFileMetaPage m;
    m.version = version;
    m.sn = sn;
    m.encode(&buf[0]);
    return buf;
}

uint32_t Oracle(const std::string& s, uint32_t crc = 0) { return oc_crc32c_sse42(crc, s.data(), s.size()); }

// ---- test/common/crc32_test.cpp --------------------------------------------
void Crc32Vectors() {
    std::string z(32, '\0'), ff(32, '\xff'), inc(32, 0), dec(32, 0);
    for (int i = 0; i < 32; i++) {
        inc[i] = (char)i;
        dec[i] = (char)(31 - i);
    }
    EXPECT(crc32c_value(z.data(), 32) == 0x8a9136aaU);
    EXPECT(crc32c_value(ff.data(), 32) == 0x62a8ab43U);
    EXPECT(crc32c_value(inc.data(), 32) == 0x46dd794eU);
    EXPECT(crc32c_value(dec.data(), 32) == 0x113fdb5cU);
    EXPECT(crc32c_value("hello world", 11) == crc32c_extend(crc32c_value("hello ", 6), "world", 5));
    EXPECT(crc32c_value("a", 1) != crc32c_value("foo", 3));
    // the drop-in wrapper headers (src/common/crc32.h:40-55, nebd/src/common/crc32.h:31-38)
    EXPECT(curve::common::CRC32("hello world", 11) == 3381945770u);
    EXPECT(curve::common::CRC32(curve::common::CRC32("hello ", 6), "world", 5) == 3381945770u);
    EXPECT(nebd::common::CRC32(z.data(), 32) == 0x8a9136aaU);
    EXPECT(nebd::common::CRC32(nebd::common::CRC32("hello ", 6), "world", 5) == 3381945770u);
}

// ---- ChunkFileMetaPage (chunkserver_chunkfile.cpp:64-130) -------------------
void MetaPageEncodeDecode() {
    std::string page = MetaPage(7);
    ChunkFileMetaPage d;
    EXPECT(d.decode(page.data()) == Success && d.sn == 7 && d.version == FORMAT_VERSION_V2);
    EXPECT(Oracle(page) == 317729701u);  // residue constant of every non-clone 4 KiB metapage
    page[3] ^= 1;
    EXPECT(d.decode(page.data()) == CrcCheckError);
    EXPECT(d.decode(MetaPage(1, 3).data()) == IncompatibleError);
    ChunkFileMetaPage clone;
    clone.sn = 2;
    clone.location = "curvefs:/f@1";
    clone.bitmapBits = 20;
    clone.bitmap = {0xA5, 0x0F, 0x03};
    std::string cp(4096, '\0');
    clone.encode(&cp[0]);
    ChunkFileMetaPage back;
    EXPECT(back.decode(cp.data()) == Success && back.location == clone.location && back.bitmapBits == 20 &&
           back.bitmap == clone.bitmap);
    // corrupt lengths: a loc_size or bitmap that overruns the page is a CRC
    // error, never a read past the buffer
    std::string huge = cp;
    const uint64_t big = 1ull << 40;
    memcpy(&huge[17], &big, 8);
    EXPECT(back.decode(huge.data(), huge.size()) == CrcCheckError);
    std::string bits = cp;
    const uint32_t many = 0xFFFFFFFFu;
    memcpy(&bits[25 + clone.location.size()], &many, 4);
    EXPECT(back.decode(bits.data(), bits.size()) == CrcCheckError);
    EXPECT(back.decode(cp.data(), 20) == CrcCheckError);  // shorter than a header
}

// ---- ScanManager::CompareMap (scan_manager_test.cpp shapes) -----------------
void CompareMapCases() {
    ScanMap a{1, 2, 3, 10, 100, 0, 4096};
    std::vector<ScanMap> failed;
    EXPECT(CompareMap(a, {a, a}, &failed) && failed.empty());
    ScanMap b = a;
    b.crc = 200;  // mismatched crc
    EXPECT(!CompareMap(a, {a, b}, &failed) && failed.size() == 1 && failed[0] == a);
    ScanMap c = a;
    c.index = 11;  // index is compared too (MessageDifferencer::Equals)
    EXPECT(!CompareMap(a, {c, a}, &failed) && failed.size() == 2);
    EXPECT(!CompareMap(a, {a}, &failed) && failed.size() == 2);  // not three maps: not failed
}

// ---- CopysetNode::GetHash (copyset_node_test.cpp:811-997) -------------------
void CopysetHashSmallFiles() {
    std::string d = MakeDir("cs_small");
    std::string h;
    EXPECT(GetCopysetHash(d, 16u << 20, 4096, &h) == 0 && h == "0");  // empty dir
    WriteFile(d + "/test-1.txt", "wwwww\n");
    WriteFile(d + "/test-4.txt", "mmmmmmmm\n");
    WriteFile(d + "/test-5.txt", "eeeeeeeeeee\n");
    WriteFile(d + "/test-3.txt", std::string(7680, '\0'));
    WriteFile(d + "/test-2.txt", "abcddddddddd333\n");
    EXPECT(GetCopysetHash(d, 16u << 20, 4096, &h) == 0 && h == "1355371765");
    EXPECT(symlink((d + "/gone").c_str(), (d + "/test-6.txt").c_str()) == 0);  // listed, cannot be opened
    EXPECT(GetCopysetHash(d, 16u << 20, 4096, &h) == -1);
    EXPECT(GetCopysetHash(d + "/no-such-dir", 16u << 20, 4096, &h) == -1);
}

// ---- ChunkServiceImpl::GetChunkHash request checks (chunk_service_test.cpp:463-502)
void ChunkServiceHashRequests() {
    DataStoreOptions o;
    o.baseDir = MakeDir("svc");
    std::string h = "x";
    EXPECT(ChunkServiceGetChunkHash(o, 100, 0, 4096, &h) == CHUNK_OP_STATUS_SUCCESS && h == "0");  // no chunk
    EXPECT(ChunkServiceGetChunkHash(o, 100, 3, 4096, &h) == CHUNK_OP_STATUS_INVALID_REQUEST);
    EXPECT(ChunkServiceGetChunkHash(o, 100, 0, 4097, &h) == CHUNK_OP_STATUS_INVALID_REQUEST);
    EXPECT(ChunkServiceGetChunkHash(o, 100, (16u << 20) - 4096, 8192, &h) == CHUNK_OP_STATUS_INVALID_REQUEST);
    // a written chunk, small ranges (CPU primitive): chunk_service_test.cpp:563-578
    std::string raw = MetaPage(1) + std::string(4096, 'a') + std::string((16u << 20) - 4096, '\0');
    WriteFile(o.baseDir + "/chunk_1", raw);
    EXPECT(ChunkServiceGetChunkHash(o, 1, 4096, 4096, &h) == CHUNK_OP_STATUS_SUCCESS && h == "650595490");
    EXPECT(ChunkServiceGetChunkHash(o, 1, 0, 4096, &h) == CHUNK_OP_STATUS_SUCCESS && h == "317729701");
}

// ---- GPU cases ----------------------------------------------------------------
void ChunkHashLongRanges() {  // CSChunkFile::GetHash over long raw ranges (engine path)
    DataStoreOptions o;
    o.baseDir = MakeDir("hash_long");
    std::mt19937_64 rng(11);
    std::string raw(4096 + (16u << 20), '\0');
    for (auto& c : raw) c = (char)(rng() & 0xFF);
    std::string meta = MetaPage(3);
    raw.replace(0, 4096, meta);
    WriteFile(o.baseDir + "/chunk_9", raw);
    std::string h;
    struct R {
        off_t off;
        size_t len;
    } rs[] = {{0, 16u << 20}, {4096, 16u << 20}, {0, (16u << 20) + 4096}, {12288, 1u << 20}, {5, 200001}};
    for (const auto& r : rs) {
        EXPECT(GetChunkHash(o, 9, r.off, r.len, &h) == Success);
        EXPECT(h == std::to_string(Oracle(raw.substr(r.off, r.len))));
    }
    EXPECT(GetChunkHash(o, 9, 4096, (16u << 20) + 1, &h) == InternalError);  // past the end of the file
    EXPECT(ChunkServiceGetChunkHash(o, 9, 0, 16u << 20, &h) == CHUNK_OP_STATUS_SUCCESS &&
           h == std::to_string(Oracle(raw.substr(0, 16u << 20))));
}

void CopysetHashOneChunk() {  // chunkserver_snapshot_test.cpp:339-388
    std::string d = MakeDir("cs_one");
    std::string data(16u << 20, '\0');
    memset(&data[0], 'b', 25 * 4096);
    WriteFile(d + "/chunk_1", MetaPage(1) + data);
    std::string h;
    EXPECT(GetCopysetHash(d, 16u << 20, 4096, &h) == 0 && h == "3049021227");
}

void CopysetHashMixed() {  // chunk files + a snapshot of other geometry + small files, sorted chain
    std::string d = MakeDir("cs_mixed");
    std::mt19937_64 rng(5);
    std::vector<std::pair<std::string, std::string>> files;
    for (uint64_t id : {1, 2, 10, 11, 100}) {
        std::string data(1u << 20, '\0');
        for (auto& c : data) c = (char)(rng() & 0xFF);
        files.emplace_back(ChunkFileName(id), MetaPage(id) + data);
    }
    files.emplace_back("chunk_2_snap_1", std::string(300000, 's'));
    files.emplace_back("zz", "tail");
    for (auto& f : files) WriteFile(d + "/" + f.first, f.second);
    std::sort(files.begin(), files.end());
    uint32_t want = 0;
    for (auto& f : files) want = Oracle(f.second, want);
    std::string h;
    EXPECT(GetCopysetHash(d, 1u << 20, 4096, &h) == 0 && h == std::to_string(want));
}

void ScanCopysetMaps() {  // ScanJobProcess + OnApply over chunk files
    DataStoreOptions o;
    o.baseDir = MakeDir("scan");
    o.chunkSize = 1u << 20;
    const uint32_t scan = 256u << 10;
    std::mt19937_64 rng(7);
    std::vector<std::pair<uint64_t, std::string>> chunks;
    for (auto idv : std::vector<std::pair<uint64_t, uint8_t>>{{12, 2}, {3, 2}, {7, 1}, {40, 2}}) {
        std::string data(o.chunkSize, '\0');
        for (auto& c : data) c = (char)(rng() & 0xFF);
        std::string raw = MetaPage(idv.first, idv.second) + data;
        WriteFile(o.baseDir + "/" + ChunkFileName(idv.first), raw);
        if (idv.second == FORMAT_VERSION_V2) chunks.emplace_back(idv.first, raw);
    }
    WriteFile(o.baseDir + "/chunk_3_snap_2", "snapshot");
    std::sort(chunks.begin(), chunks.end());
    std::vector<ScanMap> maps;
    EXPECT(ScanCopyset(o, 1, 9, scan, 100, &maps) == 0);
    EXPECT(maps.size() == chunks.size() * 5);
    size_t k = 0;
    for (auto& c : chunks) {
        for (int op = 0; op < 5 && k < maps.size(); op++, k++) {
            const ScanMap& m = maps[k];
            const uint64_t off = op == 0 ? 0 : (uint64_t)(op - 1) * scan;
            const uint64_t len = op == 0 ? 4096 : scan;
            const std::string bytes = op == 0 ? c.second.substr(0, 4096) : c.second.substr(4096 + off, len);
            EXPECT(m.chunkId == c.first && m.offset == off && m.len == len && m.index == 100 + k &&
                   m.logicalPoolId == 1 && m.copysetId == 9);
            EXPECT(m.crc == Oracle(bytes));
        }
    }
    EXPECT(ScanCopyset(o, 1, 9, 3u << 18, 0, &maps) == -1);  // scanSize must divide chunkSize
}

void PoolScanShardRccl() {  // one rank's shard, native RCCL comm (world 1)
    const uint64_t n = 6;
    const uint32_t chunk = 1u << 20, meta = 4096, scan = 256u << 10;
    const uint64_t ids[n] = {3, 1, 12, 7, 40, 2};
    const uint32_t group[n] = {0, 1, 0, 1, 0, 1};
    std::mt19937_64 rng(21);
    std::string data(n * chunk, '\0'), metas(n * meta, '\0');
    for (auto& c : data) c = (char)(rng() & 0xFF);
    for (uint64_t i = 0; i < n; i++) metas.replace(i * meta, meta, MetaPage(ids[i]));
    // copyset chain geometry: files in std::sort name order, bytes after each file
    std::vector<uint64_t> after(n, 0);
    for (uint64_t i = 0; i < n; i++)
        for (uint64_t k = 0; k < n; k++)
            if (group[k] == group[i] && ChunkFileName(ids[k]) > ChunkFileName(ids[i])) after[i] += chunk + meta;
    void *d_data = nullptr, *d_meta = nullptr, *d_after = nullptr, *d_mult = nullptr, *d_group = nullptr;
    void *d_pc = nullptr, *d_mc = nullptr, *d_sc = nullptr, *d_fc = nullptr, *d_dig = nullptr;
    EXPECT(hipMalloc(&d_data, data.size()) == hipSuccess && hipMalloc(&d_meta, metas.size()) == hipSuccess);
    EXPECT(hipMalloc(&d_after, n * 8) == hipSuccess && hipMalloc(&d_mult, n * 4) == hipSuccess &&
           hipMalloc(&d_group, n * 4) == hipSuccess);
    EXPECT(hipMalloc(&d_pc, n * chunk / 1024) == hipSuccess && hipMalloc(&d_mc, n * 4) == hipSuccess &&
           hipMalloc(&d_sc, n * 16) == hipSuccess && hipMalloc(&d_fc, n * 4) == hipSuccess &&
           hipMalloc(&d_dig, 8) == hipSuccess);
    EXPECT(hipMemcpy(d_data, data.data(), data.size(), hipMemcpyHostToDevice) == hipSuccess);
    EXPECT(hipMemcpy(d_meta, metas.data(), metas.size(), hipMemcpyHostToDevice) == hipSuccess);
    EXPECT(hipMemcpy(d_after, after.data(), n * 8, hipMemcpyHostToDevice) == hipSuccess);
    EXPECT(hipMemcpy(d_group, group, n * 4, hipMemcpyHostToDevice) == hipSuccess);
    EXPECT(cc_xpow8_dev((const uint64_t*)d_after, n, (uint32_t*)d_mult, nullptr) == CC_OK);
    char id[CC_COMM_ID_BYTES];
    cc_comm* comm = nullptr;
    EXPECT(cc_comm_unique_id(id, sizeof id) == CC_OK);
    EXPECT(cc_comm_init(&comm, 1, 0, id, sizeof id) == CC_OK && cc_comm_size(comm) == 1);
    cc_pool_shard s = {};
    s.d_data = d_data;
    s.d_meta = d_meta;
    s.n_chunks = n;
    s.chunk_bytes = chunk;
    s.meta_bytes = meta;
    s.page_bytes = 4096;
    s.slice_bytes = scan;
    s.d_after_mult = (const uint32_t*)d_mult;
    s.d_group = (const uint32_t*)d_group;
    s.n_groups = 2;
    s.d_page_crcs = (uint32_t*)d_pc;
    s.d_meta_crcs = (uint32_t*)d_mc;
    s.d_slice_crcs = (uint32_t*)d_sc;
    s.d_file_crcs = (uint32_t*)d_fc;
    s.d_digest = (uint32_t*)d_dig;
    EXPECT(cc_pool_scan_dev(&s, comm, nullptr) == CC_OK);
    EXPECT(hipDeviceSynchronize() == hipSuccess);
    uint32_t dig[2], sl[n * 4];
    EXPECT(hipMemcpy(dig, d_dig, 8, hipMemcpyDeviceToHost) == hipSuccess);
    EXPECT(hipMemcpy(sl, d_sc, sizeof sl, hipMemcpyDeviceToHost) == hipSuccess);
    for (uint32_t g = 0; g < 2; g++) {  // CopysetNode::GetHash: sorted names, chained CRC from 0
        std::vector<std::pair<std::string, uint64_t>> files;
        for (uint64_t i = 0; i < n; i++)
            if (group[i] == g) files.emplace_back(ChunkFileName(ids[i]), i);
        std::sort(files.begin(), files.end());
        uint32_t want = 0;
        for (auto& f : files)
            want = Oracle(metas.substr(f.second * meta, meta) + data.substr(f.second * chunk, chunk), want);
        EXPECT(dig[g] == want);
    }
    for (uint64_t i = 0; i < n; i++)
        for (uint32_t k = 0; k < 4; k++) EXPECT(sl[i * 4 + k] == Oracle(data.substr(i * chunk + k * scan, scan)));
    EXPECT(cc_comm_destroy(comm) == CC_OK);
    for (void* p : {d_data, d_meta, d_after, d_mult, d_group, d_pc, d_mc, d_sc, d_fc, d_dig}) EXPECT(hipFree(p) == hipSuccess);
}

void WriteLogBothModes() {  // an ordered write log from plain C++, both CRC modes
    const uint32_t pb = 4096, max_len = 5000;
    const uint64_t pool_bytes = 1 << 20, src_bytes = 1 << 16, n = 600;
    std::mt19937_64 rng(33);
    std::string pool(pool_bytes, '\0'), src(src_bytes, '\0');
    for (auto& c : pool) c = (char)(rng() & 0xFF);
    for (auto& c : src) c = (char)(rng() & 0xFF);
    std::vector<cc_update> log(n);
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t len = 1 + (uint32_t)(rng() % max_len);
        const uint64_t dst = i < 200 ? 5 * pb + rng() % (3 * pb) : rng() % (pool_bytes - len);  // overlaps first
        log[i] = {dst < pool_bytes - len ? dst : pool_bytes - len, rng() % (src_bytes - len), len, 0};
    }
    std::string want = pool;  // in-order application: later writes win
    for (const cc_update& u : log) want.replace(u.dst, u.len, src.substr(u.src, u.len));
    void *d_src = nullptr, *d_log = nullptr, *d_work = nullptr;
    EXPECT(hipMalloc(&d_src, src_bytes) == hipSuccess && hipMalloc(&d_log, n * sizeof(cc_update)) == hipSuccess);
    EXPECT(hipMemcpy(d_src, src.data(), src_bytes, hipMemcpyHostToDevice) == hipSuccess);
    EXPECT(hipMemcpy(d_log, log.data(), n * sizeof(cc_update), hipMemcpyHostToDevice) == hipSuccess);
    const uint64_t work = cc_apply_log_work_bytes(n, max_len, pb);
    EXPECT(work > 0 && hipMalloc(&d_work, work) == hipSuccess);
    for (int delta = 0; delta < 2; delta++) {
        void *d_pool = nullptr, *d_pc = nullptr;
        EXPECT(hipMalloc(&d_pool, pool_bytes) == hipSuccess && hipMalloc(&d_pc, pool_bytes / pb * 4) == hipSuccess);
        EXPECT(hipMemcpy(d_pool, pool.data(), pool_bytes, hipMemcpyHostToDevice) == hipSuccess);
        EXPECT(cc_page_crc_dev(d_pool, pool_bytes / pb, pb, (uint32_t*)d_pc, nullptr) == CC_OK);
        auto apply = delta ? cc_apply_log_delta_dev : cc_apply_log_dev;
        EXPECT(apply(d_pool, pool_bytes, pb, d_src, (const cc_update*)d_log, n, max_len, (uint32_t*)d_pc, d_work, work,
                     nullptr) == CC_OK);
        EXPECT(hipDeviceSynchronize() == hipSuccess);
        std::string got(pool_bytes, '\0');
        std::vector<uint32_t> pc(pool_bytes / pb);
        EXPECT(hipMemcpy(&got[0], d_pool, pool_bytes, hipMemcpyDeviceToHost) == hipSuccess);
        EXPECT(hipMemcpy(pc.data(), d_pc, pc.size() * 4, hipMemcpyDeviceToHost) == hipSuccess);
        EXPECT(got == want);
        for (uint64_t p = 0; p < pc.size(); p++) EXPECT(pc[p] == Oracle(want.substr(p * pb, pb)));
        for (void* q : {d_pool, d_pc}) EXPECT(hipFree(q) == hipSuccess);
    }
    for (void* q : {d_src, d_log, d_work}) EXPECT(hipFree(q) == hipSuccess);
}

// INTEGRATION.md 6b/6c per request: one client write, then reads verified one at
// a time, as WriteChunk / ReadChunk would call them (the one-launch paths)
void PerRequestWriteAndRead() {
    const uint32_t pb = 4096;
    const uint64_t pool_bytes = 1 << 20;
    std::mt19937_64 rng(77);
    std::string pool(pool_bytes, '\0'), src(8192, '\0');
    for (auto& c : pool) c = (char)(rng() & 0xFF);
    for (auto& c : src) c = (char)(rng() & 0xFF);
    void *d_pool = nullptr, *d_pc = nullptr, *d_src = nullptr, *d_log = nullptr, *d_work = nullptr;
    void *d_reads = nullptr, *d_bad = nullptr, *d_total = nullptr;
    EXPECT(hipMalloc(&d_pool, pool_bytes) == hipSuccess && hipMalloc(&d_pc, pool_bytes / pb * 4) == hipSuccess);
    EXPECT(hipMalloc(&d_src, src.size()) == hipSuccess && hipMalloc(&d_log, sizeof(cc_update)) == hipSuccess);
    EXPECT(hipMemcpy(d_pool, pool.data(), pool_bytes, hipMemcpyHostToDevice) == hipSuccess);
    EXPECT(hipMemcpy(d_src, src.data(), src.size(), hipMemcpyHostToDevice) == hipSuccess);
    EXPECT(cc_page_crc_dev(d_pool, pool_bytes / pb, pb, (uint32_t*)d_pc, nullptr) == CC_OK);
    // one write straddling pages 10 and 11
    const cc_update w = {10 * pb + 3000, 100, 2500, 0};
    EXPECT(hipMemcpy(d_log, &w, sizeof w, hipMemcpyHostToDevice) == hipSuccess);
    const uint64_t work = cc_apply_log_work_bytes(1, pb, pb);
    EXPECT(work > 0 && hipMalloc(&d_work, work) == hipSuccess);
    EXPECT(cc_apply_log_delta_dev(d_pool, pool_bytes, pb, d_src, (const cc_update*)d_log, 1, pb, (uint32_t*)d_pc,
                                  d_work, work, nullptr) == CC_OK);
    pool.replace(w.dst, w.len, src.substr(w.src, w.len));
    // then bit rot in page 40 (after its CRC was stored)
    pool[40 * pb + 9] ^= 0x20;
    EXPECT(hipMemcpy((char*)d_pool + 40 * pb + 9, &pool[40 * pb + 9], 1, hipMemcpyHostToDevice) == hipSuccess);
    const cc_range reads[3] = {{10 * pb, 2 * pb}, {36 * pb, 8 * pb}, {100 * pb + 512, 4096}};
    const uint32_t want[3] = {0, 1, 0};
    const uint64_t rwork = cc_verify_reads_work_bytes(1);
    EXPECT(rwork > 0 && hipMalloc(&d_reads, sizeof(cc_range)) == hipSuccess && hipMalloc(&d_bad, 4) == hipSuccess &&
           hipMalloc(&d_total, 8) == hipSuccess);
    void *d_rwork = nullptr;
    EXPECT(hipMalloc(&d_rwork, rwork) == hipSuccess);
    for (int i = 0; i < 3; i++) {  // ReadChunk: one read per call
        uint32_t bad = 7;
        uint64_t total = 7;
        EXPECT(hipMemset(d_bad, 0, 4) == hipSuccess && hipMemset(d_total, 0, 8) == hipSuccess);
        EXPECT(hipMemcpy(d_reads, &reads[i], sizeof(cc_range), hipMemcpyHostToDevice) == hipSuccess);
        EXPECT(cc_verify_reads_dev(d_pool, pool_bytes, pb, (const cc_range*)d_reads, 1, (const uint32_t*)d_pc,
                                   (uint32_t*)d_bad, (uint64_t*)d_total, d_rwork, rwork, nullptr) == CC_OK);
        EXPECT(hipMemcpy(&bad, d_bad, 4, hipMemcpyDeviceToHost) == hipSuccess);
        EXPECT(hipMemcpy(&total, d_total, 8, hipMemcpyDeviceToHost) == hipSuccess);
        EXPECT(bad == want[i] && total == want[i]);
    }
    std::vector<uint32_t> pc(pool_bytes / pb);
    EXPECT(hipMemcpy(pc.data(), d_pc, pc.size() * 4, hipMemcpyDeviceToHost) == hipSuccess);
    EXPECT(pc[10] == Oracle(pool.substr(10 * pb, pb)) && pc[11] == Oracle(pool.substr(11 * pb, pb)));
    for (void* q : {d_pool, d_pc, d_src, d_log, d_work, d_reads, d_bad, d_total, d_rwork}) EXPECT(hipFree(q) == hipSuccess);
}

// ---- per-page CRC persistence ------------------------------
void IntegrityTableAndService() {  // CPU: codec, metapage sn, atomic store / load, service state machine
    std::vector<uint32_t> pc(256);
    std::mt19937_64 rng(5);
    for (auto& c : pc) c = (uint32_t)rng();
    cc_pcrc_header h = {4096, 256, 9, 123456789, 4096 + (1u << 20), 0};
    std::vector<unsigned char> buf(cc_pcrc_encoded_bytes(256));
    EXPECT(cc_pcrc_encode(&h, pc.data(), buf.data(), buf.size()) == CC_OK);
    cc_pcrc_header g;
    std::vector<uint32_t> got(256);
    EXPECT(cc_pcrc_decode(buf.data(), buf.size(), &g, got.data(), 256) == CC_OK);
    EXPECT(g.chunk_sn == 9 && g.data_mtime_ns == 123456789 && g.n_pages == 256 && got == pc);
    for (size_t pos : {0ul, 12ul, 30ul, 58ul, 64ul + 5, buf.size() - 1}) {
        buf[pos] ^= 1;
        EXPECT(cc_pcrc_decode(buf.data(), buf.size(), &g, nullptr, 0) == CC_ECORRUPT);
        buf[pos] ^= 1;
    }
    uint64_t sn = 0;
    const std::string mp = MetaPage(42);
    EXPECT(cc_chunk_meta_sn(mp.data(), 4096, &sn) == CC_OK && sn == 42);
    std::string bad = mp;
    bad[2] ^= 1;
    EXPECT(cc_chunk_meta_sn(bad.data(), 4096, &sn) == CC_ECORRUPT);
    const std::string data = MakeDir("integ_cpu"), dd = data + "/data";
    mkdir(dd.c_str(), 0755);
    WriteFile(dd + "/chunk_1", mp + std::string(1 << 20, 'z'));
    const std::string tdir = TableDirFor(dd);
    EXPECT(tdir == data + "/pcrc");
    mkdir(tdir.c_str(), 0755);
    EXPECT(cc_pcrc_store((dd + "/chunk_1").c_str(), 4096, TablePath(tdir, "chunk_1").c_str(), pc.data(), 256, 4096) ==
           CC_OK);
    EXPECT(cc_pcrc_load(TablePath(tdir, "chunk_1").c_str(), &g, got.data(), 256) == CC_OK && got == pc && g.chunk_sn == 42);
    EXPECT(cc_pcrc_store((dd + "/chunk_1").c_str(), 4096, TablePath(tdir, "x").c_str(), pc.data(), 255, 4096) ==
           CC_EFORMAT);  // the file is not metapage + 255 pages (FileFormatError)
    EXPECT(cc_pcrc_load(TablePath(tdir, "none").c_str(), &g, nullptr, 0) == -ENOENT);
    // the service state machine (proto/integrity.proto) on a directory with no chunk of the geometry
    IntegrityOptions o;
    o.chunkSize = 2u << 20;  // chunk_1 is not of this geometry: nothing to check, no GPU needed
    IntegrityService svc(o);
    EXPECT(svc.PauseJob(1) == INTEGRITY_OP_STATUS_FAILURE_UNKNOWN);
    EXPECT(svc.ScheduleJob(1, 7, dd) == INTEGRITY_OP_STATUS_SUCCESS);
    EXPECT(svc.ScheduleJob(1, 7, dd) == INTEGRITY_OP_STATUS_FAILURE_UNKNOWN);
    IntegrityJob j;
    EXPECT(svc.Wait(1, 20000, &j) && j.state == INTEGRITY_OP_STATE_FINISHED && j.progress == 100 && j.copyset == 7);
    EXPECT(svc.CancelJob(1) == INTEGRITY_OP_STATUS_FAILURE_UNKNOWN);
    EXPECT(svc.ScheduleJob(2, 7, dd + "/missing") == INTEGRITY_OP_STATUS_SUCCESS);
    EXPECT(svc.Wait(2, 20000, &j) && j.state == INTEGRITY_OP_STATE_FAILED && !j.error.empty());
    std::vector<IntegrityJob> all;
    EXPECT(svc.ListJobs(&all) == INTEGRITY_OP_STATUS_SUCCESS && all.size() == 2 && all[0].id == 1);
}

// GPU: the write path keeps the tables current (no false corruption), a write
// that skips its table is STALE (refreshed, never bad pages), bit rot is
// reported page-exact.
void IntegrityWritePath() {
    const uint32_t pb = 4096, chunk = 1u << 20, meta = 4096, n_chunks = 6, ppc = chunk / pb;
    const std::string root = MakeDir("integ_gpu"), dd = root + "/data", tdir = root + "/pcrc";
    mkdir(dd.c_str(), 0755);
    mkdir(tdir.c_str(), 0755);
    std::mt19937_64 rng(77);
    std::string pool((size_t)n_chunks * chunk, '\0');
    for (auto& c : pool) c = (char)(rng() & 0xFF);
    std::vector<std::string> paths;
    for (uint32_t c = 0; c < n_chunks; c++) {
        paths.push_back(dd + "/" + ChunkFileName(c + 1));
        WriteFile(paths.back(), MetaPage(c + 1) + pool.substr((size_t)c * chunk, chunk));
    }
    // the device pool (data of every chunk) + its CRC table, persisted per chunk
    void *d_pool = nullptr, *d_pc = nullptr, *d_src = nullptr, *d_log = nullptr, *d_work = nullptr;
    const uint64_t pool_bytes = pool.size(), n_pages = pool_bytes / pb;
    EXPECT(hipMalloc(&d_pool, pool_bytes) == hipSuccess && hipMalloc(&d_pc, n_pages * 4) == hipSuccess);
    EXPECT(hipMemcpy(d_pool, pool.data(), pool_bytes, hipMemcpyHostToDevice) == hipSuccess);
    EXPECT(cc_page_crc_dev(d_pool, n_pages, pb, (uint32_t*)d_pc, nullptr) == CC_OK);
    std::vector<uint32_t> pc(n_pages);
    auto persist = [&](uint32_t c) {
        EXPECT(hipMemcpy(pc.data(), d_pc, n_pages * 4, hipMemcpyDeviceToHost) == hipSuccess);
        EXPECT(cc_pcrc_store(paths[c].c_str(), meta, TablePath(tdir, ChunkFileName(c + 1)).c_str(),
                             pc.data() + (size_t)c * ppc, ppc, pb) == CC_OK);
    };
    for (uint32_t c = 0; c < n_chunks; c++) persist(c);
    // an ordered client write log: applied on the device (delta mode keeps the
    // CRC table current), written to the chunk files (the datastore's pwrite),
    // then the touched chunks' tables persisted
    const uint32_t n = 300, max_len = 4096, src_bytes = 1 << 16;
    std::string src(src_bytes, '\0');
    for (auto& c : src) c = (char)(rng() & 0xFF);
    std::vector<cc_update> log(n);
    std::vector<bool> touched(n_chunks, false);
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t len = 1 + (uint32_t)(rng() % max_len);
        const uint32_t c = (uint32_t)(rng() % (n_chunks - 1));  // the last chunk stays untouched
        const uint64_t dst = (uint64_t)c * chunk + rng() % (chunk - len);  // inside one chunk file
        log[i] = {dst, rng() % (src_bytes - len), len, 0};
        touched[c] = true;
    }
    EXPECT(hipMalloc(&d_src, src_bytes) == hipSuccess && hipMalloc(&d_log, n * sizeof(cc_update)) == hipSuccess);
    EXPECT(hipMemcpy(d_src, src.data(), src_bytes, hipMemcpyHostToDevice) == hipSuccess);
    EXPECT(hipMemcpy(d_log, log.data(), n * sizeof(cc_update), hipMemcpyHostToDevice) == hipSuccess);
    const uint64_t work = cc_apply_log_work_bytes(n, max_len, pb);
    EXPECT(hipMalloc(&d_work, work) == hipSuccess);
    EXPECT(cc_apply_log_delta_dev(d_pool, pool_bytes, pb, d_src, (const cc_update*)d_log, n, max_len, (uint32_t*)d_pc,
                                  d_work, work, nullptr) == CC_OK);
    EXPECT(hipDeviceSynchronize() == hipSuccess);
    for (const cc_update& u : log) {
        const uint32_t c = (uint32_t)(u.dst / chunk);
        const int fd = open(paths[c].c_str(), O_WRONLY);
        EXPECT(fd >= 0 && pwrite(fd, src.data() + u.src, u.len, meta + (u.dst % chunk)) == (ssize_t)u.len);
        close(fd);
    }
    for (uint32_t c = 0; c < n_chunks; c++)
        if (touched[c]) persist(c);
    IntegrityOptions o;
    o.chunkSize = chunk;
    o.batch = 4;
    IntegrityService svc2(o);
    IntegrityJob j;
    // the tables were stored within a clock tick of the pwrites: racy
    // (cc_pcrc_is_racy).  Job 1 re-stamps them once the clock has moved a tick
    // past the writes, so that bit rot with the mtime restored (job 3) is
    // provably not a same-tick write.
    usleep(50000);
    EXPECT(svc2.ScheduleJob(1, 1, dd) == INTEGRITY_OP_STATUS_SUCCESS);
    EXPECT(svc2.Wait(1, 60000, &j) && j.state == INTEGRITY_OP_STATE_FINISHED);
    EXPECT(j.results.size() == n_chunks);
    for (const auto& r : j.results) EXPECT(r.tableState == CC_TABLE_OK && r.badPages == 0);
    // a write that does not persist its table: stale (refreshed), no bad pages
    {
        const int fd = open(paths[2].c_str(), O_WRONLY);
        EXPECT(fd >= 0 && pwrite(fd, "stale!", 6, meta + 12345) == 6);
        close(fd);
        struct timespec ts[2] = {{0, UTIME_OMIT}, {0, UTIME_NOW}};
        utimensat(AT_FDCWD, paths[2].c_str(), ts, 0);  // a later write: mtime moves on
    }
    EXPECT(svc2.ScheduleJob(2, 1, dd) == INTEGRITY_OP_STATUS_SUCCESS);
    EXPECT(svc2.Wait(2, 60000, &j) && j.state == INTEGRITY_OP_STATE_FINISHED);
    for (const auto& r : j.results)
        EXPECT(r.badPages == 0 && r.tableState == (r.name == ChunkFileName(3) ? CC_TABLE_REFRESHED : CC_TABLE_OK));
    // bit rot (mtime unchanged): exactly the flipped page, of exactly that chunk
    {
        struct stat sb;
        EXPECT(stat(paths[4].c_str(), &sb) == 0);
        const int fd = open(paths[4].c_str(), O_RDWR);
        char b = 0;
        const off_t at = meta + 77 * pb + 9;
        EXPECT(fd >= 0 && pread(fd, &b, 1, at) == 1);
        b ^= 0x20;
        EXPECT(pwrite(fd, &b, 1, at) == 1);
        struct timespec ts[2] = {sb.st_atim, sb.st_mtim};
        EXPECT(futimens(fd, ts) == 0);
        close(fd);
    }
    EXPECT(svc2.ScheduleJob(3, 1, dd) == INTEGRITY_OP_STATUS_SUCCESS);
    EXPECT(svc2.Wait(3, 60000, &j) && j.state == INTEGRITY_OP_STATE_FINISHED);
    for (const auto& r : j.results) {
        if (r.name == ChunkFileName(5)) {
            EXPECT(r.tableState == CC_TABLE_OK && r.badPages == 1 && r.firstBad == 77 && r.badList.size() == 1 &&
                   r.badList[0] == 77);
        } else {
            EXPECT(r.badPages == 0 && r.tableState == CC_TABLE_OK);
        }
    }
    for (void* q : {d_pool, d_pc, d_src, d_log, d_work}) EXPECT(hipFree(q) == hipSuccess);
}

struct Case {
    const char* name;
    bool gpu;
    std::function<void()> fn;
};

}  // namespace

int main(int argc, char** argv) {
    const bool need_gpu = argc > 1 && strcmp(argv[1], "--gpu") == 0;
    char tmpl[] = "/tmp/cchost_XXXXXX";
    const char* t = mkdtemp(tmpl);
    if (!t) {
        perror("mkdtemp");
        return 2;
    }
    g_tmp = t;
    const bool have_gpu = cc_engine_init(nullptr) == CC_OK;
    if (need_gpu && !have_gpu) {
        fprintf(stderr, "no usable GPU: %s\n", cc_strerror(cc_engine_init(nullptr)));
        return 2;
    }
    const Case cases[] = {
        {"Crc32Vectors", false, Crc32Vectors},
        {"MetaPageEncodeDecode", false, MetaPageEncodeDecode},
        {"CompareMapCases", false, CompareMapCases},
        {"CopysetHashSmallFiles", false, CopysetHashSmallFiles},
        {"ChunkServiceHashRequests", false, ChunkServiceHashRequests},
        {"ChunkHashLongRanges", true, ChunkHashLongRanges},
        {"CopysetHashOneChunk", true, CopysetHashOneChunk},
        {"CopysetHashMixed", true, CopysetHashMixed},
        {"ScanCopysetMaps", true, ScanCopysetMaps},
        {"PoolScanShardRccl", true, PoolScanShardRccl},
        {"WriteLogBothModes", true, WriteLogBothModes},
        {"PerRequestWriteAndRead", true, PerRequestWriteAndRead},
        {"IntegrityTableAndService", false, IntegrityTableAndService},
        {"IntegrityWritePath", true, IntegrityWritePath},
    };
    int ran = 0, skipped = 0, failed_cases = 0;
    for (const Case& c : cases) {
        if (c.gpu && !have_gpu) {
            printf("[ SKIP ] %s (no GPU)\n", c.name);
            skipped++;
            continue;
        }
        const int before = g_fail;
        c.fn();
        ran++;
        const bool ok = g_fail == before;
        failed_cases += !ok;
        printf("[%s] %s\n", ok ? "  OK  " : " FAIL ", c.name);
    }
    printf("%d ran, %d failed, %d skipped\n", ran, failed_cases, skipped);
    if (have_gpu) cc_engine_fini();
    std::string rm = "rm -rf " + g_tmp;
    if (system(rm.c_str()) != 0) fprintf(stderr, "cleanup of %s failed\n", g_tmp.c_str());
    return failed_cases ? 1 : 0;
}
