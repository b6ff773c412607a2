// curve_amd/host/chunkserver_host.cpp -- see chunkserver_host.h.
#include "chunkserver_host.h"

#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <memory>

#include "../../include/curve_crc.h"

namespace cchost {

namespace {

// whole-range pread (EINTR-safe); false on error or short file
bool ReadFull(int fd, char* buf, size_t n, off_t off) {
    size_t got = 0;
    while (got < n) {
        const ssize_t r = pread(fd, buf + got, n - got, off + (off_t)got);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return false;
        got += (size_t)r;
    }
    return true;
}

struct Fd {
    int fd = -1;
    explicit Fd(const std::string& path) : fd(open(path.c_str(), O_RDONLY | O_CLOEXEC)) {}
    ~Fd() {
        if (fd >= 0) close(fd);
    }
};

// CRC32(0, buf[0, n)): pages on the GPU engine + a CPU tail, combined
// (INTEGRATION.md section 5); short buffers straight on the CPU primitive.
bool HashBuffer(const char* buf, size_t n, uint32_t* crc) {
    const size_t page = 4096;
    const size_t head = n / page * page;
    if (n < kCpuHashMax || head == 0) {
        *crc = crc32c_value(buf, n);
        return true;
    }
    std::vector<uint32_t> pc(head / page);
    if (cc_page_crc_host(buf, pc.size(), (uint32_t)page, pc.data()) != CC_OK) return false;
    uint32_t c = cc_fold_host(pc.data(), pc.size(), page);
    c = crc32c_combine(c, crc32c_value(buf + head, n - head), n - head);
    *crc = c;
    return true;
}

bool ListDir(const std::string& dir, std::vector<std::string>* names) {
    DIR* d = opendir(dir.c_str());
    if (!d) return false;
    while (struct dirent* e = readdir(d)) {
        if (strcmp(e->d_name, ".") == 0 || strcmp(e->d_name, "..") == 0) continue;
        names->emplace_back(e->d_name);
    }
    closedir(d);
    return true;
}

bool ParseChunkName(const std::string& name, uint64_t* id) {
    static const char kPrefix[] = "chunk_";
    if (name.compare(0, sizeof(kPrefix) - 1, kPrefix) != 0 || name.size() == sizeof(kPrefix) - 1) return false;
    uint64_t v = 0;
    for (size_t i = sizeof(kPrefix) - 1; i < name.size(); i++) {
        if (name[i] < '0' || name[i] > '9') return false;  // chunk_<id>_snap_<sn> is not a chunk
        v = v * 10 + (uint64_t)(name[i] - '0');
    }
    *id = v;
    return true;
}

}  // namespace

bool ScanOpCrc(const char* buf, size_t size, uint32_t* crc) { return HashBuffer(buf, size, crc); }

void ChunkFileMetaPage::encode(char* buf) const {
    size_t len = 0;
    auto put = [&](const void* p, size_t n) {
        memcpy(buf + len, p, n);
        len += n;
    };
    put(&version, sizeof(version));
    put(&sn, sizeof(sn));
    put(&correctedSn, sizeof(correctedSn));
    const uint64_t loc_size = location.size();  // size_t on the LP64 reference build
    put(&loc_size, sizeof(loc_size));
    if (loc_size > 0) {
        put(location.data(), loc_size);
        put(&bitmapBits, sizeof(bitmapBits));
        std::vector<uint8_t> bm((bitmapBits + 7) >> 3, 0);
        std::copy_n(bitmap.begin(), std::min(bm.size(), bitmap.size()), bm.begin());
        put(bm.data(), bm.size());
    }
    const uint32_t crc = crc32c_value(buf, len);
    memcpy(buf + len, &crc, sizeof(crc));
}

CSErrorCode ChunkFileMetaPage::decode(const char* buf, size_t size) {
    if (size < 25 + sizeof(uint32_t)) return CrcCheckError;
    size_t len = 0;
    auto get = [&](void* p, size_t n) {
        memcpy(p, buf + len, n);
        len += n;
    };
    get(&version, sizeof(version));
    get(&sn, sizeof(sn));
    get(&correctedSn, sizeof(correctedSn));
    uint64_t loc_size = 0;
    get(&loc_size, sizeof(loc_size));
    location.clear();
    bitmap.clear();
    bitmapBits = 0;
    if (loc_size > 0) {
        // a header that claims more bytes than the page holds cannot carry a
        // valid CRC: report it as one instead of reading past the page (the
        // reference trusts loc_size / bitmap bits here)
        if (loc_size > size - len || size - len - loc_size < sizeof(bitmapBits) + sizeof(uint32_t))
            return CrcCheckError;
        location.assign(buf + len, loc_size);
        len += loc_size;
        get(&bitmapBits, sizeof(bitmapBits));
        const size_t nb = ((size_t)bitmapBits + 7) >> 3;
        if (nb > size - len - sizeof(uint32_t)) return CrcCheckError;
        bitmap.assign(buf + len, buf + len + nb);
        len += nb;
    }
    uint32_t rec = 0;
    memcpy(&rec, buf + len, sizeof(rec));
    if (crc32c_value(buf, len) != rec) return CrcCheckError;
    if (version != FORMAT_VERSION && version != FORMAT_VERSION_V2) return IncompatibleError;
    return Success;
}

std::string ChunkFileName(uint64_t chunkId) { return "chunk_" + std::to_string(chunkId); }

CSErrorCode GetChunkHash(const DataStoreOptions& opt, uint64_t chunkId, off_t offset, size_t length,
                         std::string* hash) {
    const std::string path = opt.baseDir + "/" + ChunkFileName(chunkId);
    Fd f(path);
    if (f.fd < 0) return errno == ENOENT ? ChunkNotExistError : InternalError;
    std::unique_ptr<char[]> buf(new (std::nothrow) char[length ? length : 1]);
    if (!buf) return InternalError;
    if (length && !ReadFull(f.fd, buf.get(), length, offset)) return InternalError;
    uint32_t crc = 0;
    if (!HashBuffer(buf.get(), length, &crc)) return InternalError;
    *hash = std::to_string(crc);
    return Success;
}

CHUNK_OP_STATUS ChunkServiceGetChunkHash(const DataStoreOptions& opt, uint64_t chunkId, uint32_t offset,
                                         uint32_t length, std::string* hash) {
    // CheckRequestOffsetAndLength (chunk_service.cpp:580-588)
    if ((uint64_t)offset + length > opt.chunkSize || offset % opt.blockSize || length % opt.blockSize)
        return CHUNK_OP_STATUS_INVALID_REQUEST;
    const CSErrorCode rc = GetChunkHash(opt, chunkId, offset, length, hash);
    if (rc == Success) return CHUNK_OP_STATUS_SUCCESS;
    if (rc == ChunkNotExistError) {
        *hash = "0";
        return CHUNK_OP_STATUS_SUCCESS;
    }
    return CHUNK_OP_STATUS_FAILURE_UNKNOWN;
}

int GetCopysetHash(const std::string& dataDir, uint32_t chunkSize, uint32_t metaPageSize, std::string* hash) {
    std::vector<std::string> names;
    if (!ListDir(dataDir, &names)) return -1;
    std::sort(names.begin(), names.end());  // copyset_node.cpp:938
    if (names.empty()) {
        *hash = "0";
        return 0;
    }
    const uint64_t chunkFile = (uint64_t)chunkSize + metaPageSize;
    std::vector<uint64_t> sizes(names.size());
    std::vector<std::string> paths(names.size());
    std::vector<const char*> chunkPaths;
    std::vector<size_t> chunkIdx;
    for (size_t i = 0; i < names.size(); i++) {
        paths[i] = dataDir + "/" + names[i];
        struct stat sb;
        if (stat(paths[i].c_str(), &sb) != 0) return -1;
        sizes[i] = (uint64_t)sb.st_size;
        if (S_ISREG(sb.st_mode) && sizes[i] == chunkFile) {
            chunkPaths.push_back(paths[i].c_str());
            chunkIdx.push_back(i);
        }
    }
    std::vector<uint32_t> fileCrc(names.size(), 0);
    std::vector<bool> done(names.size(), false);
    if (!chunkPaths.empty()) {
        std::vector<cc_file_result> res(chunkPaths.size());
        const uint32_t slice = std::min<uint32_t>(4u << 20, chunkSize);
        if (cc_scan_files(chunkPaths.data(), chunkPaths.size(), chunkSize, metaPageSize, 4096, slice, 0, nullptr,
                          res.data()) != CC_OK)
            return -1;
        for (size_t k = 0; k < chunkIdx.size(); k++) {
            if (res[k].status < 0 && res[k].status != CC_EFORMAT) return -1;  // open/read failed
            if (res[k].status == 0) {
                fileCrc[chunkIdx[k]] = res[k].file_crc;
                done[chunkIdx[k]] = true;
            }
        }
    }
    uint32_t crc = 0;
    for (size_t i = 0; i < names.size(); i++) {
        if (done[i]) {
            crc = crc32c_combine(crc, fileCrc[i], sizes[i]);
            continue;
        }
        // not of the chunk geometry (or changed size under us): whole-file read
        Fd f(paths[i]);
        if (f.fd < 0) return -1;
        struct stat sb;
        if (fstat(f.fd, &sb) != 0) return -1;
        const size_t n = (size_t)sb.st_size;
        std::unique_ptr<char[]> buf(new (std::nothrow) char[n ? n : 1]);
        if (!buf) return -1;
        if (n && !ReadFull(f.fd, buf.get(), n, 0)) return -1;
        uint32_t c = 0;
        if (!HashBuffer(buf.get(), n, &c)) return -1;
        crc = crc32c_combine(crc, c, n);
    }
    *hash = std::to_string(crc);
    return 0;
}

bool ScanMap::operator==(const ScanMap& o) const {
    return logicalPoolId == o.logicalPoolId && copysetId == o.copysetId && chunkId == o.chunkId &&
           index == o.index && crc == o.crc && offset == o.offset && len == o.len;
}

bool CompareMap(const ScanMap& local, const std::vector<ScanMap>& followers, std::vector<ScanMap>* failed) {
    if (followers.size() != 2) return false;  // "waitingNum is 0 but there isn't three scanmap"
    if (local == followers[0] && local == followers[1]) return true;
    if (failed) failed->push_back(local);
    return false;
}

int ScanCopyset(const DataStoreOptions& opt, uint32_t logicalPoolId, uint32_t copysetId, uint32_t scanSize,
                uint64_t firstIndex, std::vector<ScanMap>* maps) {
    if (scanSize == 0 || scanSize > opt.chunkSize || opt.chunkSize % scanSize || !maps) return -1;
    std::vector<std::string> names;
    if (!ListDir(opt.baseDir, &names)) return -1;
    std::vector<uint64_t> ids;
    for (const auto& n : names) {
        uint64_t id;
        if (ParseChunkName(n, &id)) ids.push_back(id);
    }
    std::sort(ids.begin(), ids.end());
    std::vector<std::string> paths;
    std::vector<const char*> cpaths;
    for (uint64_t id : ids) paths.push_back(opt.baseDir + "/" + ChunkFileName(id));
    for (const auto& p : paths) cpaths.push_back(p.c_str());
    const uint32_t slices = opt.chunkSize / scanSize;
    std::vector<cc_file_result> res(ids.size());
    std::vector<uint32_t> sc((size_t)ids.size() * slices);
    if (!ids.empty() && cc_scan_files(cpaths.data(), ids.size(), opt.chunkSize, opt.metaPageSize, 4096, scanSize, 0,
                                      sc.data(), res.data()) != CC_OK)
        return -1;
    uint64_t index = firstIndex;
    for (size_t k = 0; k < ids.size(); k++) {
        if (res[k].status != 0) return -1;  // InternalError -> LOG(FATAL) in OnApply
        Fd f(paths[k]);
        char version = 0;
        if (f.fd < 0 || !ReadFull(f.fd, &version, 1, 0)) return -1;
        if ((uint8_t)version != FORMAT_VERSION_V2) continue;  // scan_manager.cpp:228-231
        maps->push_back(ScanMap{logicalPoolId, copysetId, ids[k], index++, res[k].meta_crc, 0, opt.metaPageSize});
        for (uint32_t j = 0; j < slices; j++)
            maps->push_back(ScanMap{logicalPoolId, copysetId, ids[k], index++, sc[k * slices + j],
                                    (uint64_t)j * scanSize, scanSize});
    }
    return 0;
}

}  // namespace cchost
