// curve_amd/host/chunkserver_host.h -- the chunkserver-side surfaces of the
// checksum path, in C++ (the reference's language), built on the C ABI of
// libcurvecrc (include/curve_crc.h).  Same names, argument meaning and error
// behaviour as the reference operators they mirror:
//
//   ChunkFileMetaPage::encode/decode   src/chunkserver/datastore/chunkserver_chunkfile.cpp:64-130
//   CSErrorCode                        src/chunkserver/datastore/define.h:44-76
//   CSChunkFile::GetHash               chunkserver_chunkfile.cpp:785-811 (raw FILE range)
//   ChunkServiceImpl::GetChunkHash     src/chunkserver/chunk_service.cpp:500-558, :580-588
//   CopysetNode::GetHash               src/chunkserver/copyset_node.cpp:925-975
//   ScanMap / CompareMap               proto/scan.proto:23-31, scan_manager.cpp:367-409
//   ScanManager::ScanJobProcess +
//   ScanChunkRequest::OnApply          scan_manager.cpp:210-296, op_request.cpp:769-820
//
// Bulk bytes (whole chunk files, scan slices, long hash ranges) are hashed by
// the GPU engine; short buffers (metapage headers, hash ranges under
// kCpuHashMax) use the CPU primitive crc32c_* -- the drop-in for
// curve::common::CRC32, chosen for latency, never as a fallback: when the
// engine is unavailable the bulk calls fail (InternalError / -1).
#pragma once

#include <sys/types.h>

#include <cstdint>
#include <string>
#include <vector>

namespace cchost {

enum CSErrorCode {
    Success = 0,
    InternalError = 1,
    IncompatibleError = 2,
    CrcCheckError = 3,
    FileFormatError = 4,
    ChunkNotExistError = 8,
    InvalidArgError = 10,
};

// proto/chunk.proto:74-88 (the subset GetChunkHash returns)
enum CHUNK_OP_STATUS {
    CHUNK_OP_STATUS_SUCCESS = 0,
    CHUNK_OP_STATUS_INVALID_REQUEST = 4,
    CHUNK_OP_STATUS_CHUNK_NOTEXIST = 7,
    CHUNK_OP_STATUS_FAILURE_UNKNOWN = 8,
};

constexpr uint8_t FORMAT_VERSION = 1;     // datastore/define.h:39
constexpr uint8_t FORMAT_VERSION_V2 = 2;  // datastore/define.h:40
// Hash ranges below this stay on the CPU primitive.  Measured per call on the
// MI355X box (bench.py scan_op.latency_by_size_1thread), with the
// primitive's fold + crc32q split (~100 GiB/s a core on the EPYC host): the CPU
// call is faster at every size (4 MiB: 39 vs 113 us; 16 MiB: 162 vs 336 us), and
// a GPU call (~12-18 us of host CPU whatever its size) costs less host CPU from
// ~2 MiB (2 MiB: 18 vs 19 us; a 4 MiB scan slice: 15 vs 39 us).  The cutoff
// routes for host CPU, since the reference paces its scan anyway.
constexpr size_t kCpuHashMax = 2 << 20;

struct ChunkFileMetaPage {
    uint8_t version = FORMAT_VERSION_V2;
    uint64_t sn = 0;
    uint64_t correctedSn = 0;
    std::string location;            // clone chunks only
    uint32_t bitmapBits = 0;         // clone chunks only
    std::vector<uint8_t> bitmap;     // (bitmapBits + 7) / 8 bytes
    // writes the header + its CRC32 into buf (which the caller zeroed, one
    // metapage long); layout as the reference: version u8 | sn u64 |
    // correctedSn u64 | loc_size size_t [| location | bits u32 | bitmap] | crc u32
    void encode(char* buf) const;
    // size = bytes readable at buf (the metapage); a header that does not fit
    // in it is CrcCheckError
    CSErrorCode decode(const char* buf, size_t size = 4096);
};

struct DataStoreOptions {
    std::string baseDir;                  // copyset data directory (chunk_<id> files)
    uint32_t chunkSize = 16u << 20;
    uint32_t metaPageSize = 4096;
    uint32_t blockSize = 4096;            // request alignment (chunk_service.cpp:587)
};

std::string ChunkFileName(uint64_t chunkId);                      // filename_operator.h:55-57

// CSChunkFile::GetHash: to_string(CRC32(0, file[offset, offset+length))) over
// the raw chunk FILE (metapage at file offset 0).  A range past the end of the
// file is InternalError (the reference would hash whatever its buffer held).
CSErrorCode GetChunkHash(const DataStoreOptions& opt, uint64_t chunkId, off_t offset, size_t length,
                         std::string* hash);

// ChunkServiceImpl::GetChunkHash: request validation (offset + length within
// chunkSize, both blockSize aligned), a missing chunk answers SUCCESS + "0".
CHUNK_OP_STATUS ChunkServiceGetChunkHash(const DataStoreOptions& opt, uint64_t chunkId, uint32_t offset,
                                         uint32_t length, std::string* hash);

// CopysetNode::GetHash: 0 and the chained CRC of every file of dataDir in
// std::sort name order ("0" when empty); -1 when listing, opening, fstat or
// reading any file fails.
int GetCopysetHash(const std::string& dataDir, uint32_t chunkSize, uint32_t metaPageSize, std::string* hash);

struct ScanMap {
    uint32_t logicalPoolId = 0;
    uint32_t copysetId = 0;
    uint64_t chunkId = 0;
    uint64_t index = 0;
    uint32_t crc = 0;
    uint64_t offset = 0;
    uint64_t len = 0;
    bool operator==(const ScanMap& o) const;
};

// ScanManager::CompareMap: consistent only when the leader's map equals BOTH
// followers' maps in every field; an inconsistent leader map goes to *failed.
// Fewer than two follower maps: not consistent, nothing failed (logged only).
bool CompareMap(const ScanMap& local, const std::vector<ScanMap>& followers, std::vector<ScanMap>* failed);

// The CRC ScanChunkRequest::OnApply / OnApplyFromLog puts in ScanMap.crc for
// one scan op's buffer (`crc = CRC32(readBuffer, size)`, op_request.cpp:794,
// :847): the 4 MiB slice's pages on the GPU engine (cc_page_crc_host, a lane
// of its own per concurrent caller) folded on the host, a buffer under
// kCpuHashMax (the 4 KiB metapage op) on the CPU primitive.  Thread-safe; false
// when the engine call fails (the apply thread's InternalError, :813-815).
bool ScanOpCrc(const char* buf, size_t size, uint32_t* crc);

// One scan job over a copyset's chunk files: for every chunk_<id> (ascending
// id; snapshots are not in the ChunkMap) whose metapage is FORMAT_VERSION_V2,
// the metapage op then chunkSize/scanSize data slices, each a ScanMap as
// ScanChunkRequest::OnApply builds it, `index` counting from firstIndex.
// scanSize must divide chunkSize (ScanManager::Init, scan_manager.cpp:43-48).
// Returns 0, or -1 (bad geometry, unreadable chunk file, engine failure).
int ScanCopyset(const DataStoreOptions& opt, uint32_t logicalPoolId, uint32_t copysetId, uint32_t scanSize,
                uint64_t firstIndex, std::vector<ScanMap>* maps);

}  // namespace cchost
