// curve_amd/host/integrity_service.h -- IntegrityService of proto/integrity.proto
// (ScheduleJob / CancelJob / PauseJob / ResumeJob / ListJobs, :55-61), which the
// reference declares and compiles (proto/BUILD:78) but never implements.  Same
// names, enums and message fields as the proto; the RPC plumbing (brpc
// IntegrityRequest / IntegrityResponse) stays with the chunkserver, which would
// forward each RPC to the method of the same name here.
//
// A job checks one copyset's data directory: its chunk files, in std::sort name
// order (a file named as a chunk whose size is not metapage + chunk is reported
// as CC_EFORMAT, FileFormatError in the reference), in batches of `batch`
// files, each batch one cc_integrity_check call
// (native pread into pinned staging, every data page rehashed on the GPU and
// compared with the chunk's per-page CRC table under <copyset>/pcrc/).  Pause
// and Cancel take effect at batch boundaries; a paused job resumes where it
// stopped.  One worker thread runs jobs FIFO.
#pragma once

#include <condition_variable>
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/curve_crc.h"

namespace cchost {

enum INTEGRITY_JOB_STATE {  // proto/integrity.proto:23-30
    INTEGRITY_OP_STATE_WAITING = 0,
    INTEGRITY_OP_STATE_RUNNING = 1,
    INTEGRITY_OP_STATE_CANCELED = 2,
    INTEGRITY_OP_STATE_FINISHED = 3,
    INTEGRITY_OP_STATE_PAUSED = 4,
    INTEGRITY_OP_STATE_FAILED = 5,
};

enum INTEGRITY_OP_STATUS {  // proto/integrity.proto:45-48
    INTEGRITY_OP_STATUS_SUCCESS = 0,
    INTEGRITY_OP_STATUS_FAILURE_UNKNOWN = 1,
};

// Outcome of one chunk file (new; the proto carries only job-level fields).
struct IntegrityFileResult {
    std::string name;
    int32_t status = 0;        // 0, -errno (-ENOENT: the chunk vanished mid-job), CC_EINVAL, CC_ECORRUPT (metapage),
                               // CC_EFORMAT (a chunk-named file whose size is not metapage + chunk)
    std::string error;         // text of a non-zero status ("vanished" for -ENOENT)
    uint32_t tableState = 0;   // CC_TABLE_*
    uint32_t badPages = 0;
    int64_t firstBad = -1;
    std::vector<uint32_t> badList;  // every bad page (up to the batch's list capacity)
};

struct IntegrityJob {  // proto/integrity.proto:32-39 + results
    int32_t id = 0;
    int32_t copyset = 0;
    INTEGRITY_JOB_STATE state = INTEGRITY_OP_STATE_WAITING;
    int32_t progress = 0;    // percent of the chunk files done
    int32_t sched_time = 0;
    int32_t start_time = 0;
    std::string dataDir;
    std::string error;
    std::vector<IntegrityFileResult> results;
};

struct IntegrityOptions {
    uint32_t chunkSize = 16u << 20;
    uint32_t metaPageSize = 4096;
    uint32_t pageSize = 4096;
    uint32_t batch = 16;          // chunk files per cc_integrity_check call
    uint32_t ioThreads = 0;  // readers of cc_scan_files (0 = cc_default_io_threads())
    bool createMissing = true;    // write a table for a chunk without one
    bool refreshStale = true;     // rewrite stale / corrupt tables from the current bytes
};

// <copyset>/data -> <copyset>/pcrc (outside the data directory: GetHash chains every file in it)
std::string TableDirFor(const std::string& dataDir);
std::string TablePath(const std::string& tableDir, const std::string& chunkName);
// chunk_<id> or chunk_<id>_snap_<sn> (FileNameOperator, datastore/filename_operator.h:55-62)
bool IsChunkFileName(const std::string& name);

class IntegrityService {
 public:
    explicit IntegrityService(const IntegrityOptions& opt = IntegrityOptions());
    ~IntegrityService();  // stops the worker after the current batch

    INTEGRITY_OP_STATUS ScheduleJob(int32_t id, int32_t copyset, const std::string& dataDir);
    INTEGRITY_OP_STATUS CancelJob(int32_t id);
    INTEGRITY_OP_STATUS PauseJob(int32_t id);
    INTEGRITY_OP_STATUS ResumeJob(int32_t id);
    INTEGRITY_OP_STATUS ListJobs(std::vector<IntegrityJob>* jobs) const;
    // test / tool helper: block until the job leaves WAITING/RUNNING (or timeout)
    bool Wait(int32_t id, int timeoutMs, IntegrityJob* out);
    // one job's fields without its per-file results (n = results so far), and
    // one result: O(1) reads for the C ABI (include/curve_integrity.h)
    bool JobInfo(int32_t id, IntegrityJob* out, size_t* nResults) const;
    bool FileResult(int32_t id, size_t k, IntegrityFileResult* out) const;

 private:
    void Run();
    void DoJob(IntegrityJob* job);
    INTEGRITY_OP_STATUS Move(int32_t id, std::initializer_list<INTEGRITY_JOB_STATE> from, INTEGRITY_JOB_STATE to);

    IntegrityOptions opt_;
    mutable std::mutex mu_;
    std::condition_variable cv_;
    std::map<int32_t, IntegrityJob> jobs_;
    std::vector<int32_t> order_;
    bool stop_ = false;
    std::thread worker_;
};

}  // namespace cchost
