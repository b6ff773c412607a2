// curve_amd/host/integrity_service.cpp -- see integrity_service.h.
#include "integrity_service.h"

#include <dirent.h>
#include <errno.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>

#include <algorithm>
#include <chrono>

namespace cchost {

namespace {
// libcurvecrc's own codes first (CC_ECORRUPT, CC_EHIP, CC_ESTALE ... sit inside
// the errno range and would read as unrelated errno text), then errno
std::string ErrText(int rc) {
    const char* t = cc_strerror(rc);
    if (strcmp(t, "unknown error") != 0) return t;
    return rc < 0 && rc > -4096 ? strerror(-rc) : t;
}
}  // namespace

std::string TableDirFor(const std::string& dataDir) {
    std::string d = dataDir;
    while (d.size() > 1 && d.back() == '/') d.pop_back();
    const size_t slash = d.rfind('/');
    return (slash == std::string::npos ? std::string(".") : d.substr(0, slash)) + "/pcrc";
}

std::string TablePath(const std::string& tableDir, const std::string& chunkName) {
    return tableDir + "/" + chunkName + ".pcrc";
}

// FileNameOperator::ParseFileName (datastore/filename_operator.h:55-62):
// "chunk_<id>" (CHUNK) or "chunk_<id>_snap_<sn>" (SNAPSHOT), decimal ids
bool IsChunkFileName(const std::string& name) {
    auto digits = [&](size_t& i) {
        const size_t s = i;
        while (i < name.size() && name[i] >= '0' && name[i] <= '9') i++;
        return i > s;
    };
    if (name.compare(0, 6, "chunk_") != 0) return false;
    size_t i = 6;
    if (!digits(i)) return false;
    if (i == name.size()) return true;
    if (name.compare(i, 6, "_snap_") != 0) return false;
    i += 6;
    return digits(i) && i == name.size();
}

IntegrityService::IntegrityService(const IntegrityOptions& opt) : opt_(opt) {
    worker_ = std::thread([this] { Run(); });
}

IntegrityService::~IntegrityService() {
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    worker_.join();
}

INTEGRITY_OP_STATUS IntegrityService::ScheduleJob(int32_t id, int32_t copyset, const std::string& dataDir) {
    std::lock_guard<std::mutex> lk(mu_);
    if (jobs_.count(id)) return INTEGRITY_OP_STATUS_FAILURE_UNKNOWN;
    IntegrityJob j;
    j.id = id;
    j.copyset = copyset;
    j.dataDir = dataDir;
    j.sched_time = (int32_t)time(nullptr);
    jobs_[id] = j;
    order_.push_back(id);
    cv_.notify_all();
    return INTEGRITY_OP_STATUS_SUCCESS;
}

INTEGRITY_OP_STATUS IntegrityService::Move(int32_t id, std::initializer_list<INTEGRITY_JOB_STATE> from,
                                           INTEGRITY_JOB_STATE to) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = jobs_.find(id);
    if (it == jobs_.end() || std::find(from.begin(), from.end(), it->second.state) == from.end())
        return INTEGRITY_OP_STATUS_FAILURE_UNKNOWN;
    it->second.state = to;
    cv_.notify_all();
    return INTEGRITY_OP_STATUS_SUCCESS;
}

INTEGRITY_OP_STATUS IntegrityService::CancelJob(int32_t id) {
    return Move(id, {INTEGRITY_OP_STATE_WAITING, INTEGRITY_OP_STATE_RUNNING, INTEGRITY_OP_STATE_PAUSED},
                INTEGRITY_OP_STATE_CANCELED);
}

INTEGRITY_OP_STATUS IntegrityService::PauseJob(int32_t id) {
    return Move(id, {INTEGRITY_OP_STATE_WAITING, INTEGRITY_OP_STATE_RUNNING}, INTEGRITY_OP_STATE_PAUSED);
}

INTEGRITY_OP_STATUS IntegrityService::ResumeJob(int32_t id) {
    return Move(id, {INTEGRITY_OP_STATE_PAUSED}, INTEGRITY_OP_STATE_WAITING);
}

INTEGRITY_OP_STATUS IntegrityService::ListJobs(std::vector<IntegrityJob>* jobs) const {
    if (!jobs) return INTEGRITY_OP_STATUS_FAILURE_UNKNOWN;
    std::lock_guard<std::mutex> lk(mu_);
    jobs->clear();
    for (int32_t id : order_) jobs->push_back(jobs_.at(id));
    return INTEGRITY_OP_STATUS_SUCCESS;
}

bool IntegrityService::JobInfo(int32_t id, IntegrityJob* out, size_t* nResults) const {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = jobs_.find(id);
    if (it == jobs_.end()) return false;
    const IntegrityJob& j = it->second;
    out->id = j.id;
    out->copyset = j.copyset;
    out->state = j.state;
    out->progress = j.progress;
    out->sched_time = j.sched_time;
    out->start_time = j.start_time;
    out->dataDir = j.dataDir;
    out->error = j.error;
    out->results.clear();
    if (nResults) *nResults = j.results.size();
    return true;
}

bool IntegrityService::FileResult(int32_t id, size_t k, IntegrityFileResult* out) const {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = jobs_.find(id);
    if (it == jobs_.end() || k >= it->second.results.size()) return false;
    *out = it->second.results[k];
    return true;
}

bool IntegrityService::Wait(int32_t id, int timeoutMs, IntegrityJob* out) {
    std::unique_lock<std::mutex> lk(mu_);
    auto it = jobs_.find(id);
    if (it == jobs_.end()) return false;
    const bool done = cv_.wait_for(lk, std::chrono::milliseconds(timeoutMs), [&] {
        const INTEGRITY_JOB_STATE s = jobs_.at(id).state;
        return s != INTEGRITY_OP_STATE_WAITING && s != INTEGRITY_OP_STATE_RUNNING;
    });
    if (out) *out = jobs_.at(id);
    return done;
}

void IntegrityService::Run() {
    for (;;) {
        IntegrityJob* job = nullptr;
        {
            std::unique_lock<std::mutex> lk(mu_);
            auto next = [&]() -> int32_t {
                for (int32_t i : order_)
                    if (jobs_.at(i).state == INTEGRITY_OP_STATE_WAITING) return i;
                return -1;
            };
            cv_.wait(lk, [&] { return stop_ || next() >= 0; });
            if (stop_) return;
            job = &jobs_.at(next());  // map nodes are stable; the job's fields are touched under mu_
            job->state = INTEGRITY_OP_STATE_RUNNING;
            if (!job->start_time) job->start_time = (int32_t)time(nullptr);
        }
        DoJob(job);
    }
}

void IntegrityService::DoJob(IntegrityJob* job) {
    std::string dataDir, error;
    std::vector<std::string> done;
    {
        std::lock_guard<std::mutex> lk(mu_);
        dataDir = job->dataDir;
        for (const auto& r : job->results) done.push_back(r.name);
    }
    auto fail = [&](const std::string& why) {
        std::lock_guard<std::mutex> lk(mu_);
        job->state = INTEGRITY_OP_STATE_FAILED;
        job->error = why;
        cv_.notify_all();
    };
    // the copyset's chunk files in std::sort name order (as GetHash lists them):
    // every regular file of the chunk geometry, and every file NAMED as a chunk
    // or snapshot (FileNameOperator, datastore/filename_operator.h:55-62) whose
    // size is not metapage + chunk -- a truncated or extended chunk is exactly
    // the damage a scan exists to find; CSChunkFile::Open reports it as
    // FileFormatError (chunkserver_chunkfile.cpp:233-238), so it becomes that
    // file's result (CC_EFORMAT), not a silent omission
    const uint64_t fileBytes = (uint64_t)opt_.chunkSize + opt_.metaPageSize;
    std::vector<std::string> names;
    std::vector<std::string> misfit;  // chunk-named, wrong size (sorted below)
    DIR* d = opendir(dataDir.c_str());
    if (!d) return fail("cannot list " + dataDir + ": " + strerror(errno));
    while (struct dirent* e = readdir(d)) {
        if (!strcmp(e->d_name, ".") || !strcmp(e->d_name, "..")) continue;
        struct stat sb;
        const std::string p = dataDir + "/" + e->d_name;
        if (stat(p.c_str(), &sb) != 0 || !S_ISREG(sb.st_mode)) continue;
        if ((uint64_t)sb.st_size == fileBytes) {
            names.push_back(e->d_name);
        } else if (IsChunkFileName(e->d_name)) {
            names.push_back(e->d_name);
            misfit.push_back(e->d_name);
        }
    }
    closedir(d);
    std::sort(names.begin(), names.end());
    std::sort(misfit.begin(), misfit.end());
    std::sort(done.begin(), done.end());
    std::vector<std::string> todo;
    for (const auto& n : names)
        if (!std::binary_search(done.begin(), done.end(), n)) todo.push_back(n);
    const std::string tdir = TableDirFor(dataDir);
    if (mkdir(tdir.c_str(), 0755) != 0 && errno != EEXIST) return fail("cannot create " + tdir);
    const uint32_t n_pages = opt_.chunkSize / opt_.pageSize;
    const uint64_t batch = opt_.batch ? opt_.batch : 16;
    for (size_t b0 = 0; b0 < todo.size(); b0 += batch) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (stop_ || job->state != INTEGRITY_OP_STATE_RUNNING) {  // paused / canceled at a batch boundary
                cv_.notify_all();
                return;
            }
        }
        const size_t nb = std::min<size_t>(batch, todo.size() - b0);
        std::vector<IntegrityFileResult> out(nb);
        std::vector<std::string> cp, tp;
        std::vector<size_t> at;  // out index of each file checked on the device
        for (size_t k = 0; k < nb; k++) {
            out[k].name = todo[b0 + k];
            if (std::binary_search(misfit.begin(), misfit.end(), out[k].name)) {
                out[k].status = CC_EFORMAT;
                out[k].tableState = CC_TABLE_MISSING;  // no table is read or written for it
                out[k].error = ErrText(CC_EFORMAT);
                continue;
            }
            cp.push_back(dataDir + "/" + out[k].name);
            tp.push_back(TablePath(tdir, out[k].name));
            at.push_back(k);
        }
        const size_t nc = at.size();
        std::vector<const char*> cpp(nc), tpp(nc);
        for (size_t k = 0; k < nc; k++) {
            cpp[k] = cp[k].c_str();
            tpp[k] = tp[k].c_str();
        }
        cc_integrity_opts o = {opt_.chunkSize, opt_.metaPageSize, opt_.pageSize, opt_.ioThreads,
                               opt_.createMissing ? 1u : 0u, opt_.refreshStale ? 1u : 0u};
        std::vector<cc_integrity_result> res(nc);
        const uint64_t cap = (uint64_t)nc * n_pages;
        std::vector<uint64_t> bad(cap);
        uint64_t nbad = 0;
        if (nc) {
            const int rc = cc_integrity_check(cpp.data(), tpp.data(), nc, &o, res.data(), bad.data(), cap, &nbad);
            if (rc) return fail(std::string("cc_integrity_check: ") + ErrText(rc));
        }
        // a file's own failure (metapage header CRC -> CC_ECORRUPT, unreadable,
        // -ENOENT: deleted between the listing and the check, or a size that
        // changed since the listing -> CC_EFORMAT) is that file's result, never
        // the job's: the rest of the copyset is still checked
        for (size_t k = 0; k < nc; k++) {
            IntegrityFileResult& r = out[at[k]];
            r.status = res[k].status;
            r.tableState = res[k].table_state;
            r.badPages = res[k].bad_pages;
            r.firstBad = res[k].first_bad;
            if (res[k].status) r.error = res[k].status == -ENOENT ? "vanished" : ErrText(res[k].status);
        }
        for (uint64_t q = 0; q < std::min(nbad, cap); q++) out[at[bad[q] >> 32]].badList.push_back((uint32_t)bad[q]);
        std::lock_guard<std::mutex> lk(mu_);
        for (auto& r : out) job->results.push_back(std::move(r));
        // percent of ALL the listed chunk files, format errors included
        job->progress = (int32_t)(100 * job->results.size() / std::max<size_t>(1, names.size()));
    }
    std::lock_guard<std::mutex> lk(mu_);
    if (job->state == INTEGRITY_OP_STATE_RUNNING) {
        job->state = INTEGRITY_OP_STATE_FINISHED;
        job->progress = 100;
    }
    cv_.notify_all();
}

}  // namespace cchost
