// curve_amd/host/integrity_capi.cpp -- include/curve_integrity.h over
// cchost::IntegrityService: plain C structs across the boundary, the job state
// machine stays in integrity_service.cpp.
#include <string.h>

#include <new>

#include "../../include/curve_crc.h"
#include "../../include/curve_integrity.h"
#include "integrity_service.h"

struct cc_isvc {
    explicit cc_isvc(const cchost::IntegrityOptions& o) : svc(o) {}
    cchost::IntegrityService svc;
};

namespace {

void copy_str(char* dst, size_t cap, const std::string& s) {
    const size_t n = s.size() < cap - 1 ? s.size() : cap - 1;
    memcpy(dst, s.data(), n);
    dst[n] = 0;
}

}  // namespace

extern "C" {

cc_isvc* cc_isvc_create(const cc_isvc_opts* o) {
    cchost::IntegrityOptions opt;
    if (o) {
        if (o->chunk_bytes) opt.chunkSize = o->chunk_bytes;
        if (o->meta_bytes) opt.metaPageSize = o->meta_bytes;
        if (o->page_bytes) opt.pageSize = o->page_bytes;
        if (o->batch) opt.batch = o->batch;
        if (o->io_threads) opt.ioThreads = o->io_threads;
        opt.createMissing = o->create_missing != 0;
        opt.refreshStale = o->refresh_stale != 0;
    }
    if (opt.pageSize == 0 || opt.chunkSize % opt.pageSize) return nullptr;
    return new (std::nothrow) cc_isvc(opt);
}

void cc_isvc_destroy(cc_isvc* s) { delete s; }

int cc_isvc_schedule(cc_isvc* s, int32_t id, int32_t copyset, const char* dir) {
    if (!s || !dir) return cchost::INTEGRITY_OP_STATUS_FAILURE_UNKNOWN;
    return s->svc.ScheduleJob(id, copyset, dir);
}
int cc_isvc_cancel(cc_isvc* s, int32_t id) { return s ? s->svc.CancelJob(id) : 1; }
int cc_isvc_pause(cc_isvc* s, int32_t id) { return s ? s->svc.PauseJob(id) : 1; }
int cc_isvc_resume(cc_isvc* s, int32_t id) { return s ? s->svc.ResumeJob(id) : 1; }

int cc_isvc_list(cc_isvc* s, int32_t* ids, uint64_t cap, uint64_t* n) {
    if (!s || !n || (cap && !ids)) return CC_EINVAL;
    std::vector<cchost::IntegrityJob> jobs;
    s->svc.ListJobs(&jobs);
    for (uint64_t k = 0; k < jobs.size() && k < cap; k++) ids[k] = jobs[k].id;
    *n = jobs.size();
    return CC_OK;
}

int cc_isvc_job_info(cc_isvc* s, int32_t id, cc_isvc_job* out) {
    if (!s || !out) return CC_EINVAL;
    cchost::IntegrityJob j;
    size_t n = 0;
    if (!s->svc.JobInfo(id, &j, &n)) return CC_EINVAL;
    out->id = j.id;
    out->copyset = j.copyset;
    out->state = j.state;
    out->progress = j.progress;
    out->sched_time = j.sched_time;
    out->start_time = j.start_time;
    out->n_results = n;
    copy_str(out->error, sizeof(out->error), j.error);
    return CC_OK;
}

int cc_isvc_file_result(cc_isvc* s, int32_t id, uint64_t k, cc_isvc_file* out, uint32_t* bad, uint64_t bad_cap) {
    if (!s || !out || (bad_cap && !bad)) return CC_EINVAL;
    cchost::IntegrityFileResult r;
    if (!s->svc.FileResult(id, (size_t)k, &r)) return CC_EINVAL;
    copy_str(out->name, sizeof(out->name), r.name);
    out->status = r.status;
    out->table_state = r.tableState;
    out->bad_pages = r.badPages;
    out->first_bad = r.firstBad;
    out->n_bad_listed = (uint32_t)r.badList.size();
    for (uint64_t q = 0; q < r.badList.size() && q < bad_cap; q++) bad[q] = r.badList[q];
    return CC_OK;
}

int cc_isvc_wait(cc_isvc* s, int32_t id, int32_t timeout_ms) {
    if (!s) return CC_EINVAL;
    cchost::IntegrityJob j;
    if (!s->svc.JobInfo(id, &j, nullptr)) return CC_EINVAL;
    return s->svc.Wait(id, timeout_ms, nullptr) ? 1 : 0;
}

}  // extern "C"
