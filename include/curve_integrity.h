/* include/curve_integrity.h -- C ABI of the host layer's IntegrityService
 * (curve_amd/host/integrity_service.h), the service proto/integrity.proto
 * declares (IntegrityService: ScheduleJob / CancelJob / PauseJob / ResumeJob /
 * ListJobs, :55-61) and the reference never implements.  Library:
 * curve_amd/host/libcurvehost.so (links libcurvecrc.so).
 *
 * This is what a brpc service stub or any non-C++ caller binds (the Python
 * mirror curve_amd/integrity.py is a ctypes facade over it: ONE job state
 * machine, in C++).  Return values of the job-control calls are
 * INTEGRITY_OP_STATUS (0 = SUCCESS, 1 = FAILURE_UNKNOWN, proto/integrity.proto:45-48);
 * the rest return 0 or a negative CC_* code. */
#ifndef CURVE_INTEGRITY_H_
#define CURVE_INTEGRITY_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cc_isvc cc_isvc; /* opaque: one IntegrityService (one worker thread) */

typedef struct cc_isvc_opts {   /* cchost::IntegrityOptions */
    uint32_t chunk_bytes;       /* 16 MiB (conf/chunkserver.conf global.chunk_size) */
    uint32_t meta_bytes;        /* 4 KiB metapage (global.meta_page_size) */
    uint32_t page_bytes;        /* 4 KiB (the per-page CRC granularity) */
    uint32_t batch;             /* chunk files per cc_integrity_check call */
    uint32_t io_threads;
    uint32_t create_missing;
    uint32_t refresh_stale;
} cc_isvc_opts;

typedef struct cc_isvc_job {    /* IntegrityJob, proto/integrity.proto:32-39, + counts */
    int32_t id;
    int32_t copyset;
    int32_t state;              /* INTEGRITY_JOB_STATE, proto/integrity.proto:23-30 */
    int32_t progress;           /* percent of the chunk files done */
    int32_t sched_time;
    int32_t start_time;
    uint64_t n_results;         /* chunk files checked so far */
    char error[256];            /* job-level error (state FAILED), NUL-terminated */
} cc_isvc_job;

typedef struct cc_isvc_file {   /* IntegrityFileResult */
    char name[256];
    int32_t status;             /* 0; -errno (-ENOENT: vanished mid-job); CC_ECORRUPT (metapage header) */
    uint32_t table_state;       /* CC_TABLE_* of include/curve_crc.h */
    uint32_t bad_pages;
    uint32_t n_bad_listed;      /* entries of its bad-page list */
    int64_t first_bad;
} cc_isvc_file;

cc_isvc* cc_isvc_create(const cc_isvc_opts* opts); /* NULL opts = defaults; NULL on failure */
void cc_isvc_destroy(cc_isvc* s);                   /* stops the worker after its current batch */
int cc_isvc_schedule(cc_isvc* s, int32_t id, int32_t copyset, const char* data_dir);
int cc_isvc_cancel(cc_isvc* s, int32_t id);
int cc_isvc_pause(cc_isvc* s, int32_t id);
int cc_isvc_resume(cc_isvc* s, int32_t id);
/* ListJobs: up to cap job ids in schedule order; *n = all */
int cc_isvc_list(cc_isvc* s, int32_t* ids, uint64_t cap, uint64_t* n);
int cc_isvc_job_info(cc_isvc* s, int32_t id, cc_isvc_job* out);      /* CC_EINVAL: unknown id */
/* result k of job id (0 <= k < n_results) and up to bad_cap of its bad pages */
int cc_isvc_file_result(cc_isvc* s, int32_t id, uint64_t k, cc_isvc_file* out, uint32_t* bad, uint64_t bad_cap);
/* block until the job leaves WAITING/RUNNING: 1 = it did, 0 = timeout, CC_EINVAL = unknown id */
int cc_isvc_wait(cc_isvc* s, int32_t id, int32_t timeout_ms);

#ifdef __cplusplus
}
#endif
#endif /* CURVE_INTEGRITY_H_ */
