// curve_amd/csrc/pool.hip -- full-pool integrity scan sharded over the GPUs of
// a node (BASELINE config 5): one process per GPU, one rank's scan
// pass as ONE C call, and the per-copyset digest exchange over RCCL (xGMI).
//
// Reference: CopysetNode::GetHash (src/chunkserver/copyset_node.cpp:925-975)
// chains CRC32 over the copyset's files in std::sort name order; the scan
// hasher (ScanChunkRequest::OnApply, src/chunkserver/op_request.cpp:769-820)
// produces one ScanMap.crc per metapage / 4 MiB slice op that
// ScanManager::ScanJobProcess schedules (scan_manager.cpp:210-296).  The
// reference has no multi-GPU (or multi-process) form of either; the sharding is
// new and is exact because the chain is linear over GF(2):
//     V(f1 || .. || fn) = XOR_i shift(V(fi), bytes after fi)
// so each rank contributes order-free XOR partials for the files it holds and
// one all-gather of 4 B per copyset per rank completes every digest.  XOR is
// not an RCCL reduction op (sum/prod/min/max/avg), hence all-gather + a local
// XOR fold rather than all-reduce; the payload (4 B x copysets x ranks) is
// latency-bound, far below one xGMI link's bandwidth.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <string.h>

#include <stdlib.h>

#include <chrono>
#include <mutex>
#include <thread>

#include "../../include/curve_crc.h"
#include "kernels.h"

struct cc_comm {
    ncclComm_t nc = nullptr;     // null once aborted by cc_comm_wait (a peer gone)
    int nranks = 0, rank = 0, device = -1;
    uint32_t* gather = nullptr;  // nranks x cap words of all-gather scratch on `device`
    uint64_t cap = 0;
    hipEvent_t done = nullptr;   // cc_comm_wait's completion marker
    uint32_t stall_ms = 0;       // failpoint only: $CC_INJECT_EXCHANGE_STALL_MS, read once at init
    uint32_t* stall_abort = nullptr;  // failpoint only: host-mapped word the stall kernel polls
    uint32_t* stall_word = nullptr;   // its device address
    std::mutex mu;               // guards the scratch (re)allocation and the event
};

static_assert(CC_COMM_ID_BYTES == sizeof(ncclUniqueId), "RCCL unique id size");

namespace {

int map_hip(hipError_t e) {
    if (e == hipSuccess) return CC_OK;
    if (e == hipErrorOutOfMemory) return CC_ENOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return CC_ENODEV;
    return CC_EHIP;
}

int map_nccl(ncclResult_t r) { return r == ncclSuccess ? CC_OK : CC_ECOMM; }

constexpr uint32_t kDefaultInitTimeoutMs = 120000;

uint32_t init_timeout_ms(uint32_t asked) {
    if (asked) return asked;
    if (const char* e = getenv("CC_COMM_INIT_TIMEOUT_MS")) {
        const long v = strtol(e, nullptr, 10);
        if (v > 0) return (uint32_t)v;
    }
    return kDefaultInitTimeoutMs;
}

// The communicator is non-blocking (ncclConfig_t.blocking = 0): every call may
// return ncclInProgress, and the next call on it may only be issued once
// ncclCommGetAsyncError reports the state left ncclInProgress.  Polls that
// state until `deadline`; ncclInProgress past it = CC_ETIMEDOUT (the caller
// aborts the communicator).  This is what keeps a rank whose peers never join
// (one rank's init failed before it reached RCCL) from blocking forever inside
// the bootstrap, as a blocking ncclCommInitRank would.
int settle(ncclComm_t nc, ncclResult_t r, std::chrono::steady_clock::time_point deadline) {
    while (r == ncclInProgress) {
        if (std::chrono::steady_clock::now() > deadline) return CC_ETIMEDOUT;
        std::this_thread::sleep_for(std::chrono::microseconds(50));
        if (ncclCommGetAsyncError(nc, &r) != ncclSuccess) return CC_ECOMM;
    }
    return map_nccl(r);
}

// enqueue-side wait of an already initialised communicator: bounded as well
// (a collective's enqueue never waits for peers, so this is microseconds)
int settle_call(ncclComm_t nc, ncclResult_t r) {
    return settle(nc, r, std::chrono::steady_clock::now() + std::chrono::seconds(60));
}

constexpr uint32_t kDefaultWaitTimeoutMs = 60000;

uint32_t wait_timeout_ms(uint32_t asked) {
    if (asked) return asked;
    if (const char* e = getenv("CC_COMM_WAIT_TIMEOUT_MS")) {
        const long v = strtol(e, nullptr, 10);
        if (v > 0) return (uint32_t)v;
    }
    return kDefaultWaitTimeoutMs;
}

// Failure injection (tests only; the reference's libfiu failpoints play this
// role, test/failpoint/): $CC_INJECT_EXCHANGE_STALL_MS > 0 when a communicator
// is created makes every digest exchange on it first spin one wave on the
// stream for that long (at most 30 s), as a collective whose peer stopped
// participating after init would sit in its kernel.  The variable is read once,
// in cc_comm_init: the exchange path itself never consults the environment.  cc_comm_wait must then give up at its deadline.  Like RCCL's own
// kernels, which poll the communicator's abort flag, the stall also ends as
// soon as cc_comm_wait raises the comm's host-mapped abort word (an abort
// cannot preempt a kernel: without the word it would wait out the stall).
uint32_t injected_stall_ms() {
    const char* e = getenv("CC_INJECT_EXCHANGE_STALL_MS");
    if (!e) return 0;
    const long v = strtol(e, nullptr, 10);
    return v <= 0 ? 0u : (uint32_t)(v < 30000 ? v : 30000);
}

// s_memrealtime runs at a constant 100 MHz on gfx9: 10 ns a tick.  One wave;
// every exit path is bounded by the tick count.
__global__ void stall_kernel(uint64_t ticks, const uint32_t* abort_word) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks &&
           __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u)
        __builtin_amdgcn_s_sleep(127);
}

}  // namespace

extern "C" {

static int comm_release(cc_comm* comm, bool abort);
static int comm_release_abort(cc_comm* comm) { return comm_release(comm, true); }

int cc_comm_unique_id(void* id, size_t bytes) {
    if (!id || bytes < sizeof(ncclUniqueId)) return CC_EINVAL;
    ncclUniqueId u;
    const int rc = map_nccl(ncclGetUniqueId(&u));
    if (rc) return rc;
    memcpy(id, &u, sizeof(u));
    return CC_OK;
}

int cc_comm_init_timeout(cc_comm** comm, int nranks, int rank, const void* id, size_t bytes, uint32_t timeout_ms) {
    if (!comm || !id || bytes < sizeof(ncclUniqueId) || nranks < 1 || rank < 0 || rank >= nranks) return CC_EINVAL;
    *comm = nullptr;
    int dev = -1, n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || hipGetDevice(&dev) != hipSuccess) return CC_ENODEV;
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(init_timeout_ms(timeout_ms));
    ncclComm_t nc = nullptr;
    const ncclResult_t r = ncclCommInitRankConfig(&nc, nranks, u, rank, &cfg);
    if (!nc) return CC_ECOMM;  // failed before a communicator existed
    const int rc = settle(nc, r, deadline);
    if (rc) {  // failed or timed out: tear down without waiting for the peers
        (void)ncclCommAbort(nc);
        return rc;
    }
    cc_comm* c = new cc_comm();
    c->nc = nc;
    c->nranks = nranks;
    c->rank = rank;
    c->device = dev;
    if ((c->stall_ms = injected_stall_ms())) {  // failpoint armed: its abort word, mapped for the stall kernel
        void* p = nullptr;
        void* d = nullptr;
        hipError_t e = hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) {
            c->stall_abort = static_cast<uint32_t*>(p);
            *c->stall_abort = 0u;
            e = hipHostGetDevicePointer(&d, p, 0);
        }
        if (e != hipSuccess) {
            (void)comm_release_abort(c);
            return map_hip(e);
        }
        c->stall_word = static_cast<uint32_t*>(d);
    }
    *comm = c;
    return CC_OK;
}

int cc_comm_init(cc_comm** comm, int nranks, int rank, const void* id, size_t bytes) {
    return cc_comm_init_timeout(comm, nranks, rank, id, bytes, 0);
}

static int comm_release(cc_comm* comm, bool abort) {
    if (!comm) return CC_OK;
    int cur = -1;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(comm->device);
    int rc = CC_OK;
    if (comm->nc) {
        if (abort) {
            rc = map_nccl(ncclCommAbort(comm->nc));
        } else {
            // finalize flushes this rank's outstanding work (non-blocking: settle
            // it), then destroy frees the resources; a finalize that fails or
            // does not settle (a peer gone) is aborted instead of destroyed
            rc = settle_call(comm->nc, ncclCommFinalize(comm->nc));
            const int rd = rc ? map_nccl(ncclCommAbort(comm->nc)) : map_nccl(ncclCommDestroy(comm->nc));
            if (!rc) rc = rd;
        }
    }
    if (comm->gather) (void)hipFree(comm->gather);
    if (comm->done) (void)hipEventDestroy(comm->done);
    if (comm->stall_abort) (void)hipHostFree(comm->stall_abort);
    if (cur >= 0) (void)hipSetDevice(cur);
    delete comm;
    return rc;
}

int cc_comm_destroy(cc_comm* comm) { return comm_release(comm, false); }
int cc_comm_abort(cc_comm* comm) { return comm_release(comm, true); }

int cc_comm_size(const cc_comm* comm) { return comm ? comm->nranks : 0; }
int cc_comm_rank(const cc_comm* comm) { return comm ? comm->rank : -1; }

int cc_comm_wait(cc_comm* comm, void* stream, uint32_t timeout_ms) {
    if (!comm) return CC_EINVAL;
    if (!comm->nc) return CC_ECOMM;  // aborted by an earlier wait
    hipStream_t s = static_cast<hipStream_t>(stream);
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (cur != comm->device && hipSetDevice(comm->device) != hipSuccess) return CC_ENODEV;
    auto back = [&](int rc) {
        if (cur >= 0 && cur != comm->device) (void)hipSetDevice(cur);
        return rc;
    };
    hipError_t e;
    {
        std::lock_guard<std::mutex> lk(comm->mu);
        if (!comm->done && (e = hipEventCreateWithFlags(&comm->done, hipEventDisableTiming)) != hipSuccess)
            return back(map_hip(e));
        if ((e = hipEventRecord(comm->done, s)) != hipSuccess) return back(map_hip(e));
    }
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(wait_timeout_ms(timeout_ms));
    for (;;) {
        e = hipEventQuery(comm->done);
        if (e == hipSuccess) return back(CC_OK);
        if (e != hipErrorNotReady) return back(map_hip(e));
        ncclResult_t ar = ncclSuccess;
        const bool failed = ncclCommGetAsyncError(comm->nc, &ar) != ncclSuccess || (ar != ncclSuccess && ar != ncclInProgress);
        const bool late = std::chrono::steady_clock::now() > deadline;
        if (failed || late) {
            // leave without the peers: the abort also releases the collective's
            // kernels still waiting for them, so the stream drains
            if (comm->stall_abort) __atomic_store_n(comm->stall_abort, 1u, __ATOMIC_RELEASE);
            (void)ncclCommAbort(comm->nc);
            comm->nc = nullptr;
            return back(failed ? CC_ECOMM : CC_ETIMEDOUT);
        }
        std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
}

int cc_digest_allreduce_dev(cc_comm* comm, uint32_t* d_digest, uint64_t n, void* stream) {
    if (!comm || (!d_digest && n)) return CC_EINVAL;
    if (!comm->nc) return CC_ECOMM;  // aborted: a peer was lost
    if (n == 0) return CC_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    {
        std::lock_guard<std::mutex> lk(comm->mu);
        if (n > comm->cap) {  // grows once per layout; the old scratch may still be in use on s
            if (comm->gather) {
                hipError_t e = hipStreamSynchronize(s);
                if (e != hipSuccess) return map_hip(e);
                (void)hipFree(comm->gather);
                comm->gather = nullptr;
                comm->cap = 0;
            }
            hipError_t e = hipMalloc(reinterpret_cast<void**>(&comm->gather), (size_t)comm->nranks * n * 4);
            if (e != hipSuccess) return map_hip(e);
            comm->cap = n;
        }
    }
    if (comm->stall_ms) {  // failpoint (armed at init)
        hipLaunchKernelGGL(stall_kernel, dim3(1), dim3(64), 0, s, (uint64_t)comm->stall_ms * 100000ull,
                           static_cast<const uint32_t*>(comm->stall_word));
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return map_hip(e);
    }
    // ring all-gather of the partials into [rank][n], then out = XOR over ranks
    int rc = settle_call(comm->nc, ncclAllGather(d_digest, comm->gather, n, ncclUint32, comm->nc, s));
    if (rc) return rc;
    return cc_digest_fold_dev(comm->gather, (uint32_t)comm->nranks, n, d_digest, stream);
}

int cc_pool_scan_dev(const cc_pool_shard* p, cc_comm* comm, void* stream) {
    if (!p) return CC_EINVAL;
    if (p->page_bytes == 0 || p->slice_bytes == 0 || p->chunk_bytes % p->page_bytes ||
        p->chunk_bytes % p->slice_bytes || p->slice_bytes % p->page_bytes)
        return CC_EINVAL;
    if (p->n_chunks && (!p->d_data || !p->d_meta || !p->d_page_crcs || !p->d_meta_crcs || !p->d_slice_crcs))
        return CC_EINVAL;
    const bool dig = p->d_digest != nullptr;
    if (dig && p->n_chunks && (!p->d_after_mult || !p->d_group)) return CC_EINVAL;
    if (comm && !dig) return CC_EINVAL;  // nothing to exchange
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint64_t pages = p->n_chunks * (uint64_t)(p->chunk_bytes / p->page_bytes);
    int rc;
    hipError_t e;
    if (p->n_chunks == 0) {  // an empty shard: zero partials (full digests after the exchange)
        if (dig && (e = hipMemsetAsync(p->d_digest, 0, p->n_groups * 4, s)) != hipSuccess) return map_hip(e);
    } else {
        // readMetaPage ops (one "page" of meta_bytes per chunk; this launch also
        // zeroes the digest partials and the next launch's tail counter), then the
        // hot kernel over every data page of the shard, bracketed by the caller's events
        if ((rc = cc::pool_page_launches(p->d_data, pages, p->page_bytes, p->d_page_crcs, p->d_meta, p->n_chunks,
                                         p->meta_bytes, p->d_meta_crcs, dig ? p->d_digest : nullptr,
                                         dig ? p->n_groups : 0, s, p->ev_pages_begin, p->ev_pages_end)))
            return rc;
        // slices + file CRCs + digest partials in one launch
        if ((rc = cc_scan_epilogue_dev(p->d_page_crcs, p->d_meta_crcs, p->n_chunks, p->chunk_bytes / p->page_bytes,
                                       p->page_bytes, p->slice_bytes / p->page_bytes, p->d_slice_crcs,
                                       p->d_file_crcs, dig ? p->d_after_mult : nullptr, dig ? p->d_group : nullptr,
                                       dig ? p->d_digest : nullptr, stream)))
            return rc;
    }
    if (!comm) return CC_OK;
    if (p->ev_exchange_begin && (e = hipEventRecord(static_cast<hipEvent_t>(p->ev_exchange_begin), s)) != hipSuccess)
        return map_hip(e);
    if ((rc = cc_digest_allreduce_dev(comm, p->d_digest, p->n_groups, stream))) return rc;
    if (p->ev_exchange_end && (e = hipEventRecord(static_cast<hipEvent_t>(p->ev_exchange_end), s)) != hipSuccess)
        return map_hip(e);
    return CC_OK;
}

}  // extern "C"
