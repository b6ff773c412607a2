// tests/native/rccl_stub.cpp -- TEST INFRASTRUCTURE: a stand-in for the seven
// RCCL entry points libcurvecrc's digest exchange calls (curve_amd/csrc/pool.hip),
// for N ranks that share ONE GPU, where real RCCL refuses to build a
// communicator ("Duplicate GPU detected").  It lets the multi-rank native path
// -- cc_comm_init_timeout with nranks > 1, the all-gather of every rank's
// digest partials into [rank][n], the XOR fold over the ranks, cc_comm_wait,
// finalize/destroy -- run end to end in one-GPU tests (a build of libcurvecrc
// linked against this file instead of librccl: make -C curve_amd/csrc stubrccl;
// tests/test_distributed_gpu.py).  Nothing in the product loads it.
//
// Transport: one POSIX shared-memory segment per communicator, named by the
// unique id.  ncclAllGather is synchronous: it waits for the stream, copies
// its send buffer into its rank's slot, meets the other ranks at a barrier,
// copies every slot into the receive buffer and meets them again, so the
// stream order of the caller is kept (the collective is complete when it
// returns).  Every wait is bounded (wait_s()); a rank that never arrives makes
// the others fail with ncclSystemError instead of hanging.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>

namespace {
constexpr size_t kHeader = 4096;
constexpr size_t kSlot = 1u << 20;  // bytes a rank may contribute to one all-gather
constexpr int kMaxRanks = 16;
int wait_s() {  // $CC_RCCL_STUB_WAIT_S (tests of a missing peer), else 120
    const char* e = getenv("CC_RCCL_STUB_WAIT_S");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 120;
}

struct Shared {
    std::atomic<uint32_t> count, gen, joined;
};
}  // namespace

struct ncclComm {
    int nranks = 0, rank = 0;
    unsigned char* map = nullptr;
    size_t bytes = 0;
    char name[64] = {};
};

namespace {
Shared* hdr(ncclComm* c) { return reinterpret_cast<Shared*>(c->map); }

// sense-reversing barrier over the segment; false after wait_s()
bool barrier(ncclComm* c) {
    Shared* h = hdr(c);
    const uint32_t g = h->gen.load(std::memory_order_acquire);
    if (h->count.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)c->nranks) {
        h->count.store(0, std::memory_order_relaxed);
        h->gen.store(g + 1, std::memory_order_release);
        return true;
    }
    const auto end = std::chrono::steady_clock::now() + std::chrono::seconds(wait_s());
    while (h->gen.load(std::memory_order_acquire) == g) {
        if (std::chrono::steady_clock::now() > end) return false;
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    return true;
}

void release(ncclComm* c, bool unlink_it) {
    if (c->map) munmap(c->map, c->bytes);
    if (unlink_it) shm_unlink(c->name);
    delete c;
}
}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    memset(id, 0, sizeof(*id));
    std::random_device rd;
    snprintf(id->internal, sizeof(id->internal), "/ccrcclstub-%d-%08x%08x", (int)getpid(), rd(), rd());
    return ncclSuccess;
}

ncclResult_t ncclCommInitRankConfig(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank, ncclConfig_t*) {
    if (!comm || nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    ncclComm* c = new ncclComm();
    c->nranks = nranks;
    c->rank = rank;
    snprintf(c->name, sizeof(c->name), "%s", id.internal);
    c->bytes = kHeader + (size_t)kMaxRanks * kSlot;
    const int fd = shm_open(c->name, O_CREAT | O_RDWR, 0600);
    if (fd < 0 || ftruncate(fd, (off_t)c->bytes) != 0) {
        if (fd >= 0) close(fd);
        release(c, false);
        return ncclSystemError;
    }
    void* p = mmap(nullptr, c->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
        release(c, false);
        return ncclSystemError;
    }
    c->map = static_cast<unsigned char*>(p);
    hdr(c)->joined.fetch_add(1);
    if (!barrier(c)) {  // a peer never joined
        release(c, true);
        return ncclSystemError;
    }
    *comm = c;
    return ncclSuccess;  // a non-blocking caller may see ncclSuccess at once
}

ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* err) {
    if (!comm || !err) return ncclInvalidArgument;
    *err = ncclSuccess;
    return ncclSuccess;
}

ncclResult_t ncclAllGather(const void* send, void* recv, size_t count, ncclDataType_t type, ncclComm_t c,
                           hipStream_t stream) {
    if (!c || (type != ncclUint32 && type != ncclInt32 && type != ncclFloat32)) return ncclInvalidArgument;
    const size_t bytes = count * 4;
    if (bytes > kSlot) return ncclInvalidArgument;
    if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
    unsigned char* slots = c->map + kHeader;
    if (bytes && hipMemcpy(slots + (size_t)c->rank * kSlot, send, bytes, hipMemcpyDeviceToHost) != hipSuccess)
        return ncclUnhandledCudaError;
    if (!barrier(c)) return ncclSystemError;
    for (int r = 0; r < c->nranks && bytes; r++)
        if (hipMemcpy(static_cast<unsigned char*>(recv) + (size_t)r * bytes, slots + (size_t)r * kSlot, bytes,
                      hipMemcpyHostToDevice) != hipSuccess)
            return ncclUnhandledCudaError;
    return barrier(c) ? ncclSuccess : ncclSystemError;  // every slot read before the next gather writes
}

ncclResult_t ncclCommFinalize(ncclComm_t c) { return c ? ncclSuccess : ncclInvalidArgument; }

ncclResult_t ncclCommDestroy(ncclComm_t c) {
    if (!c) return ncclInvalidArgument;
    const bool last = hdr(c)->joined.fetch_sub(1) == 1;  // the last rank out removes the segment
    release(c, last);
    return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t c) { return ncclCommDestroy(c); }

}  // extern "C"
