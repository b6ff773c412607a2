// curve_amd/csrc/engine.hip -- C ABI of the device path: per-device contexts
// (LDS image, CU count, pinned staging), argument checking, error mapping.
//
// Threading: the reference calls its CRC primitive from raft apply threads and
// brpc bthread workers.  A device context is created once under a
// mutex and then reached through a lock-free shared_ptr load, so *_dev calls
// take no lock (they only enqueue).  Every call holds its own reference to the
// context: cc_engine_fini unpublishes the contexts and the last call still
// using one frees it.  A blocking cc_page_crc_host call of at most 16 MiB runs
// on a lane of its own (device buffer, stream, completion signal), so
// concurrent callers overlap; the other blocking *_host calls, and larger page
// calls, serialise on a per-device submission lock over two shared staging slots.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <stdio.h>
#include <sys/prctl.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/curve_crc.h"
#include "gf2.h"
#include "kernels.h"
#include "reader_pool.h"

namespace cc {

// ---------------------------------------------------------------------------
// LDS image (163840 B):
//   [0, 128K)  G-tables, G = x^(32*64) mod P (= 256 zero bytes):
//              region r in {0,1} (64 KiB), row b (256 B), half h (128 B), slot s (4 B)
//              holds G(b << 8*(2r+h)); s = lane mod 32 -> bank = lane mod 32.
//   [128K,160K) final maps F^(64-l), F = x^32 mod P, per lane l, by nibble:
//              kFinBase + n*4096 + v*256 + l*4 holds F^(64-l)(v << 4n).
// ---------------------------------------------------------------------------
void build_lds_image(uint32_t* img) {
    const uint32_t g = xpow(32ull * 64);
    for (uint32_t r = 0; r < 2; r++)
        for (uint32_t b = 0; b < 256; b++)
            for (uint32_t h = 0; h < 2; h++) {
                const uint32_t k = 2 * r + h;
                const uint32_t v = mulmod(g, b << (8 * k));
                for (uint32_t s = 0; s < 32; s++) img[(r * 65536 + b * 256 + h * 128 + s * 4) / 4] = v;
            }
    for (uint32_t l = 0; l < 64; l++) {
        const uint32_t f = xpow(32ull * (64 - l));
        for (uint32_t n = 0; n < 8; n++)
            for (uint32_t v = 0; v < 16; v++)
                img[(kFinBase + n * 4096 + v * 256 + l * 4) / 4] = mulmod(f, v << (4 * n));
    }
}

namespace {

// Completion of a staging slot's batch, delivered by a host function enqueued
// behind the batch: the waiting caller sleeps on a condition variable.
struct SlotSignal {
    std::mutex m;
    std::condition_variable cv;
    bool fired = true;
};

struct Staging {
    bool ready = false;
    size_t bytes = 0;            // per slot
    void* host[2] = {nullptr, nullptr};
    void* dev[2] = {nullptr, nullptr};
    uint32_t* dcrc[2] = {nullptr, nullptr};
    uint32_t* hcrc[2] = {nullptr, nullptr};
    hipStream_t stream[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
    SlotSignal sig[2];
    // cc_scan_files' host->device copies, both slots', in FIFO order on ONE
    // stream: copies of the two slots on their own streams run side by side at
    // half the link each, so every batch completes late and the reads of the
    // batch after next (gated on it) start late (a host trace: pairs of batches
    // completing together, 37.8 GiB/s against 53 GiB/s of H2D)
    hipStream_t copy = nullptr;
    hipEvent_t copied[2] = {nullptr, nullptr};
    // per-call device inputs of the streamed digest (after bytes, multipliers,
    // copyset index per chunk, digest accumulator): grown on demand
    void* aux = nullptr;
    size_t aux_bytes = 0;
    hipEvent_t aux_ready = nullptr;
};

// Per-caller lanes of the blocking page call (cc_page_crc_host) at the scan
// op's call shape: one 4 MiB slice or the 4 KiB metapage per raft-applied op
// (ScanChunkRequest::OnApply, op_request.cpp:776-794), from up to
// wconcurrentapply.size = 10 apply threads at once (conf/chunkserver.conf:183,
// op_request.cpp:179-187).  A call of at most kLaneBytes takes a lane of its
// own -- device buffer, CRC buffers, stream, completion signal -- so concurrent
// callers overlap their H2D, kernel and D2H instead of queueing one whole call
// after another on the two shared staging slots.  Lanes are made on first
// demand (up to kMaxLanes) and reused; a caller finding none idle waits for one.
constexpr uint64_t kLaneBytes = 16ull << 20;
constexpr size_t kMaxLanes = 16;
constexpr uint64_t kLanePiece = 1ull << 20;  // pageable input: memcpy a piece, its DMA runs behind the next
struct Lane {
    void* dev = nullptr;        // kLaneBytes
    uint32_t* hcrc = nullptr;   // pinned: the page kernel stores the CRCs here directly (kLaneBytes / 256 of them)
    void* host = nullptr;       // pinned staging for pageable input, made on the first such call
    uint32_t* hflag = nullptr;  // pinned completion word, written by the lane's stream after the kernel
    uint32_t seq = 0;           // the last value asked of hflag
    hipStream_t stream = nullptr;
};
struct LanePool {
    std::mutex m;
    std::condition_variable cv;
    std::vector<Lane*> idle;
    std::vector<std::unique_ptr<Lane>> all;
    size_t making = 0;                       // lanes being created outside the lock
    std::atomic<uint64_t> inflight{0};       // bytes the lanes have enqueued and not yet seen complete
};

// Product tables of the fused epilogue, one per (page_bytes, q): a small
// lock-free cache (lookups from concurrent *_dev calls take no lock; the rare
// insert takes the context's table mutex).
constexpr int kEpiSlots = 16;

// Per-stream state (the page kernel's tail counters, the write log's table,
// the range scratch) is keyed by stream.  The null stream and hipStreamLegacy
// name ONE real stream of the device (the legacy default stream: this library
// is built without per-thread default streams), so their key is the handle,
// like a created stream's; the per-state mutex orders enqueues on it.
// hipStreamPerThread names a different real stream in each thread: its key is
// the handle AND the calling thread, and a thread's entries are dropped when
// the thread exits (ThreadEntries below), so a later thread that reuses the
// id (glibc reuses pthread_t) never inherits scratch whose kernels may still
// run on the old thread's stream, and short-lived threads do not use up the
// kMaxTailBlocks entries.
struct StreamKey {
    hipStream_t s = nullptr;
    std::thread::id tid;
    bool operator==(const StreamKey& o) const { return s == o.s && tid == o.tid; }
};
inline StreamKey stream_key(hipStream_t s) {
    StreamKey k;
    k.s = s;
    if (s == hipStreamPerThread) k.tid = std::this_thread::get_id();
    return k;
}

struct DevCtx : std::enable_shared_from_this<DevCtx> {
    int device = -1;
    bool ready = false;
    int cus = 256;
    void* image = nullptr;
    std::mutex submit;  // serialises *_host calls on this device
    Staging st;
    std::mutex tab_mu;  // epilogue-table inserts
    std::atomic<uint64_t> epi_key[kEpiSlots];  // key + 1 (0 = empty); published after epi_ptr
    std::atomic<void*> epi_ptr[kEpiSlots];
    // the page kernel's tail counters, one block of two slot sets per stream:
    // zeroed on the stream when created; a launch pulls from slot set `parity`
    // and zeroes the other for the stream's next launch, so a call needs no
    // allocation or memset.  tail_mu is held over the flip and the enqueue.
    struct TailBlock {
        StreamKey s;
        unsigned long long* p;
        uint32_t parity;  // the slot set the stream's next launch pulls from
        bool dirty;       // a launch may not have zeroed the next slot set: clear first
    };
    std::mutex tail_mu;
    std::vector<TailBlock> tails;
    // the write log's page tables, one per stream (apply_log); log_mu is held
    // over a call's whole enqueue (insert + pages) so calls sharing a stream
    // cannot interleave on its table
    struct LogTable {
        StreamKey s;
        unsigned char* p;
        uint64_t entries;
        bool dirty;
    };
    std::mutex log_mu;
    std::vector<LogTable> log_tabs;
    // the range kernel's scratch, one per stream (range_work): tile words, the
    // tail block and the split-range accumulators; range_mu is held over a
    // call's enqueue so the epoch order is the stream order
    struct RangeWork {
        StreamKey s;
        unsigned char* p;
        uint64_t cap;    // accumulator pairs (ranges a call may have)
        uint32_t epoch;  // the last call's
        bool dirty;
    };
    std::mutex range_mu;
    std::vector<RangeWork> range_works;
    ReaderPool readers;  // cc_scan_files' io threads
    LanePool lanes;      // cc_page_crc_host's per-caller lanes
    DevCtx() {
        for (int i = 0; i < kEpiSlots; i++) {
            epi_key[i].store(0);
            epi_ptr[i].store(nullptr);
        }
    }
    ~DevCtx();
};

using CtxRef = std::shared_ptr<DevCtx>;

// A thread's hipStreamPerThread entries, dropped when the thread exits: taken
// out of the context's lists under their mutexes (no call can reach them after
// that), then handed to hipFreeAsync on the exiting thread's own per-thread
// stream -- the only stream that used them -- so the memory goes back once
// that stream's work is done.  Nothing here waits: a device-synchronising call
// (hipFree, a stream sync) in a thread-exit destructor would make the exit,
// and any join() on it, wait for every stream of the device, including a
// collective stuck on a lost peer.  No lock is held while enqueueing.
void drop_thread_entries(DevCtx* c, std::thread::id tid) {
    StreamKey key;
    key.s = hipStreamPerThread;
    key.tid = tid;
    std::vector<void*> dead;
    auto take = [&](auto& vec, std::mutex& mu) {
        std::lock_guard<std::mutex> lk(mu);
        for (size_t i = 0; i < vec.size();) {
            if (vec[i].s == key) {
                if (vec[i].p) dead.push_back(vec[i].p);
                vec.erase(vec.begin() + i);
            } else {
                i++;
            }
        }
    };
    take(c->tails, c->tail_mu);
    take(c->log_tabs, c->log_mu);
    take(c->range_works, c->range_mu);
    if (dead.empty()) return;
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (hipSetDevice(c->device) == hipSuccess)
        for (void* p : dead) (void)hipFreeAsync(p, hipStreamPerThread);  // stream-ordered: after the thread's work
    if (cur >= 0) (void)hipSetDevice(cur);
}

struct ThreadEntries {
    std::vector<std::weak_ptr<DevCtx>> ctxs;  // contexts holding entries of this thread
    ~ThreadEntries() {
        const std::thread::id tid = std::this_thread::get_id();
        for (auto& w : ctxs)
            if (std::shared_ptr<DevCtx> c = w.lock()) drop_thread_entries(c.get(), tid);
    }
};
thread_local ThreadEntries t_entries;

// Called when an entry keyed by hipStreamPerThread is created for the calling thread.
void note_thread_entry(DevCtx* c) {
    for (auto& w : t_entries.ctxs)
        if (w.lock().get() == c) return;
    t_entries.ctxs.push_back(c->weak_from_this());
}

constexpr int kMaxDevices = 64;
std::mutex g_mu;                 // context creation / teardown only
CtxRef g_ctx[kMaxDevices];       // read with std::atomic_load (lock-free fast path)
cc_opts g_opts = {4096u, 4u << 20, 256ull << 20};

int map_err(hipError_t e) {
    if (e == hipSuccess) return CC_OK;
    if (e == hipErrorOutOfMemory) return CC_ENOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice || e == hipErrorNoBinaryForGpu ||
        e == hipErrorInsufficientDriver)
        return CC_ENODEV;
    return CC_EHIP;
}

void staging_free(Staging& st) {
    for (int i = 0; i < 2; i++) {
        // teardown: nothing to do about a failure here but go on freeing the rest
        if (st.stream[i]) (void)hipStreamSynchronize(st.stream[i]);
        if (st.host[i]) (void)hipHostFree(st.host[i]);
        if (st.dev[i]) (void)hipFree(st.dev[i]);
        if (st.dcrc[i]) (void)hipFree(st.dcrc[i]);
        if (st.hcrc[i]) (void)hipHostFree(st.hcrc[i]);
        if (st.stream[i]) (void)hipStreamDestroy(st.stream[i]);
        if (st.done[i]) (void)hipEventDestroy(st.done[i]);
        if (st.copied[i]) (void)hipEventDestroy(st.copied[i]);
        st.copied[i] = nullptr;
        st.host[i] = st.dev[i] = nullptr;
        st.dcrc[i] = st.hcrc[i] = nullptr;
        st.stream[i] = nullptr;
        st.done[i] = nullptr;
        st.sig[i].fired = true;
    }
    if (st.copy) {
        (void)hipStreamSynchronize(st.copy);
        (void)hipStreamDestroy(st.copy);
        st.copy = nullptr;
    }
    if (st.aux) (void)hipFree(st.aux);
    if (st.aux_ready) (void)hipEventDestroy(st.aux_ready);
    st.aux = nullptr;
    st.aux_ready = nullptr;
    st.aux_bytes = 0;
    st.ready = false;
    st.bytes = 0;
}

void lane_free(Lane* l) {
    if (l->stream) (void)hipStreamSynchronize(l->stream);
    if (l->dev) (void)hipFree(l->dev);
    if (l->hcrc) (void)hipHostFree(l->hcrc);
    if (l->host) (void)hipHostFree(l->host);
    if (l->hflag) (void)hipHostFree(l->hflag);
    if (l->stream) (void)hipStreamDestroy(l->stream);
    l->dev = l->host = nullptr;
    l->hcrc = l->hflag = nullptr;
    l->stream = nullptr;
}

// Runs when the last reference drops (cc_engine_fini, or the last call still
// holding the context after it): nothing can be enqueued on it any more, so
// finish whatever was enqueued and free on the context's own device.
DevCtx::~DevCtx() {
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (device >= 0 && hipSetDevice(device) == hipSuccess) {
        (void)hipDeviceSynchronize();  // kernels enqueued by *_dev calls may still read the image / tables
        staging_free(st);
        if (image) (void)hipFree(image);
        for (int i = 0; i < kEpiSlots; i++)
            if (void* p = epi_ptr[i].load()) (void)hipFree(p);
        for (auto& t : tails) (void)hipFreeAsync(t.p, nullptr);
        for (auto& t : log_tabs) (void)hipFreeAsync(t.p, nullptr);
        for (auto& t : range_works) (void)hipFreeAsync(t.p, nullptr);
        for (auto& l : lanes.all) lane_free(l.get());
        (void)hipDeviceSynchronize();
    }
    if (cur >= 0) (void)hipSetDevice(cur);
}

// Context of the calling thread's current device, created on first use.
int get_ctx(CtxRef* out) {
    int dev = -1, n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return CC_ENODEV;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return CC_ENODEV;
    CtxRef c = std::atomic_load(&g_ctx[dev]);
    if (c) {
        *out = std::move(c);
        return CC_OK;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    c = std::atomic_load(&g_ctx[dev]);
    if (c) {
        *out = std::move(c);
        return CC_OK;
    }
    c = std::make_shared<DevCtx>();
    c->device = dev;
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties(&prop, dev);
    if (e != hipSuccess) return map_err(e);
    c->cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    // test hook: $CC_TEST_CUS sizes every grid as if the device had that many
    // CUs (e.g. a 304-CU part's grids on this 256-CU one); never needed in use
    if (const char* v = getenv("CC_TEST_CUS"))
        if (atoi(v) > 0 && atoi(v) <= 4096) c->cus = atoi(v);
    std::vector<uint32_t> img(kLdsBytes / 4);
    build_lds_image(img.data());
    // device image: the LDS image, then for t < kXinvEntries the 32 products
    // x^(-8t) * x^i, i = 0..31 (range kernel: a lane-parallel multiply by x^(-8t))
    img.resize(kLdsBytes / 4 + kXinvEntries * 32);
    uint32_t r = xinv_bytes(0);
    for (uint32_t t = 0; t < kXinvEntries; t++, r = div_x8(r)) {  // r = x^(-8t)
        uint32_t b = r;
        for (uint32_t i = 0; i < 32; i++, b = (b >> 1) ^ (kPoly & (0u - (b & 1u))))  // b *= x
            img[kLdsBytes / 4 + t * 32 + i] = b;
    }
    if ((e = hipMalloc(&c->image, img.size() * 4)) != hipSuccess) return map_err(e);
    if ((e = hipMemcpy(c->image, img.data(), img.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) return map_err(e);
    if ((e = upload_x2k(x2k().t)) != hipSuccess) return map_err(e);
    c->ready = true;
    std::atomic_store(&g_ctx[dev], c);
    *out = std::move(c);
    return CC_OK;
}

inline uint64_t align256(uint64_t x) { return (x + 255) & ~255ull; }

inline bool page_size_ok(uint32_t page_bytes) {
    return page_bytes >= 256 && page_bytes <= (1u << 20) && page_bytes % 256 == 0;
}

// V(page) = raw(page) ^ K(P),  K(P) = ~shift(~0, P)  == crc32c_zeros(P).
inline uint32_t kconst_for(uint32_t page_bytes) { return ~shift_bytes(0xFFFFFFFFu, page_bytes); }

// Grid + tile size.  Exactly one 160 KiB-LDS workgroup fits per CU, so the
// grid is one block per CU (or fewer for tiny batches).  Each wave owns tiles
// of 2^ts consecutive pages (one coalesced CRC store per tile); the tile is the
// largest power of two <= 64 that still gives every wave of the grid a tile.
void geometry_for(const DevCtx* c, uint64_t n_pages, PageLaunch* a) {
    const uint64_t waves = (uint64_t)c->cus * kWavesPerBlock;
    uint32_t ts = 6;
    while (ts > 0 && (n_pages >> ts) < waves) ts--;
    const uint64_t tiles = (n_pages + (1ull << ts) - 1) >> ts;
    const uint64_t need = (tiles + kWavesPerBlock - 1) / kWavesPerBlock;
    a->blocks = (int)(need < (uint64_t)c->cus ? (need ? need : 1) : (uint64_t)c->cus);
    a->tile_shift = ts;
}

// 1/16 of a large launch's tiles form the dynamic tail (A/B 2.464 ms vs
// 2.474-2.478 at 1/8, 2.474 at 1/12, 2.51 at 1/24 and 1/32)
constexpr uint64_t kPageDynDiv = 16;
// Tile schedule of a page launch: geometry, and (true) a dynamic tail of the
// last 1/kPageDynDiv of the tiles when the batch is large and the page size
// has a fixed-M instantiation.
bool plan_tail(const DevCtx* c, PageLaunch& a) {
    geometry_for(c, a.n_pages, &a);
    const uint32_t m = a.words_per_lane;
    const uint64_t tiles = (a.n_pages + (1ull << a.tile_shift) - 1) >> a.tile_shift;
    const uint64_t waves = (uint64_t)a.blocks * kWavesPerBlock;
    if (m > 32 || (m & (m - 1)) || tiles < waves * 8) return false;
    a.static_tiles = tiles - tiles / kPageDynDiv;
    return true;
}

constexpr size_t kMaxTailBlocks = 256;  // streams with a block of their own

// The stream's tail-counter block, created (and zeroed on the stream) on first
// use; null when kMaxTailBlocks streams already hold one.  Caller holds
// c->tail_mu.  Keyed by the stream (stream_key: a pseudo-handle is per calling
// thread): a destroyed stream's handle is only reused for a new stream after
// hipStreamDestroy, which the caller orders after that stream's work as for any
// of its buffers.
DevCtx::TailBlock* tail_block(DevCtx* c, hipStream_t s) {
    const StreamKey key = stream_key(s);
    for (auto& t : c->tails)
        if (t.s == key) {
            if (t.dirty) {
                if (hipMemsetAsync(t.p, 0, kTailBlockBytes, s) != hipSuccess) return nullptr;
                t.dirty = false;
            }
            return &t;
        }
    if (c->tails.size() >= kMaxTailBlocks) return nullptr;
    void* p = nullptr;  // stream-ordered, like every per-stream entry (freed by hipFreeAsync)
    if (hipMallocAsync(&p, kTailBlockBytes, s) != hipSuccess) return nullptr;
    if (hipMemsetAsync(p, 0, kTailBlockBytes, s) != hipSuccess) {
        (void)hipFreeAsync(p, s);
        return nullptr;
    }
    c->tails.push_back({key, static_cast<unsigned long long*>(p), 0u, false});
    if (s == hipStreamPerThread) note_thread_entry(c);
    return &c->tails.back();
}

// Page kernel launch (kernels.hip, page_crc_kernel) with its dynamic tail when
// plan_tail() gives one: the tail's counters are one slot set of the stream's
// block (the launch zeroes the other for the next), or (no block free) a
// counter allocated + zeroed for this launch.
hipError_t launch_page_tail(DevCtx* c, PageLaunch& a, bool verify, hipStream_t s, bool load_probe = false) {
    auto launch = [&]() {
        return load_probe ? launch_page_load_probe(a, s) : verify ? launch_page_verify(a, s) : launch_page_crc(a, s);
    };
    if (!plan_tail(c, a)) return launch();
    {
        std::lock_guard<std::mutex> lk(c->tail_mu);
        if (DevCtx::TailBlock* t = tail_block(c, s)) {
            a.dyn_ctr = t->p + t->parity * kDynCtrWords64;
            a.dyn_next = t->p + (t->parity ^ 1u) * kDynCtrWords64;
            const hipError_t e = launch();
            if (e == hipSuccess)
                t->parity ^= 1u;
            else
                t->dirty = true;  // may or may not have run: clear both slot sets before the next use
            return e;
        }
    }
    unsigned long long* ctr = nullptr;
    hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&ctr), kDynCtrBytes, s);
    if (e != hipSuccess) return e;
    if ((e = hipMemsetAsync(ctr, 0, kDynCtrBytes, s)) == hipSuccess) {
        a.dyn_ctr = ctr;
        e = launch();
    }
    const hipError_t f = hipFreeAsync(ctr, s);
    return e != hipSuccess ? e : f;
}

int staging_init(DevCtx* c) {
    Staging& st = c->st;
    if (st.ready) return CC_OK;
    size_t per = (size_t)(g_opts.staging_bytes / 2);
    per -= per % (1u << 20);
    if (per < (1u << 20)) per = 1u << 20;
    st.bytes = per;
    for (int i = 0; i < 2; i++) {
        hipError_t e;
        if ((e = hipHostMalloc(&st.host[i], per, hipHostMallocDefault)) != hipSuccess) return map_err(e);
        if ((e = hipMalloc(&st.dev[i], per)) != hipSuccess) return map_err(e);
        if ((e = hipMalloc(&st.dcrc[i], per / 256 * 4)) != hipSuccess) return map_err(e);
        if ((e = hipHostMalloc(&st.hcrc[i], per / 256 * 4, hipHostMallocDefault)) != hipSuccess) return map_err(e);
        if ((e = hipStreamCreateWithFlags(&st.stream[i], hipStreamNonBlocking)) != hipSuccess) return map_err(e);
        if ((e = hipEventCreateWithFlags(&st.done[i], hipEventDisableTiming)) != hipSuccess) return map_err(e);
        if ((e = hipEventCreateWithFlags(&st.copied[i], hipEventDisableTiming)) != hipSuccess) return map_err(e);
    }
    if (hipError_t e = hipStreamCreateWithFlags(&st.copy, hipStreamNonBlocking); e != hipSuccess) return map_err(e);
    hipError_t e = hipEventCreateWithFlags(&st.aux_ready, hipEventDisableTiming);
    if (e != hipSuccess) return map_err(e);
    st.ready = true;
    return CC_OK;
}

// Blocking *_host calls come from bthread workers / apply threads (SURVEY
// §8b) and must not burn the caller's CPU.  hipEventSynchronize spins on this
// ROCm unless the whole device was put in BlockingSync mode before its context
// existed (measured: scripts/spin_probe.py), and a sleep-poll loop wakes late
// and stalls the next batch's submission (-2 % e2e).  So each batch ends with
// a host function that signals a condition variable: the caller parks in the
// kernel and is woken as soon as the batch's last copy completes.
void fire_slot(void* p) {
    SlotSignal* sg = static_cast<SlotSignal*>(p);
    {
        std::lock_guard<std::mutex> lk(sg->m);
        sg->fired = true;
    }
    sg->cv.notify_all();
}

hipError_t arm_signal(SlotSignal& sg, hipEvent_t done, hipStream_t s) {
    hipError_t e = hipEventRecord(done, s);
    if (e != hipSuccess) return e;
    {
        std::lock_guard<std::mutex> lk(sg.m);
        sg.fired = false;
    }
    e = hipLaunchHostFunc(s, fire_slot, &sg);
    if (e != hipSuccess) {
        std::lock_guard<std::mutex> lk(sg.m);
        sg.fired = true;  // nothing will fire: never leave a waiter hanging
    }
    return e;
}

hipError_t park_signal(SlotSignal& sg, hipEvent_t done) {
    {
        std::unique_lock<std::mutex> lk(sg.m);
        sg.cv.wait(lk, [&] { return sg.fired; });
    }
    return hipEventSynchronize(done);  // already complete: returns its status
}

hipError_t arm_slot(Staging& st, int slot, hipStream_t s) { return arm_signal(st.sig[slot], st.done[slot], s); }
hipError_t park_slot(Staging& st, int slot) { return park_signal(st.sig[slot], st.done[slot]); }

int lane_make(Lane* l) {
    hipError_t e;
    if ((e = hipMalloc(&l->dev, kLaneBytes)) != hipSuccess ||
        (e = hipHostMalloc(reinterpret_cast<void**>(&l->hcrc), kLaneBytes / 256 * 4, hipHostMallocDefault)) !=
            hipSuccess ||
        (e = hipHostMalloc(reinterpret_cast<void**>(&l->hflag), 256, hipHostMallocDefault)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&l->stream, hipStreamNonBlocking)) != hipSuccess)
        return map_err(e);
    __atomic_store_n(l->hflag, 0u, __ATOMIC_RELEASE);
    return CC_OK;
}

// Wait for the lane's completion word to reach `want`, sleeping, never
// spinning and never in a HIP wait: hipStreamSynchronize / a blocking-sync
// event spin the caller for the whole call, and a host function keeps a HIP
// runtime thread busy while it is pending (process CPU ~= call time either
// way: profiles/lane_wait_ab_r06.jsonl).  The caller sleeps ~80 % of the
// expected time -- its bytes plus those the other lanes had enqueued, at
// ~50 GB/s of H2D -- then polls with a growing sleep (2 .. 32 us) under a 1 us
// timer slack (the default 50 us slack would add ~50 us to a 4 KiB call), the
// thread's own slack restored on the way out.  A stream error ends the wait.
hipError_t lane_wait(Lane* l, uint32_t want, uint64_t ahead_bytes) {
    const int old = prctl(PR_GET_TIMERSLACK, 0, 0, 0, 0);
    (void)prctl(PR_SET_TIMERSLACK, 1000ul, 0, 0, 0);
    const uint64_t est_ns = 15000 + ahead_bytes / 50;  // 15 us + bytes at 50 GB/s
    timespec ts = {(time_t)(est_ns * 8 / 10 / 1000000000ull), (long)(est_ns * 8 / 10 % 1000000000ull)};
    nanosleep(&ts, nullptr);
    hipError_t r = hipSuccess;
    long nap = 2000;
    for (uint32_t k = 0; __atomic_load_n(l->hflag, __ATOMIC_ACQUIRE) != want; k++) {
        if ((k & 15u) == 15u) {
            const hipError_t q = hipStreamQuery(l->stream);
            if (q != hipSuccess && q != hipErrorNotReady) {
                r = q;
                break;
            }
        }
        timespec t2 = {0, nap};
        nanosleep(&t2, nullptr);
        if (nap < 32000) nap *= 2;
    }
    if (old > 0) (void)prctl(PR_SET_TIMERSLACK, (unsigned long)old, 0, 0, 0);
    return r;
}

// An idle lane of the device, made if fewer than kMaxLanes exist, else the
// next one released (the caller sleeps).  nullptr + *rc on an allocation failure.
Lane* lane_get(DevCtx* c, int* rc) {
    LanePool& lp = c->lanes;
    std::unique_lock<std::mutex> lk(lp.m);
    while (lp.idle.empty() && lp.all.size() + lp.making >= kMaxLanes) lp.cv.wait(lk);
    if (!lp.idle.empty()) {
        Lane* l = lp.idle.back();
        lp.idle.pop_back();
        return l;
    }
    lp.making++;
    lk.unlock();
    auto l = std::make_unique<Lane>();
    const int r = lane_make(l.get());
    if (r) lane_free(l.get());
    lk.lock();
    lp.making--;
    if (r) {
        lk.unlock();
        lp.cv.notify_one();  // a waiter may make it instead
        *rc = r;
        return nullptr;
    }
    lp.all.push_back(std::move(l));
    return lp.all.back().get();
}

void lane_put(DevCtx* c, Lane* l) {
    {
        std::lock_guard<std::mutex> lk(c->lanes.m);
        c->lanes.idle.push_back(l);
    }
    c->lanes.cv.notify_one();
}

bool is_pinned(const void* p) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeHost;
}

// The two staging slots' in-flight batches of one blocking call.  Every exit
// goes through drain() or fail(): a call never returns while a batch it
// enqueued may still read or write the shared pinned staging (the next call,
// possibly from another thread, reuses the same slots).
struct SlotRing {
    Staging& st;
    uint64_t first[2] = {0, 0};
    uint64_t n[2] = {0, 0};
    explicit SlotRing(Staging& s) : st(s) {}
    // wait for slot s's batch; `take` copies its results out
    template <class F>
    int drain(int s, F&& take) {
        if (!n[s]) return CC_OK;
        const hipError_t e = park_slot(st, s);
        const uint64_t f = first[s], k = n[s];
        n[s] = 0;
        if (e != hipSuccess) return fail(map_err(e));
        take(f, k);
        return CC_OK;
    }
    // error exit: park whatever is still in flight (its status no longer
    // matters) and hand back rc
    int fail(int rc) {
        for (int s = 0; s < 2; s++)
            if (n[s]) {
                (void)park_slot(st, s);
                n[s] = 0;
            }
        // a slot armed by arm_slot may have failed before its host function was
        // enqueued: make sure the streams are idle either way
        for (int s = 0; s < 2; s++)
            if (st.stream[s]) (void)hipStreamSynchronize(st.stream[s]);
        if (st.copy) (void)hipStreamSynchronize(st.copy);
        return rc;
    }
};

}  // namespace
}  // namespace cc

using namespace cc;

extern "C" {

const char* cc_version(void) { return "libcurvecrc 0.2 (gfx950)"; }

const char* cc_strerror(int code) {
    switch (code) {
        case CC_OK: return "ok";
        case CC_EINVAL: return "invalid argument";
        case CC_ENODEV: return "no usable HIP device";
        case CC_ENOMEM: return "out of memory";
        case CC_EHIP: return "HIP runtime error";
        case CC_ECORRUPT: return "checksum mismatch";
        case CC_ECOMM: return "RCCL communication error";
        case CC_EIO: return "I/O error";
        case CC_ESTALE: return "per-page CRC table is stale";
        case CC_ETIMEDOUT: return "timed out";
        case CC_EFORMAT: return "chunk file size is not metapage + chunk (file format error)";
        default: return "unknown error";
    }
}

int cc_lds_image(void* out, size_t bytes) {
    if (!out || bytes < kLdsBytes) return CC_EINVAL;
    build_lds_image(static_cast<uint32_t*>(out));
    return CC_OK;
}

int cc_hbm_read_probe_dev(const void* d_buf, uint64_t bytes, uint32_t* d_sink, void* stream) {
    if (!d_buf || !d_sink || bytes % 4096 || ((uintptr_t)d_buf & 15u)) return CC_EINVAL;
    if (bytes == 0) return CC_OK;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    return map_err(launch_read_probe(d_buf, bytes, d_sink, 2 * c->cus, static_cast<hipStream_t>(stream)));
}

int cc_page_load_probe_dev(const void* d_pages, uint64_t n_pages, uint32_t* d_out, void* stream) {
    if (n_pages == 0) return CC_OK;
    if (!d_pages || !d_out || ((uintptr_t)d_pages & 3u)) return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    PageLaunch a = {};
    a.pages = static_cast<const uint32_t*>(d_pages);
    a.n_pages = n_pages;
    a.words_per_lane = 4096 / kWaveBytes;
    a.image = c->image;
    a.out = d_out;
    return map_err(launch_page_tail(c.get(), a, false, static_cast<hipStream_t>(stream), true));
}

int cc_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int cc_engine_init(const cc_opts* opts) {
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (opts) {
            if (opts->page_bytes && !page_size_ok(opts->page_bytes)) return CC_EINVAL;
            if (opts->page_bytes) g_opts.page_bytes = opts->page_bytes;
            if (opts->slice_bytes) g_opts.slice_bytes = opts->slice_bytes;
            if (opts->staging_bytes) g_opts.staging_bytes = opts->staging_bytes;
        }
    }
    CtxRef c;
    return get_ctx(&c);
}

int cc_engine_fini(void) {
    // unpublish every context; each is freed here, or by the last call still
    // holding it (that call's kernels are synchronised before the free)
    std::vector<CtxRef> old;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        for (int d = 0; d < kMaxDevices; d++) {
            CtxRef c = std::atomic_exchange(&g_ctx[d], CtxRef());
            if (c) old.push_back(std::move(c));
        }
    }
    old.clear();
    return CC_OK;
}

int cc_engine_trim(void) {
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    // take the cached tables and scratch out of the context under their
    // mutexes (a call after this point creates fresh ones), then wait for the
    // device WITHOUT the mutexes: a stream stuck in a collective whose peer is
    // gone (what cc_comm_wait bounds) then blocks only this call, never the
    // write-log / range / verify calls of other threads
    std::vector<void*> dead;
    {
        std::lock_guard<std::mutex> lk(c->log_mu);
        for (auto& t : c->log_tabs)
            if (t.p) dead.push_back(t.p);
        c->log_tabs.clear();
    }
    {
        std::lock_guard<std::mutex> lk(c->range_mu);
        for (auto& t : c->range_works)
            if (t.p) dead.push_back(t.p);
        c->range_works.clear();
    }
    const hipError_t e = hipDeviceSynchronize();  // kernels of earlier calls may still use them
    if (e != hipSuccess) return map_err(e);  // (not freed: a faulted device keeps them)
    for (void* p : dead) (void)hipFree(p);
    return CC_OK;
}

uint64_t cc_engine_stream_entries(void) {
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return 0;
    CtxRef c = std::atomic_load(&g_ctx[dev]);
    if (!c) return 0;
    uint64_t n = 0;
    {
        std::lock_guard<std::mutex> lk(c->tail_mu);
        n += c->tails.size();
    }
    {
        std::lock_guard<std::mutex> lk(c->log_mu);
        n += c->log_tabs.size();
    }
    {
        std::lock_guard<std::mutex> lk(c->range_mu);
        n += c->range_works.size();
    }
    return n;
}

int cc_page_crc_dev(const void* d_pages, uint64_t n_pages, uint32_t page_bytes, uint32_t* d_out, void* stream) {
    if (!page_size_ok(page_bytes)) return CC_EINVAL;
    if (n_pages == 0) return CC_OK;
    if (!d_pages || !d_out || ((uintptr_t)d_pages & 3u)) return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    PageLaunch a = {};
    a.pages = static_cast<const uint32_t*>(d_pages);
    a.n_pages = n_pages;
    a.words_per_lane = page_bytes / kWaveBytes;
    a.image = c->image;
    a.kconst = kconst_for(page_bytes);
    a.out = d_out;
    return map_err(launch_page_tail(c.get(), a, false, static_cast<hipStream_t>(stream)));
}

extern "C++" {  // engine-internal (C++ linkage), used by pool.hip
namespace cc {
// cc_pool_scan_dev's page launches (pool.hip): the metapage launch (static
// walk) clears the data launch's tail counter and the digest partials as its
// block 0 starts, so the scan step needs no memset launches; the data launch
// then runs with that counter.
int pool_page_launches(const void* d_data, uint64_t n_data_pages, uint32_t page_bytes, uint32_t* d_page_crcs,
                       const void* d_meta, uint64_t n_meta, uint32_t meta_bytes, uint32_t* d_meta_crcs,
                       uint32_t* d_digest, uint64_t digest_words, hipStream_t s, void* ev_begin, void* ev_end) {
    if (!page_size_ok(page_bytes) || !page_size_ok(meta_bytes)) return CC_EINVAL;
    if (!d_data || !d_page_crcs || !d_meta || !d_meta_crcs || ((uintptr_t)d_data & 3u) || ((uintptr_t)d_meta & 3u))
        return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    PageLaunch a = {};
    a.pages = static_cast<const uint32_t*>(d_data);
    a.n_pages = n_data_pages;
    a.words_per_lane = page_bytes / kWaveBytes;
    a.image = c->image;
    a.kconst = kconst_for(page_bytes);
    a.out = d_page_crcs;
    hipError_t e = hipSuccess;
    if (meta_bytes == page_bytes && n_meta && plan_tail(c.get(), a)) {
        // ONE launch: the metapages are chunks of the data launch's dynamic tail
        // (same page size, same kconst); block 0 clears the digest
        a.meta_pages = static_cast<const uint32_t*>(d_meta);
        a.n_meta = n_meta;
        a.meta_out = d_meta_crcs;
        a.zero[0] = d_digest;
        a.zero_words[0] = d_digest ? digest_words : 0;
        // the caller's event pair rides the data launch itself (no marker packets in the step)
        a.ev_begin = static_cast<hipEvent_t>(ev_begin);
        a.ev_end = static_cast<hipEvent_t>(ev_end);
        e = launch_page_tail(c.get(), a, false, s);
        return map_err(e);
    } else {
        // a metapage launch of its own (static walk; clears the digest), then the data
        PageLaunch m = {};
        m.pages = static_cast<const uint32_t*>(d_meta);
        m.n_pages = n_meta;
        m.words_per_lane = meta_bytes / kWaveBytes;
        m.image = c->image;
        m.kconst = kconst_for(meta_bytes);
        m.out = d_meta_crcs;
        m.zero[0] = d_digest;
        m.zero_words[0] = d_digest ? digest_words : 0;
        geometry_for(c.get(), n_meta, &m);
        e = launch_page_meta(m, s);
        a.ev_begin = static_cast<hipEvent_t>(ev_begin);
        a.ev_end = static_cast<hipEvent_t>(ev_end);
        if (e == hipSuccess) e = launch_page_tail(c.get(), a, false, s);
    }
    return map_err(e);
}
}  // namespace cc
}  // extern "C++"

int cc_page_verify_list_dev(const void* d_pages, uint64_t n_pages, uint32_t page_bytes, const uint32_t* d_expected,
                            uint64_t* d_bad_count, uint64_t* d_first_bad, uint64_t* d_bad_pages,
                            uint64_t max_bad_pages, void* stream) {
    if (!page_size_ok(page_bytes)) return CC_EINVAL;
    if (n_pages == 0) return CC_OK;
    if (!d_pages || !d_expected || !d_bad_count || !d_first_bad || ((uintptr_t)d_pages & 3u)) return CC_EINVAL;
    if (max_bad_pages && !d_bad_pages) return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    PageLaunch a = {};
    a.pages = static_cast<const uint32_t*>(d_pages);
    a.n_pages = n_pages;
    a.words_per_lane = page_bytes / kWaveBytes;
    a.image = c->image;
    a.kconst = kconst_for(page_bytes);
    a.expected = d_expected;
    a.sink.bad_count = reinterpret_cast<unsigned long long*>(d_bad_count);
    a.sink.first_bad = reinterpret_cast<unsigned long long*>(d_first_bad);
    a.sink.list = max_bad_pages ? reinterpret_cast<unsigned long long*>(d_bad_pages) : nullptr;
    a.sink.max_list = max_bad_pages;
    return map_err(launch_page_tail(c.get(), a, true, static_cast<hipStream_t>(stream)));
}

int cc_page_verify_dev(const void* d_pages, uint64_t n_pages, uint32_t page_bytes, const uint32_t* d_expected,
                       uint64_t* d_bad_count, uint64_t* d_first_bad, void* stream) {
    return cc_page_verify_list_dev(d_pages, n_pages, page_bytes, d_expected, d_bad_count, d_first_bad, nullptr, 0,
                                   stream);
}

int cc_fold_dev(const uint32_t* d_crcs, uint64_t n_groups, uint32_t per_group, uint64_t unit_bytes,
                uint32_t* d_out, void* stream) {
    if (n_groups == 0) return CC_OK;
    if (!d_crcs || !d_out || per_group == 0 || unit_bytes == 0) return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    FoldLaunch a = {};
    a.crcs = d_crcs;
    a.n_groups = n_groups;
    a.per_group = per_group;
    a.m_unit = xpow(unit_bytes << 3);
    const uint64_t q = per_group / 64;
    for (int t = 0; t < 6; t++) a.m_tree[t] = xpow((unit_bytes * q << t) << 3);
    a.out = d_out;
    return map_err(launch_fold(a, static_cast<hipStream_t>(stream)));
}

int cc_shift_dev(const uint32_t* d_crcs, const uint64_t* d_shift_bytes, uint64_t n, uint32_t* d_out, void* stream) {
    if (n == 0) return CC_OK;
    if (!d_crcs || !d_shift_bytes || !d_out) return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    return map_err(launch_shift(d_crcs, d_shift_bytes, n, d_out, static_cast<hipStream_t>(stream)));
}

extern "C++" {
namespace {
// The stream's range scratch: kRangeTiles tile words, the tail block, then the
// accumulator pairs of up to `cap` ranges; zero when created (cleared on the
// stream), kept so by every launch (kernels.h RangeLaunch).  A call with more
// ranges than kRangeCacheRanges, or past kMaxTailBlocks streams, gets scratch
// of its own for the call (nullptr here).  Caller holds c->range_mu.
constexpr uint64_t kRangeHeader = (kRangeTiles * 8 + kTailBlockBytes + 255) & ~255ull;
constexpr uint64_t kRangeCacheRanges = 1ull << 22;  // 32 MiB of accumulators a stream at most
DevCtx::RangeWork* range_work(DevCtx* c, hipStream_t s, uint64_t n, hipError_t* err) {
    *err = hipSuccess;
    if (n > kRangeCacheRanges) return nullptr;
    const StreamKey key = stream_key(s);
    DevCtx::RangeWork* t = nullptr;
    for (auto& x : c->range_works)
        if (x.s == key) t = &x;
    if (t && t->cap < n) {
        if ((*err = hipFreeAsync(t->p, s)) != hipSuccess) return nullptr;
        t->p = nullptr;
        t->cap = 0;
    }
    if (!t) {
        if (c->range_works.size() >= kMaxTailBlocks) return nullptr;
        c->range_works.push_back({key, nullptr, 0, 0, false});
        if (s == hipStreamPerThread) note_thread_entry(c);
        t = &c->range_works.back();
    }
    if (!t->p) {
        uint64_t cap = 1ull << 16;
        while (cap < n) cap <<= 1;
        void* p = nullptr;
        if ((*err = hipMallocAsync(&p, kRangeHeader + cap * 8, s)) != hipSuccess) return nullptr;
        t->p = static_cast<unsigned char*>(p);
        t->cap = cap;
        t->dirty = true;
    }
    if (t->dirty) {
        if ((*err = hipMemsetAsync(t->p, 0, kRangeHeader + t->cap * 8, s)) != hipSuccess) return nullptr;
        t->dirty = false;
    }
    return t;
}

// The stream's range scratch for one launch: the tile words, the tail slots,
// `n_acc` accumulator pairs, and the call's epoch, handed to launch(tiles,
// tail, acc, epoch) under c->range_mu (the epoch order is the stream order).
// Scratch of the call's own (allocated and cleared on the stream) when the
// stream has none cached for that size.
template <typename F>
hipError_t with_range_scratch(DevCtx* c, hipStream_t s, uint64_t n_acc, F launch) {
    std::lock_guard<std::mutex> lk(c->range_mu);
    hipError_t e;
    DevCtx::RangeWork* w = range_work(c, s, n_acc, &e);
    if (e != hipSuccess) return e;
    unsigned char* base = nullptr;
    unsigned char* tmp = nullptr;
    uint32_t epoch = 1;
    if (w) {
        base = w->p;
        // 24-bit epochs; the wrap keeps the parity alternating (2^24 - 1 is odd:
        // next 2), as the tail's counter slots need
        w->epoch = w->epoch + 1 < (1u << 24) ? w->epoch + 1 : 2u;
        epoch = w->epoch;
    } else {
        const uint64_t bytes = kRangeHeader + n_acc * 8;
        if ((e = hipMallocAsync(reinterpret_cast<void**>(&tmp), bytes, s)) != hipSuccess) return e;
        if ((e = hipMemsetAsync(tmp, 0, bytes, s)) != hipSuccess) {
            (void)hipFreeAsync(tmp, s);
            return e;
        }
        base = tmp;
    }
    e = launch(reinterpret_cast<uint64_t*>(base), reinterpret_cast<unsigned long long*>(base + kRangeTiles * 8),
               reinterpret_cast<uint32_t*>(base + kRangeHeader), epoch);
    if (w && e != hipSuccess) w->dirty = true;  // may have run in part: clear before the next use
    if (tmp) {
        const hipError_t f = hipFreeAsync(tmp, s);
        if (e == hipSuccess) e = f;
    }
    return e;
}

// One range batch (the flat kernel, kernels.h launch_range_flat) on stream s.
hipError_t range_batch(DevCtx* c, const unsigned char* buf, const RangeDesc* rd, uint64_t n, uint32_t* out,
                       hipStream_t s) {
    if (n == 0) return hipSuccess;
    RangeLaunch a = {};
    a.buf = buf;
    a.ranges = rd;
    a.n = n;
    a.image = c->image;
    a.out = out;
    a.blocks = c->cus;
    return with_range_scratch(c, s, n, [&](uint64_t* tiles, unsigned long long* tail, uint32_t* acc, uint32_t epoch) {
        a.tiles = tiles;
        a.tail = tail;
        a.acc = acc;
        a.epoch = epoch;
        return launch_range_flat(a, s);
    });
}
}  // namespace
}  // extern "C++"

int cc_crc_ranges_dev(const void* d_buf, const cc_range* d_ranges, uint64_t n, uint32_t* d_out, void* stream) {
    if (n == 0) return CC_OK;
    if (!d_buf || !d_ranges || !d_out) return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    // every wave an equal share of the batch's 4 KiB blocks, in one launch
    return map_err(range_batch(c.get(), static_cast<const unsigned char*>(d_buf),
                               reinterpret_cast<const RangeDesc*>(d_ranges), n, d_out,
                               static_cast<hipStream_t>(stream)));
}

int cc_crc_bufs_host(const void* const* h_bufs, const uint64_t* h_lens, uint64_t n, uint32_t* h_out) {
    if (n == 0) return CC_OK;
    if (!h_bufs || !h_lens || !h_out) return CC_EINVAL;
    for (uint64_t i = 0; i < n; i++)
        if (h_lens[i] && !h_bufs[i]) return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(c->submit);
    if ((rc = staging_init(c.get()))) return rc;
    Staging& st = c->st;
    SlotRing ring(st);
    // batches of whole buffers packed back to back (4-byte aligned) into a
    // staging slot; a buffer larger than a slot is hashed in slot-sized pieces
    // combined on the host.  Records go in the result region's tail.
    const uint64_t slot = st.bytes;
    // result region per slot (st.bytes / 64 bytes): k CRCs, then the k range
    // records at the next 256-byte boundary
    const uint64_t max_recs = (st.bytes / 64 - 256) / (sizeof(RangeDesc) + 4);
    uint64_t i = 0, off_in_i = 0;
    int s = 0;
    struct Item {
        uint64_t buf;  // index of the buffer
        uint64_t off;  // byte offset inside the buffer
        uint64_t len;
    };
    std::vector<Item> items[2];
    std::vector<uint32_t> acc(n, 0);       // running CRC of each buffer (pieces in order)
    std::vector<uint8_t> started(n, 0);
    auto take = [&](int sl) {
        return [&, sl](uint64_t, uint64_t k) {
            const uint32_t* r = st.hcrc[sl];
            for (uint64_t j = 0; j < k; j++) {
                const Item& it = items[sl][j];
                acc[it.buf] = started[it.buf] ? crc32c_combine(acc[it.buf], r[j], it.len) : r[j];
                started[it.buf] = 1;
            }
        };
    };
    while (i < n) {
        if ((rc = ring.drain(s, take(s)))) return rc;
        items[s].clear();
        unsigned char* hs = static_cast<unsigned char*>(st.host[s]);
        uint64_t used = 0;
        while (i < n && items[s].size() < max_recs) {
            const uint64_t rem = h_lens[i] - off_in_i;
            const uint64_t room = slot - used;
            if (rem == 0) {  // empty buffer: CRC 0, no bytes
                if (!started[i]) acc[i] = 0;
                started[i] = 1;
                i++;
                off_in_i = 0;
                continue;
            }
            if (room < 256) break;
            const uint64_t take_n = rem < room ? rem : (room & ~255ull);
            memcpy(hs + used, static_cast<const unsigned char*>(h_bufs[i]) + off_in_i, take_n);
            items[s].push_back(Item{i, off_in_i, take_n});
            used = (used + take_n + 255) & ~255ull;
            off_in_i += take_n;
            if (off_in_i == h_lens[i]) {
                i++;
                off_in_i = 0;
            }
        }
        const uint64_t k = items[s].size();
        if (k == 0) continue;
        hipStream_t strm = st.stream[s];
        const uint64_t rec_off = align256(k * 4);
        RangeDesc* recs = reinterpret_cast<RangeDesc*>(reinterpret_cast<unsigned char*>(st.hcrc[s]) + rec_off);
        RangeDesc* drecs = reinterpret_cast<RangeDesc*>(reinterpret_cast<unsigned char*>(st.dcrc[s]) + rec_off);
        uint64_t o = 0;
        for (uint64_t j = 0; j < k; j++) {
            recs[j] = RangeDesc{o, items[s][j].len};
            o = (o + items[s][j].len + 255) & ~255ull;
        }
        hipError_t e;
        if ((e = hipMemcpyAsync(st.dev[s], hs, used, hipMemcpyHostToDevice, strm)) != hipSuccess)
            return ring.fail(map_err(e));
        if ((e = hipMemcpyAsync(drecs, recs, k * sizeof(RangeDesc), hipMemcpyHostToDevice, strm)) != hipSuccess)
            return ring.fail(map_err(e));
        if ((e = range_batch(c.get(), static_cast<const unsigned char*>(st.dev[s]), drecs, k, st.dcrc[s], strm)) !=
            hipSuccess)
            return ring.fail(map_err(e));
        if ((e = hipMemcpyAsync(st.hcrc[s], st.dcrc[s], k * 4, hipMemcpyDeviceToHost, strm)) != hipSuccess)
            return ring.fail(map_err(e));
        if ((e = arm_slot(st, s, strm)) != hipSuccess) return ring.fail(map_err(e));
        ring.first[s] = 0;
        ring.n[s] = k;
        s ^= 1;
    }
    if ((rc = ring.drain(s, take(s)))) return rc;
    if ((rc = ring.drain(s ^ 1, take(s ^ 1)))) return rc;
    for (uint64_t j = 0; j < n; j++) h_out[j] = acc[j];
    return CC_OK;
}

namespace cc {
namespace {
// Geometry check + multipliers for the fused epilogue; false if unsupported.
bool epilogue_geometry(DevCtx* c, uint32_t pages_per_chunk, uint32_t page_bytes, uint32_t pages_per_slice,
                       EpilogueLaunch* a) {
    if (pages_per_chunk == 0 || pages_per_chunk % 256 || pages_per_slice == 0) return false;
    const uint32_t q = pages_per_chunk / 256;
    if (pages_per_slice % q) return false;
    const uint32_t tps = pages_per_slice / q;  // threads per slice
    if (tps & (tps - 1) || tps > 256) return false;
    uint32_t j = 0;
    while ((1u << j) < tps) j++;
    a->pages_per_chunk = pages_per_chunk;
    a->q = q;
    a->slice_shift = j;
    // product tables of the 10 geometry constants, built on the host once per
    // (page_bytes, q) and kept on the device; looked up without a lock
    const uint64_t key = (((uint64_t)page_bytes << 32) | q) + 1;
    for (int i = 0; i < kEpiSlots; i++)
        if (c->epi_key[i].load(std::memory_order_acquire) == key) {
            a->mtab = static_cast<const uint32_t*>(c->epi_ptr[i].load(std::memory_order_relaxed));
            return true;
        }
    std::lock_guard<std::mutex> lk(c->tab_mu);
    int free_slot = -1;
    for (int i = 0; i < kEpiSlots; i++) {
        const uint64_t k = c->epi_key[i].load(std::memory_order_acquire);
        if (k == key) {
            a->mtab = static_cast<const uint32_t*>(c->epi_ptr[i].load(std::memory_order_relaxed));
            return true;
        }
        if (k == 0 && free_slot < 0) free_slot = i;
    }
    if (free_slot < 0) return false;  // more geometries than slots: refuse rather than evict a table in use
    uint32_t m[10];
    m[0] = xpow((uint64_t)page_bytes << 3);
    for (int k = 0; k < 8; k++) m[1 + k] = xpow(((uint64_t)page_bytes * q << k) << 3);
    m[9] = xpow((uint64_t)pages_per_chunk * page_bytes << 3);
    std::vector<uint32_t> h(10 * 1024);
    for (int t = 0; t < 10; t++)
        for (uint32_t k = 0; k < 4; k++)
            for (uint32_t b = 0; b < 256; b++) h[t * 1024 + k * 256 + b] = mulmod(m[t], b << (8 * k));
    void* dev = nullptr;
    if (hipMalloc(&dev, h.size() * 4) != hipSuccess) return false;
    if (hipMemcpy(dev, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(dev);  // never publish a half-initialised table
        return false;
    }
    c->epi_ptr[free_slot].store(dev, std::memory_order_relaxed);
    c->epi_key[free_slot].store(key, std::memory_order_release);
    a->mtab = static_cast<const uint32_t*>(dev);
    return true;
}
}  // namespace
}  // namespace cc

int cc_xpow8_dev(const uint64_t* d_nbytes, uint64_t n, uint32_t* d_out, void* stream) {
    if (n == 0) return CC_OK;
    if (!d_nbytes || !d_out) return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    return map_err(launch_xpow8(d_nbytes, n, d_out, static_cast<hipStream_t>(stream)));
}

int cc_scan_epilogue_dev(const uint32_t* d_page_crcs, const uint32_t* d_meta_crcs, uint64_t n_chunks,
                         uint32_t pages_per_chunk, uint32_t page_bytes, uint32_t pages_per_slice,
                         uint32_t* d_slice_crcs, uint32_t* d_file_crcs, const uint32_t* d_after_mult,
                         const uint32_t* d_group, uint32_t* d_digest, void* stream) {
    if (n_chunks == 0) return CC_OK;
    if (!d_page_crcs || !d_meta_crcs || !d_slice_crcs || page_bytes == 0) return CC_EINVAL;
    const bool dig = d_after_mult || d_group || d_digest;
    if (dig && !(d_after_mult && d_group && d_digest)) return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    EpilogueLaunch a = {};
    if (!epilogue_geometry(c.get(), pages_per_chunk, page_bytes, pages_per_slice, &a)) return CC_EINVAL;
    a.page_crcs = d_page_crcs;
    a.meta_crcs = d_meta_crcs;
    a.n_chunks = n_chunks;
    a.slice_crcs = d_slice_crcs;
    a.file_crcs = d_file_crcs;
    a.after_mult = d_after_mult;
    a.group = d_group;
    a.digest = d_digest;
    return map_err(launch_epilogue(a, static_cast<hipStream_t>(stream)));
}

int cc_combine_dev(const uint32_t* d_a, const uint32_t* d_b, uint64_t len_b, uint64_t n, uint32_t* d_out,
                   void* stream) {
    if (n == 0) return CC_OK;
    if (!d_a || !d_b || !d_out) return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    return map_err(launch_combine(d_a, d_b, xpow(len_b << 3), n, d_out, static_cast<hipStream_t>(stream)));
}

int cc_digest_dev(const uint32_t* d_file_crcs, const uint64_t* d_after_bytes, const uint32_t* d_group,
                  uint64_t n_files, uint32_t* d_digest, void* stream) {
    if (n_files == 0) return CC_OK;
    if (!d_file_crcs || !d_after_bytes || !d_group || !d_digest) return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    return map_err(launch_digest(d_file_crcs, d_after_bytes, d_group, n_files, d_digest,
                                 static_cast<hipStream_t>(stream)));
}

int cc_digest_fold_dev(const uint32_t* d_gathered, uint32_t nranks, uint64_t n, uint32_t* d_digest, void* stream) {
    if (n == 0) return CC_OK;
    if (!d_gathered || !d_digest || nranks == 0) return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    return map_err(launch_xor_fold(d_gathered, nranks, n, d_digest, static_cast<hipStream_t>(stream)));
}

namespace cc {
namespace {
// One call on a lane of its own (LanePool): H2D (straight from the caller's
// buffer when it is pinned, else through the lane's pinned staging a piece at
// a time, each piece's DMA running while the next is copied), the page kernel
// storing the CRCs straight into the lane's pinned CRC buffer (no D2H copy),
// then a stream write of the lane's completion word, which the caller sleeps
// on (lane_wait).  The lane goes back idle only with its stream drained.
int page_crc_lane(DevCtx* c, const void* h_pages, uint64_t n_pages, uint32_t page_bytes, uint32_t* h_out) {
    int rc = CC_OK;
    Lane* l = lane_get(c, &rc);
    if (!l) return rc;
    const uint64_t bytes = n_pages * page_bytes;
    const uint64_t ahead = c->lanes.inflight.fetch_add(bytes) + bytes;
    hipError_t e = hipSuccess;
    if (is_pinned(h_pages)) {
        e = hipMemcpyAsync(l->dev, h_pages, bytes, hipMemcpyHostToDevice, l->stream);
    } else {
        if (!l->host) e = hipHostMalloc(&l->host, kLaneBytes, hipHostMallocDefault);
        for (uint64_t o = 0; e == hipSuccess && o < bytes; o += kLanePiece) {
            const uint64_t k = bytes - o < kLanePiece ? bytes - o : kLanePiece;
            memcpy(static_cast<unsigned char*>(l->host) + o, static_cast<const unsigned char*>(h_pages) + o, k);
            e = hipMemcpyAsync(static_cast<unsigned char*>(l->dev) + o, static_cast<unsigned char*>(l->host) + o, k,
                               hipMemcpyHostToDevice, l->stream);
        }
    }
    if (e == hipSuccess) {
        PageLaunch a = {};
        a.pages = static_cast<const uint32_t*>(l->dev);
        a.n_pages = n_pages;
        a.words_per_lane = page_bytes / kWaveBytes;
        a.image = c->image;
        a.kconst = kconst_for(page_bytes);
        a.out = l->hcrc;
        geometry_for(c, n_pages, &a);
        e = launch_page_crc(a, l->stream);
    }
    const uint32_t want = ++l->seq;
    if (e == hipSuccess) e = hipStreamWriteValue32(l->stream, l->hflag, want, 0);
    if (e == hipSuccess)
        e = lane_wait(l, want, ahead);
    else
        (void)hipStreamSynchronize(l->stream);  // whatever was enqueued finishes before the lane is reused
    c->lanes.inflight.fetch_sub(bytes);
    if (e == hipSuccess) memcpy(h_out, l->hcrc, n_pages * 4);
    lane_put(c, l);
    return map_err(e);
}
}  // namespace
}  // namespace cc

// Host in / host out.  A call of at most kLaneBytes runs on a lane of its own
// (page_crc_lane: concurrent callers overlap).  A larger one takes the
// device's two shared staging slots (held for the whole call): while slot i's
// pages are copied in and hashed on stream i, the CPU fills slot i^1 (pageable
// input) or -- when the caller's buffer is already pinned (chunk files pread
// into pinned memory) -- the DMA reads it directly.
int cc_page_crc_host(const void* h_pages, uint64_t n_pages, uint32_t page_bytes, uint32_t* h_out) {
    if (!page_size_ok(page_bytes)) return CC_EINVAL;
    if (n_pages == 0) return CC_OK;
    if (!h_pages || !h_out) return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    if (n_pages <= kLaneBytes / page_bytes) return page_crc_lane(c.get(), h_pages, n_pages, page_bytes, h_out);
    std::lock_guard<std::mutex> lk(c->submit);
    if ((rc = staging_init(c.get()))) return rc;
    Staging& st = c->st;
    SlotRing ring(st);
    const bool pinned = is_pinned(h_pages);
    const uint64_t per_slot = st.bytes / page_bytes;
    const unsigned char* src = static_cast<const unsigned char*>(h_pages);
    auto take = [&](int s) {
        return [&, s](uint64_t f, uint64_t k) { memcpy(h_out + f, st.hcrc[s], k * 4); };
    };
    uint64_t done = 0;
    int slot = 0;
    hipError_t e = hipSuccess;
    while (done < n_pages) {
        const uint64_t n = (n_pages - done < per_slot) ? n_pages - done : per_slot;
        // reclaim this slot: wait for its previous batch and copy its CRCs out
        if ((rc = ring.drain(slot, take(slot)))) return rc;
        const void* hsrc = src + done * page_bytes;
        if (!pinned) {
            memcpy(st.host[slot], hsrc, n * page_bytes);
            hsrc = st.host[slot];
        }
        // H2D on the FIFO copy stream (Staging::copy), the slot's stream waits for it
        if ((e = hipMemcpyAsync(st.dev[slot], hsrc, n * page_bytes, hipMemcpyHostToDevice, st.copy)) != hipSuccess ||
            (e = hipEventRecord(st.copied[slot], st.copy)) != hipSuccess ||
            (e = hipStreamWaitEvent(st.stream[slot], st.copied[slot], 0)) != hipSuccess)
            return ring.fail(map_err(e));
        PageLaunch a = {};
        a.pages = static_cast<const uint32_t*>(st.dev[slot]);
        a.n_pages = n;
        a.words_per_lane = page_bytes / kWaveBytes;
        a.image = c->image;
        a.kconst = kconst_for(page_bytes);
        a.out = st.dcrc[slot];
        geometry_for(c.get(), n, &a);
        if ((e = launch_page_crc(a, st.stream[slot])) != hipSuccess) return ring.fail(map_err(e));
        if ((e = hipMemcpyAsync(st.hcrc[slot], st.dcrc[slot], n * 4, hipMemcpyDeviceToHost, st.stream[slot])) !=
            hipSuccess)
            return ring.fail(map_err(e));
        if ((e = arm_slot(st, slot, st.stream[slot])) != hipSuccess) return ring.fail(map_err(e));
        ring.first[slot] = done;
        ring.n[slot] = n;
        done += n;
        slot ^= 1;
    }
    if ((rc = ring.drain(slot, take(slot)))) return rc;
    return ring.drain(slot ^ 1, take(slot ^ 1));
}

namespace {
inline bool log_page_ok(uint32_t page_bytes) {
    const uint32_t m = page_bytes / kWaveBytes;
    return page_bytes % kWaveBytes == 0 && m >= 1 && m <= 32 && (m & (m - 1)) == 0;
}
inline uint32_t log_slots(uint32_t max_len, uint32_t page_bytes) { return (max_len - 1) / page_bytes + 2; }
}  // namespace

namespace {
// The caller's work buffer of the write log: next links | head segments (one
// per insert block) | segment counts (none needs clearing).  The page table
// lives in the engine (LogTable): a 256-byte header (unused), then the
// open-addressing table.
struct LogWork {
    uint64_t n_pieces, table_entries, next_off, heads_off, counts_off, bytes;
    uint32_t n_segs, seg_cap;
};
constexpr uint64_t kLogTableHeader = 256;
bool log_work(uint64_t n_updates, uint32_t max_len, uint32_t page_bytes, LogWork* w) {
    if (!log_page_ok(page_bytes) || max_len == 0 || n_updates == 0) return false;
    w->n_pieces = n_updates * log_slots(max_len, page_bytes);
    if (w->n_pieces >= (1ull << 31)) return false;
    // table entries >= 8 x pieces (2 x -> 4 x: insert 15.8 -> 11.2 us; 8 x cost a
    // 5 us memset until the engine-owned table needed none: round 3, 8 x -1.1 % a
    // batch): load <= 1/8, up to the 2^32 slots 32-bit slot indices reach; never above 1/4
    uint64_t te = 1024;
    while (te < 8 * w->n_pieces && te < (1ull << 32)) te <<= 1;
    if (te < 4 * w->n_pieces) return false;
    w->table_entries = te;
    // insert blocks: one per 1,024-piece chunk up to kInsertBlocks (then
    // grid-stride); block b's head segment holds the records of its chunks
    const uint64_t chunks = (w->n_pieces + kInsertThreads - 1) / kInsertThreads;
    w->n_segs = (uint32_t)(chunks < kInsertBlocks ? chunks : kInsertBlocks);
    const uint64_t cap = (chunks + w->n_segs - 1) / w->n_segs * kInsertThreads;
    if (cap >= (1ull << 32)) return false;
    w->seg_cap = (uint32_t)cap;
    w->next_off = 0;
    w->heads_off = align256(w->n_pieces * 4);
    w->counts_off = w->heads_off + align256((uint64_t)w->n_segs * cap * 8);  // head records {table slot, claiming piece}
    w->bytes = w->counts_off + align256(kInsertBlocks * 4);
    return true;
}

// The stream's write-log table with >= `entries` slots, zero when the call's
// launches run (caller holds c->log_mu).  Created or grown (stream-ordered
// free of the old one) with a clear on the stream; a table a failed call left
// dirty is cleared.  nullptr when kMaxTailBlocks streams already hold one, or
// when the log needs more than kLogTableCacheEntries slots (such a call takes a
// table of its own, freed with it: one huge log must not pin device memory for
// the rest of the process).  cc_engine_trim frees every cached table.
constexpr uint64_t kLogTableCacheEntries = 1ull << 23;  // 64 MiB a stream: logs of up to 1M pieces (512K two-page writes)
DevCtx::LogTable* log_table(DevCtx* c, hipStream_t s, uint64_t entries, hipError_t* err) {
    *err = hipSuccess;
    if (entries > kLogTableCacheEntries) return nullptr;  // a log this big: a table for its call only
    const StreamKey key = stream_key(s);
    DevCtx::LogTable* t = nullptr;
    for (auto& x : c->log_tabs)
        if (x.s == key) t = &x;
    if (t && t->entries < entries) {
        if ((*err = hipFreeAsync(t->p, s)) != hipSuccess) return nullptr;
        t->p = nullptr;
        t->entries = 0;
    }
    if (!t) {
        if (c->log_tabs.size() >= kMaxTailBlocks) return nullptr;
        c->log_tabs.push_back({key, nullptr, 0, false});
        if (s == hipStreamPerThread) note_thread_entry(c);
        t = &c->log_tabs.back();
    }
    if (!t->p) {
        void* p = nullptr;
        if ((*err = hipMallocAsync(&p, kLogTableHeader + entries * 8, s)) != hipSuccess) return nullptr;
        t->p = static_cast<unsigned char*>(p);
        t->entries = entries;
        t->dirty = true;
    }
    if (t->dirty) {
        if ((*err = hipMemsetAsync(t->p, 0, kLogTableHeader + t->entries * 8, s)) != hipSuccess) return nullptr;
        t->dirty = false;
    }
    return t;
}
}  // namespace

uint64_t cc_apply_log_work_bytes(uint64_t n_updates, uint32_t max_len, uint32_t page_bytes) {
    LogWork w;
    return log_work(n_updates, max_len, page_bytes, &w) ? w.bytes : 0;
}

namespace {
int apply_log(void* d_pool, uint64_t pool_bytes, uint32_t page_bytes, const void* d_src, const cc_update* d_log,
              uint64_t n_updates, uint32_t max_len, uint32_t* d_page_crcs, void* d_work, uint64_t work_bytes,
              void* stream, int delta) {
    if (!log_page_ok(page_bytes)) return CC_EINVAL;
    if (n_updates == 0) return CC_OK;
    if (!d_pool || !d_src || !d_log || !d_page_crcs || !d_work || max_len == 0) return CC_EINVAL;
    if (pool_bytes % page_bytes || ((uintptr_t)d_pool & 3u) || ((uintptr_t)d_src & 3u)) return CC_EINVAL;
    const uint64_t n_pages = pool_bytes / page_bytes;
    if (n_pages >= kNoPiece) return CC_EINVAL;  // page + 1 must fit the table entry's 32-bit key
    LogWork lw;
    if (!log_work(n_updates, max_len, page_bytes, &lw) || work_bytes < lw.bytes) return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    unsigned char* w = static_cast<unsigned char*>(d_work);
    LogLaunch a = {};
    a.pool = static_cast<unsigned char*>(d_pool);
    a.pool_bytes = pool_bytes;
    a.src = static_cast<const unsigned char*>(d_src);
    a.upd = reinterpret_cast<const UpdateDesc*>(d_log);
    a.n_updates = n_updates;
    a.page_bytes = page_bytes;
    a.max_len = max_len;
    a.slots = log_slots(max_len, page_bytes);
    a.n_pieces = lw.n_pieces;
    a.next = reinterpret_cast<uint32_t*>(w + lw.next_off);
    a.heads = reinterpret_cast<uint32_t*>(w + lw.heads_off);
    a.seg_count = reinterpret_cast<uint32_t*>(w + lw.counts_off);
    a.n_segs = lw.n_segs;
    a.seg_cap = lw.seg_cap;
    a.image = c->image;
    a.kconst = kconst_for(page_bytes);
    a.page_crcs = d_page_crcs;
    a.delta = delta;
    // at most n_pieces touched pages: a wave per page up to one block per CU
    const uint64_t blocks = (lw.n_pieces + kLogWaves - 1) / kLogWaves;
    a.blocks = (int)(blocks < (uint64_t)c->cus ? (blocks ? blocks : 1) : (uint64_t)c->cus);
    hipError_t e;
    // logs of up to 64 writes (each within one page's length) take the one-launch path
    if (n_updates <= 64 && a.slots <= 2) return map_err(launch_log_small(a, s));
    // (memset + insert + pages as ONE cooperative launch with two grid barriers
    // measured 0.221 vs 0.162 ms a batch: not kept)
    std::lock_guard<std::mutex> lk(c->log_mu);
    DevCtx::LogTable* t = log_table(c.get(), s, lw.table_entries, &e);
    if (e != hipSuccess) return map_err(e);
    unsigned char* tmp = nullptr;  // no table free for this stream: a cleared one for this call
    if (t) {
        a.clear_table = 1;
        a.table = reinterpret_cast<uint64_t*>(t->p + kLogTableHeader);
        a.table_mask = (uint32_t)(t->entries - 1);
    } else {
        const uint64_t bytes = kLogTableHeader + lw.table_entries * 8;
        if ((e = hipMallocAsync(reinterpret_cast<void**>(&tmp), bytes, s)) != hipSuccess) return map_err(e);
        if ((e = hipMemsetAsync(tmp, 0, bytes, s)) != hipSuccess) {
            (void)hipFreeAsync(tmp, s);
            return map_err(e);
        }
        a.table = reinterpret_cast<uint64_t*>(tmp + kLogTableHeader);
        a.table_mask = (uint32_t)(lw.table_entries - 1);
    }
    e = launch_log_insert(a, s);
    if (e == hipSuccess) e = launch_log_pages(a, s);
    if (t && e != hipSuccess) t->dirty = true;  // the insert may have run: clear before the next use
    if (tmp) {
        const hipError_t f = hipFreeAsync(tmp, s);
        if (e == hipSuccess) e = f;
    }
    return map_err(e);
}
}  // namespace

int cc_apply_log_dev(void* d_pool, uint64_t pool_bytes, uint32_t page_bytes, const void* d_src,
                     const cc_update* d_log, uint64_t n_updates, uint32_t max_len, uint32_t* d_page_crcs,
                     void* d_work, uint64_t work_bytes, void* stream) {
    return apply_log(d_pool, pool_bytes, page_bytes, d_src, d_log, n_updates, max_len, d_page_crcs, d_work,
                     work_bytes, stream, 0);
}

int cc_apply_log_delta_dev(void* d_pool, uint64_t pool_bytes, uint32_t page_bytes, const void* d_src,
                           const cc_update* d_log, uint64_t n_updates, uint32_t max_len, uint32_t* d_page_crcs,
                           void* d_work, uint64_t work_bytes, void* stream) {
    return apply_log(d_pool, pool_bytes, page_bytes, d_src, d_log, n_updates, max_len, d_page_crcs, d_work,
                     work_bytes, stream, 1);
}

// ---- a queue of write logs, pipelined (cc_apply_logs_dev) ----
namespace {
// Head segments of a batch grouped in chunks of T pieces by G blocks (block b
// takes chunks b, b + G, ...): G segments of seg_cap records.
struct SegLayout {
    uint32_t n_segs, seg_cap;
};
bool seg_layout(uint64_t n_pieces, uint32_t T, uint32_t G, SegLayout* l) {
    if (G == 0 || G > kInsertBlocks) return false;
    const uint64_t chunks = (n_pieces + T - 1) / T;
    const uint64_t cap = (chunks + G - 1) / G * T;
    if (cap >= (1ull << 32)) return false;
    l->n_segs = G;
    l->seg_cap = (uint32_t)cap;
    return true;
}

// The caller's work buffer of cc_apply_logs_dev: two regions (batches
// alternate between them) of next links | head segments | segment counts,
// sized for the largest batch under either grouping (the insert kernel's
// chunks of kInsertThreads, or a page kernel's tail over <= kInsertBlocks
// blocks), then the three chunk counters of the tail groupings.  The two hash
// tables are the two halves of the stream's engine table (kept zero).
struct LogsWork {
    uint64_t max_pieces, table_entries, heads_off, counts_off, region, ctr_off, bytes;
};
bool logs_work(uint64_t max_updates, uint32_t max_len, uint32_t page_bytes, LogsWork* w) {
    LogWork one;
    if (!log_work(max_updates, max_len, page_bytes, &one)) return false;
    w->max_pieces = one.n_pieces;
    w->table_entries = one.table_entries;
    // head records: the insert kernel's layout <= pieces + 512 (kInsertBlocks + 1);
    // a page kernel's tail grouping G x rounds x T, rounds = 2 ceil(chunks / G)
    // rounded up to kGroupTake: <= 2 (pieces + T (G + 1)) + (kGroupTake - 1) G T,
    // T <= 1024, G <= kInsertBlocks
    const uint64_t recs = 2 * (w->max_pieces + 1024ull * (kInsertBlocks + 1)) + (kGroupTake - 1) * 1024ull * kInsertBlocks;
    w->heads_off = align256(w->max_pieces * 4);
    w->counts_off = w->heads_off + align256(recs * 8);
    w->region = w->counts_off + align256(kInsertBlocks * 4);
    w->ctr_off = 2 * w->region;
    w->bytes = w->ctr_off + 256;
    return true;
}
}  // namespace

uint64_t cc_apply_logs_work_bytes(uint64_t max_updates, uint32_t max_len, uint32_t page_bytes) {
    LogsWork w;
    return logs_work(max_updates, max_len, page_bytes, &w) ? w.bytes : 0;
}

int cc_apply_logs_dev(void* d_pool, uint64_t pool_bytes, uint32_t page_bytes, const cc_log_batch* batches,
                      uint32_t n_batches, uint32_t max_len, uint32_t* d_page_crcs, int delta, void* d_work,
                      uint64_t work_bytes, void* stream) {
    if (!log_page_ok(page_bytes)) return CC_EINVAL;
    if (n_batches == 0) return CC_OK;
    if (!batches || !d_pool || !d_page_crcs || !d_work || max_len == 0) return CC_EINVAL;
    if (pool_bytes % page_bytes || ((uintptr_t)d_pool & 3u)) return CC_EINVAL;
    if (pool_bytes / page_bytes >= kNoPiece) return CC_EINVAL;
    uint64_t max_n = 0;
    for (uint32_t k = 0; k < n_batches; k++) {
        const cc_log_batch& b = batches[k];
        if (b.n_updates && (!b.d_log || !b.d_src || ((uintptr_t)b.d_src & 3u))) return CC_EINVAL;
        max_n = b.n_updates > max_n ? b.n_updates : max_n;
    }
    if (max_n == 0) return CC_OK;
    LogsWork W;
    if (!logs_work(max_n, max_len, page_bytes, &W) || work_bytes < W.bytes) return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint32_t slots = log_slots(max_len, page_bytes);
    auto small = [&](uint64_t n) { return n <= 64 && slots <= 2; };
    const uint32_t M = page_bytes / kWaveBytes;
    const uint32_t T = 64u * (uint32_t)(M > 16 ? kLogWaves : (delta ? kLogWavesDelta : kLogWavesFull));
    auto base = [&](const cc_log_batch& b) {
        LogLaunch a = {};
        a.pool = static_cast<unsigned char*>(d_pool);
        a.pool_bytes = pool_bytes;
        a.src = static_cast<const unsigned char*>(b.d_src);
        a.upd = reinterpret_cast<const UpdateDesc*>(b.d_log);
        a.n_updates = b.n_updates;
        a.page_bytes = page_bytes;
        a.max_len = max_len;
        a.slots = slots;
        a.n_pieces = b.n_updates * slots;
        a.image = c->image;
        a.kconst = kconst_for(page_bytes);
        a.page_crcs = d_page_crcs;
        a.delta = delta;
        const uint64_t blocks = (a.n_pieces + kLogWaves - 1) / kLogWaves;
        a.blocks = (int)(blocks < (uint64_t)c->cus ? (blocks ? blocks : 1) : (uint64_t)c->cus);
        return a;
    };
    std::unique_lock<std::mutex> lk(c->log_mu);
    hipError_t e;
    DevCtx::LogTable* t = log_table(c.get(), s, 2 * W.table_entries, &e);  // two tables: its halves
    if (e != hipSuccess) return map_err(e);
    if (!t) {  // no engine table for this stream (kMaxTailBlocks streams hold one, or a huge log): one call a batch
        lk.unlock();
        for (uint32_t k = 0; k < n_batches; k++)
            if (batches[k].n_updates &&
                (rc = apply_log(d_pool, pool_bytes, page_bytes, batches[k].d_src, batches[k].d_log, batches[k].n_updates,
                                max_len, d_page_crcs, d_work, W.region, stream, delta)))
                return rc;
        return CC_OK;
    }
    unsigned char* w = static_cast<unsigned char*>(d_work);
    uint64_t* const t0 = reinterpret_cast<uint64_t*>(t->p + kLogTableHeader);
    uint64_t* tabs[2] = {t0, t0 + W.table_entries};
    const uint32_t masks[2] = {(uint32_t)(W.table_entries - 1), (uint32_t)(W.table_entries - 1)};
    // the three chunk counters of the tail groupings: grouping kernel q takes
    // from counter q % 3 and zeroes counter (q + 2) % 3; every insert kernel of
    // the call zeroes all three (one precedes every grouping on the stream)
    unsigned long long* ctrs = reinterpret_cast<unsigned long long*>(w + W.ctr_off);
    uint64_t gq = 0;  // tail groupings so far
    auto region = [&](LogLaunch& a, int r, const SegLayout& l) {
        unsigned char* q = w + (uint64_t)r * W.region;
        a.table = tabs[r];
        a.table_mask = masks[r];
        a.clear_table = 1;  // both tables are left zero for the batch after next
        a.next = reinterpret_cast<uint32_t*>(q);
        a.heads = reinterpret_cast<uint32_t*>(q + W.heads_off);
        a.seg_count = reinterpret_cast<uint32_t*>(q + W.counts_off);
        a.n_segs = l.n_segs;
        a.seg_cap = l.seg_cap;
    };
    int r = 0;             // region (and table) of the batch being applied
    bool grouped = false;  // batch k already grouped (by the page kernel before it)
    SegLayout lay = {};
    for (uint32_t k = 0; k < n_batches && e == hipSuccess; k++) {
        const cc_log_batch& b = batches[k];
        if (b.n_updates == 0) continue;
        LogLaunch a = base(b);
        if (small(b.n_updates)) {
            e = launch_log_small(a, s);
            grouped = false;
            continue;
        }
        if (!grouped) {  // the first batch (or one after a small batch): the insert kernel
            const uint64_t chunks = (a.n_pieces + kInsertThreads - 1) / kInsertThreads;
            if (!seg_layout(a.n_pieces, kInsertThreads, (uint32_t)(chunks < kInsertBlocks ? chunks : kInsertBlocks), &lay)) {
                e = hipErrorInvalidValue;  // (not reached: log_work accepted the largest batch)
                break;
            }
            region(a, r, lay);
            a.zero_ctrs = ctrs;
            if ((e = launch_log_insert(a, s)) != hipSuccess) break;
            a.zero_ctrs = nullptr;
        } else {
            region(a, r, lay);
        }
        // the next non-empty batch, grouped inside this page kernel when it takes the table path
        uint32_t j = k + 1;
        while (j < n_batches && batches[j].n_updates == 0) j++;
        grouped = false;
        if (j < n_batches && !small(batches[j].n_updates)) {
            const LogLaunch nb = base(batches[j]);
            // a workgroup may take up to twice its even share of the chunks, in
            // takes of kGroupTake
            const uint64_t chunks = (nb.n_pieces + T - 1) / T;
            // the grouping writes one head segment per workgroup: at most
            // kInsertBlocks of them, so a device with more CUs runs this page
            // kernel on kInsertBlocks workgroups rather than lose the grouping
            const uint32_t G = a.blocks < (int)kInsertBlocks ? (uint32_t)a.blocks : kInsertBlocks;
            uint64_t rounds = 2 * ((chunks + G - 1) / G);
            rounds = (rounds + kGroupTake - 1) / kGroupTake * kGroupTake;
            SegLayout nl = {G, (uint32_t)(rounds * T)};
            if (rounds * T < (1ull << 32)) {
                a.blocks = (int)G;
                unsigned char* q = w + (uint64_t)(r ^ 1) * W.region;
                a.nx.upd = nb.upd;
                a.nx.n_pieces = nb.n_pieces;
                a.nx.pool_bytes = pool_bytes;
                a.nx.page_bytes = page_bytes;
                a.nx.max_len = max_len;
                a.nx.slots = slots;
                a.nx.table = tabs[r ^ 1];
                a.nx.table_mask = masks[r ^ 1];
                a.nx.next = reinterpret_cast<uint32_t*>(q);
                a.nx.heads = reinterpret_cast<uint32_t*>(q + W.heads_off);
                a.nx.seg_count = reinterpret_cast<uint32_t*>(q + W.counts_off);
                a.nx.seg_cap = nl.seg_cap;
                a.nx.rounds = (uint32_t)rounds;
                a.nx.take = ctrs + gq % 3;
                a.nx.zero = ctrs + (gq + 2) % 3;
                gq++;
                lay = nl;
                grouped = true;
            }
        }
        e = launch_log_pages(a, s);
        r ^= 1;
    }
    if (e != hipSuccess) t->dirty = true;  // a launch may have run in part: clear the engine table before its next use
    return map_err(e);
}

int cc_page_list_probe_dev(const void* d_pool, uint64_t pool_bytes, const uint64_t* d_pages, uint64_t n,
                           uint32_t* d_out, void* stream) {
    if (n == 0) return CC_OK;
    if (!d_pool || !d_pages || !d_out || pool_bytes % 4096 || ((uintptr_t)d_pool & 3u) || ((uintptr_t)d_pages & 7u))
        return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    PageListProbeLaunch a = {};
    a.pool = static_cast<const uint32_t*>(d_pool);
    a.pool_pages = pool_bytes / 4096;
    a.pages = d_pages;
    a.n = n;
    a.out = d_out;
    a.blocks = c->cus;  // one workgroup per CU, as verify-on-read
    hipStream_t s = static_cast<hipStream_t>(stream);
    // the dynamic tail's counter: one slot set of the stream's tail block, as the page kernel's
    {
        std::lock_guard<std::mutex> lk(c->tail_mu);
        if (DevCtx::TailBlock* t = tail_block(c.get(), s)) {
            a.dyn_ctr = t->p + t->parity * kDynCtrWords64;
            a.dyn_next = t->p + (t->parity ^ 1u) * kDynCtrWords64;
            const hipError_t e = launch_page_list_probe(a, s);
            if (e == hipSuccess)
                t->parity ^= 1u;
            else
                t->dirty = true;
            return map_err(e);
        }
    }
    return map_err(launch_page_list_probe(a, s));  // no tail block free: a static split
}

int cc_apply_log_probe_dev(void* d_pool, uint64_t pool_bytes, const void* d_src, const cc_log_probe_desc* d_desc,
                           uint64_t n, uint32_t* d_out, void* stream) {
    static_assert(sizeof(cc_log_probe_desc) == sizeof(LogProbeDesc), "probe descriptor layout");
    if (n == 0) return CC_OK;
    if (!d_pool || !d_src || !d_desc || !d_out || pool_bytes % 4096 || ((uintptr_t)d_pool & 3u) ||
        ((uintptr_t)d_desc & 7u))
        return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    LogProbeLaunch a = {};
    a.pool = static_cast<unsigned char*>(d_pool);
    a.pool_pages = pool_bytes / 4096;
    a.src = static_cast<const unsigned char*>(d_src);
    a.desc = reinterpret_cast<const LogProbeDesc*>(d_desc);
    a.n = n;
    a.out = d_out;
    // the write log's page pass grid: a workgroup per CU, fewer for a short list
    const uint64_t blocks = (n + kLogWavesFull - 1) / kLogWavesFull;
    a.blocks = (int)(blocks < (uint64_t)c->cus ? blocks : (uint64_t)c->cus);
    return map_err(launch_log_probe(a, static_cast<hipStream_t>(stream)));
}

// The engine holds the schedule scratch (the stream's range scratch); d_work is
// kept in the ABI (a caller sized it with this function) and not used.
uint64_t cc_verify_reads_work_bytes(uint64_t n_reads) {
    if (n_reads == 0 || n_reads >= (1ull << 31)) return 0;
    return 256;
}

int cc_verify_reads_dev(const void* d_pool, uint64_t pool_bytes, uint32_t page_bytes, const cc_range* d_reads,
                        uint64_t n_reads, const uint32_t* d_page_crcs, uint32_t* d_bad_per_read, uint64_t* d_bad_total,
                        void* d_work, uint64_t work_bytes, void* stream) {
    if (!log_page_ok(page_bytes)) return CC_EINVAL;
    if (n_reads == 0) return CC_OK;
    if (!d_pool || !d_reads || !d_page_crcs || !d_bad_per_read || !d_bad_total || !d_work) return CC_EINVAL;
    if (pool_bytes % page_bytes || ((uintptr_t)d_pool & 3u)) return CC_EINVAL;
    const uint64_t need = cc_verify_reads_work_bytes(n_reads);
    if (need == 0 || work_bytes < need) return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    ReadVerifyLaunch a = {};
    a.pool = static_cast<const uint32_t*>(d_pool);
    a.pool_bytes = pool_bytes;
    a.page_bytes = page_bytes;
    a.page_shift = (uint32_t)__builtin_ctz(page_bytes);  // a power of two (log_page_ok)
    a.reads = reinterpret_cast<const RangeDesc*>(d_reads);
    a.n_reads = n_reads;
    a.page_crcs = d_page_crcs;
    a.bad_per_read = d_bad_per_read;
    a.bad_total = reinterpret_cast<unsigned long long*>(d_bad_total);
    a.image = c->image;
    a.kconst = kconst_for(page_bytes);
    a.blocks = c->cus;  // every wave takes an equal share of the (device-counted) page slots
    // batches of up to 64 reads take the one-launch small path (page counts summed in
    // 32 bits there: pools of < 2^26 pages keep 64 reads' sum exact)
    if (n_reads <= 64 && pool_bytes / page_bytes < (1ull << 26))
        return map_err(launch_read_verify_small(a, s));
    return map_err(with_range_scratch(c.get(), s, 0,
                                      [&](uint64_t* tiles, unsigned long long* tail, uint32_t*, uint32_t epoch) {
                                          a.tiles = tiles;
                                          a.tail = tail;
                                          a.epoch = epoch;
                                          return launch_read_verify(a, s);
                                      }));
}

// Streaming scan.  Each staging slot holds a batch of whole chunks (data and
// metapages in separate device regions) plus the per-chunk results; a batch is
// {H2D data+meta, page kernel over data, page kernel over metapages, fused
// epilogue (slices, file CRCs, digest contributions), D2H results} on the
// slot's stream, so consecutive batches on the two streams overlap copy and
// compute.  Pinned sources are DMA'd directly, chunk by chunk (a mix of pinned
// and pageable chunks is fine); pageable ones are staged through the slot's
// pinned buffer first.
int cc_scan_host_digest(const cc_chunk_src* chunks, uint64_t n_chunks, uint32_t chunk_bytes, uint32_t meta_bytes,
                        uint32_t page_bytes, uint32_t slice_bytes, uint32_t* h_meta_crcs, uint32_t* h_slice_crcs,
                        uint32_t* h_file_crcs, const cc_scan_digest* dg) {
    if (n_chunks == 0) {
        if (dg && dg->h_digest && dg->n_groups) memset(dg->h_digest, 0, dg->n_groups * 4);
        return CC_OK;
    }
    if (!chunks || !page_size_ok(page_bytes) || !page_size_ok(meta_bytes) || chunk_bytes == 0 ||
        slice_bytes == 0 || chunk_bytes % slice_bytes || slice_bytes % page_bytes)
        return CC_EINVAL;
    // every argument is checked before the first byte moves: a bad chunk or a
    // copyset index outside the digest must not surface half way through
    for (uint64_t i = 0; i < n_chunks; i++)
        if (!chunks[i].data || !chunks[i].meta) return CC_EINVAL;
    if (dg) {
        if (!dg->h_after_bytes || !dg->h_group || !dg->h_digest || dg->n_groups == 0 ||
            dg->n_groups >= (1ull << 32))
            return CC_EINVAL;
        for (uint64_t i = 0; i < n_chunks; i++)
            if (dg->h_group[i] >= dg->n_groups) return CC_EINVAL;
    }
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(c->submit);
    if ((rc = staging_init(c.get()))) return rc;
    Staging& st = c->st;
    SlotRing ring(st);
    const uint64_t per_chunk_dev = (uint64_t)chunk_bytes + meta_bytes;
    const uint64_t batch = st.bytes / per_chunk_dev;
    if (batch == 0) return CC_EINVAL;  // staging smaller than one chunk file
    const uint32_t slices = chunk_bytes / slice_bytes;
    const uint64_t pages_per_chunk = chunk_bytes / page_bytes;
    // per-slot device result region (carved from dcrc, sized per/256*4 bytes):
    // meta [batch] | slices [batch*slices] | file [batch] | data [batch] | page CRCs [batch*pages_per_chunk]
    const uint64_t need_words = batch * pages_per_chunk + batch * (3 + (uint64_t)slices);
    if (need_words * 4 > st.bytes / 256 * 4) return CC_EINVAL;
    const uint32_t k_page = kconst_for(page_bytes), k_meta = kconst_for(meta_bytes);
    FoldLaunch f1 = {}, f2 = {};
    f1.per_group = slice_bytes / page_bytes;
    f1.m_unit = xpow((uint64_t)page_bytes << 3);
    for (int t = 0; t < 6; t++) f1.m_tree[t] = xpow(((uint64_t)page_bytes * (f1.per_group / 64) << t) << 3);
    f2.per_group = slices;
    f2.m_unit = xpow((uint64_t)slice_bytes << 3);
    for (int t = 0; t < 6; t++) f2.m_tree[t] = xpow(((uint64_t)slice_bytes * (slices / 64) << t) << 3);
    const uint32_t m_chunk = xpow((uint64_t)chunk_bytes << 3);
    EpilogueLaunch epi = {};
    const bool use_epi = chunk_bytes % page_bytes == 0 &&
                         epilogue_geometry(c.get(), (uint32_t)pages_per_chunk, page_bytes, slice_bytes / page_bytes,
                                           &epi);
    hipError_t e = hipSuccess;

    // streamed digest: after bytes + copyset index uploaded once, multipliers
    // x^(8*after) computed on the device, accumulator zeroed; both slot streams
    // wait for that before their first epilogue
    uint64_t* d_after = nullptr;
    uint32_t *d_mult = nullptr, *d_group = nullptr, *d_digest = nullptr;
    if (dg) {
        const uint64_t bytes = align256(n_chunks * 8) + 2 * align256(n_chunks * 4) + align256(dg->n_groups * 4);
        if (bytes > st.aux_bytes) {
            if (st.aux) (void)hipFree(st.aux);  // previous calls are drained: not in use
            st.aux = nullptr;
            st.aux_bytes = 0;
            if ((e = hipMalloc(&st.aux, bytes)) != hipSuccess) return map_err(e);
            st.aux_bytes = bytes;
        }
        unsigned char* a = static_cast<unsigned char*>(st.aux);
        d_after = reinterpret_cast<uint64_t*>(a);
        d_mult = reinterpret_cast<uint32_t*>(a + align256(n_chunks * 8));
        d_group = reinterpret_cast<uint32_t*>(a + align256(n_chunks * 8) + align256(n_chunks * 4));
        d_digest = reinterpret_cast<uint32_t*>(a + align256(n_chunks * 8) + 2 * align256(n_chunks * 4));
        hipStream_t s0 = st.stream[0];
        if ((e = hipMemcpyAsync(d_after, dg->h_after_bytes, n_chunks * 8, hipMemcpyHostToDevice, s0)) != hipSuccess ||
            (e = hipMemcpyAsync(d_group, dg->h_group, n_chunks * 4, hipMemcpyHostToDevice, s0)) != hipSuccess ||
            (e = hipMemsetAsync(d_digest, 0, dg->n_groups * 4, s0)) != hipSuccess ||
            (e = launch_xpow8(d_after, n_chunks, d_mult, s0)) != hipSuccess ||
            (e = hipEventRecord(st.aux_ready, s0)) != hipSuccess ||
            (e = hipStreamWaitEvent(st.stream[1], st.aux_ready, 0)) != hipSuccess)
            return ring.fail(map_err(e));
    }

    auto take = [&](int s) {
        return [&, s](uint64_t f, uint64_t nb) {
            const uint32_t* r = st.hcrc[s];
            if (h_meta_crcs) memcpy(h_meta_crcs + f, r, nb * 4);
            if (h_slice_crcs) memcpy(h_slice_crcs + f * slices, r + nb, nb * slices * 4);
            if (h_file_crcs) memcpy(h_file_crcs + f, r + nb + nb * slices, nb * 4);
        };
    };
    int slot = 0;
    for (uint64_t first = 0; first < n_chunks; first += batch) {
        const uint64_t nb = (n_chunks - first < batch) ? n_chunks - first : batch;
        if ((rc = ring.drain(slot, take(slot)))) return rc;  // the slot's staging is free again
        unsigned char* ddata = static_cast<unsigned char*>(st.dev[slot]);
        unsigned char* dmeta = ddata + nb * (uint64_t)chunk_bytes;
        unsigned char* hstage = static_cast<unsigned char*>(st.host[slot]);
        hipStream_t s = st.stream[slot];
        // pageable metapages are staged contiguously and copied as runs
        uint64_t run0 = 0, run_n = 0;
        auto flush_meta_run = [&]() -> hipError_t {
            if (!run_n) return hipSuccess;
            const uint64_t o = nb * (uint64_t)chunk_bytes + run0 * (uint64_t)meta_bytes;
            const hipError_t ee = hipMemcpyAsync(ddata + o, hstage + o, run_n * meta_bytes, hipMemcpyHostToDevice, s);
            run_n = 0;
            return ee;
        };
        for (uint64_t i = 0; i < nb; i++) {
            const cc_chunk_src& cs = chunks[first + i];
            const uint64_t od = i * (uint64_t)chunk_bytes;
            if (is_pinned(cs.data)) {
                e = hipMemcpyAsync(ddata + od, cs.data, chunk_bytes, hipMemcpyHostToDevice, s);
            } else {
                memcpy(hstage + od, cs.data, chunk_bytes);
                e = hipMemcpyAsync(ddata + od, hstage + od, chunk_bytes, hipMemcpyHostToDevice, s);
            }
            if (e != hipSuccess) return ring.fail(map_err(e));
            if (is_pinned(cs.meta)) {
                if ((e = flush_meta_run()) != hipSuccess) return ring.fail(map_err(e));
                e = hipMemcpyAsync(dmeta + i * (uint64_t)meta_bytes, cs.meta, meta_bytes, hipMemcpyHostToDevice, s);
                if (e != hipSuccess) return ring.fail(map_err(e));
            } else {
                memcpy(hstage + nb * (uint64_t)chunk_bytes + i * (uint64_t)meta_bytes, cs.meta, meta_bytes);
                if (!run_n) run0 = i;
                run_n++;
            }
        }
        if ((e = flush_meta_run()) != hipSuccess) return ring.fail(map_err(e));
        // (the copies stay on the slot's stream here: no read gates a batch, and
        // the FIFO copy stream measured 48.7 vs 51.6 GiB/s on the stream leg's
        // per-chunk pinned copies, round 5)
        uint32_t* res = st.dcrc[slot];
        uint32_t* d_pages = res + nb * (3 + (uint64_t)slices);
        uint32_t* d_meta = res;
        uint32_t* d_slices = res + nb;
        uint32_t* d_file = res + nb + nb * slices;
        uint32_t* d_data = d_file + nb;
        PageLaunch a = {};
        a.pages = reinterpret_cast<const uint32_t*>(ddata);
        a.n_pages = nb * pages_per_chunk;
        a.words_per_lane = page_bytes / kWaveBytes;
        a.image = c->image;
        a.kconst = k_page;
        a.out = d_pages;
        geometry_for(c.get(), a.n_pages, &a);
        if ((e = launch_page_crc(a, s)) != hipSuccess) return ring.fail(map_err(e));
        a.pages = reinterpret_cast<const uint32_t*>(dmeta);
        a.n_pages = nb;
        a.words_per_lane = meta_bytes / kWaveBytes;
        a.kconst = k_meta;
        a.out = d_meta;
        geometry_for(c.get(), nb, &a);
        if ((e = launch_page_crc(a, s)) != hipSuccess) return ring.fail(map_err(e));
        if (use_epi) {  // one fused launch: slices + file CRCs (+ digest contributions)
            EpilogueLaunch ea = epi;
            ea.page_crcs = d_pages;
            ea.meta_crcs = d_meta;
            ea.n_chunks = nb;
            ea.slice_crcs = d_slices;
            ea.file_crcs = d_file;
            if (dg) {
                ea.after_mult = d_mult + first;
                ea.group = d_group + first;
                ea.digest = d_digest;
            }
            if ((e = launch_epilogue(ea, s)) != hipSuccess) return ring.fail(map_err(e));
        } else {
            f1.crcs = d_pages;
            f1.n_groups = nb * slices;
            f1.out = d_slices;
            if ((e = launch_fold(f1, s)) != hipSuccess) return ring.fail(map_err(e));
            f2.crcs = d_slices;
            f2.n_groups = nb;
            f2.out = d_data;
            if ((e = launch_fold(f2, s)) != hipSuccess) return ring.fail(map_err(e));
            if ((e = launch_combine(d_meta, d_data, m_chunk, nb, d_file, s)) != hipSuccess)
                return ring.fail(map_err(e));
            if (dg && (e = launch_digest(d_file, d_after + first, d_group + first, nb, d_digest, s)) != hipSuccess)
                return ring.fail(map_err(e));
        }
        if ((e = hipMemcpyAsync(st.hcrc[slot], res, nb * (2 + (uint64_t)slices) * 4, hipMemcpyDeviceToHost, s)) !=
            hipSuccess)
            return ring.fail(map_err(e));
        if ((e = arm_slot(st, slot, s)) != hipSuccess) return ring.fail(map_err(e));
        ring.first[slot] = first;
        ring.n[slot] = nb;
        slot ^= 1;
    }
    if ((rc = ring.drain(slot, take(slot)))) return rc;
    if ((rc = ring.drain(slot ^ 1, take(slot ^ 1)))) return rc;
    if (dg) {  // every epilogue has completed (both slots drained)
        hipStream_t s0 = st.stream[0];
        if ((e = hipMemcpyAsync(st.hcrc[0], d_digest, dg->n_groups * 4 <= st.bytes / 256 * 4 ? dg->n_groups * 4 : 0,
                                hipMemcpyDeviceToHost, s0)) != hipSuccess ||
            (e = hipStreamSynchronize(s0)) != hipSuccess)
            return map_err(e);
        if (dg->n_groups * 4 <= st.bytes / 256 * 4) {
            memcpy(dg->h_digest, st.hcrc[0], dg->n_groups * 4);
        } else if ((e = hipMemcpy(dg->h_digest, d_digest, dg->n_groups * 4, hipMemcpyDeviceToHost)) != hipSuccess) {
            return map_err(e);
        }
    }
    return CC_OK;
}

int cc_scan_host(const cc_chunk_src* chunks, uint64_t n_chunks, uint32_t chunk_bytes, uint32_t meta_bytes,
                 uint32_t page_bytes, uint32_t slice_bytes, uint32_t* h_meta_crcs, uint32_t* h_slice_crcs,
                 uint32_t* h_file_crcs) {
    return cc_scan_host_digest(chunks, n_chunks, chunk_bytes, meta_bytes, page_bytes, slice_bytes, h_meta_crcs,
                               h_slice_crcs, h_file_crcs, nullptr);
}

// Native file scan.  Batch layout in a staging slot = data of the batch's
// files back to back, then their metapages, so one H2D per batch; files that
// fail get status != 0 and their slots are zero-filled (their CRCs are
// discarded).
namespace {
constexpr uint64_t kReadPiece = 2ull << 20;  // io work item

// CPUs this process may run on: the affinity mask, capped by the cgroup v2
// CPU quota (cpu.max) when there is one -- a GPU box hands each GPU a share of
// a larger host, and readers beyond the quota only get throttled.
uint32_t usable_cpus() {
    cpu_set_t set;
    uint32_t n = 0;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = (uint32_t)CPU_COUNT(&set);
    if (n == 0) {
        const long v = sysconf(_SC_NPROCESSORS_ONLN);
        n = v > 0 ? (uint32_t)v : 1u;
    }
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        unsigned long long per = 0;
        if (fscanf(f, "%31s %llu", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0) {
            const unsigned long long quota = strtoull(q, nullptr, 10);
            const uint32_t cap = (uint32_t)(quota / per);  // whole CPUs of quota
            if (cap >= 1 && cap < n) n = cap;
        }
        fclose(f);
    }
    return n;
}

// Default reader count: half the usable CPUs (the HIP runtime's threads and the
// caller need the rest), at least 2, at most kMaxDefaultReaders.
constexpr uint32_t kMaxDefaultReaders = 8;
// Computed per call (an affinity mask set after the first call -- a NUMA
// binding -- counts; the mask and quota reads cost microseconds a batch call).
uint32_t default_io_threads() {
    const uint32_t h = usable_cpus() / 2;
    return h < 2 ? 2u : (h > kMaxDefaultReaders ? kMaxDefaultReaders : h);
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
        if (r == 0) return -EIO;  // short file
        got += (size_t)r;
    }
    return 0;
}
}  // namespace

uint32_t cc_default_io_threads(void) { return default_io_threads(); }

int cc_scan_files(const char* const* paths, uint64_t n_files, uint32_t chunk_bytes, uint32_t meta_bytes,
                  uint32_t page_bytes, uint32_t slice_bytes, uint32_t io_threads, uint32_t* h_slice_crcs,
                  cc_file_result* h_results) {
    if (n_files == 0) return CC_OK;
    if (!paths || !h_results || !page_size_ok(page_bytes) || !page_size_ok(meta_bytes) || chunk_bytes == 0 ||
        slice_bytes == 0 || chunk_bytes % slice_bytes || slice_bytes % page_bytes)
        return CC_EINVAL;
    CtxRef c;
    int rc = get_ctx(&c);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(c->submit);
    if ((rc = staging_init(c.get()))) return rc;
    Staging& st = c->st;
    SlotRing ring(st);
    const uint64_t per_file = (uint64_t)chunk_bytes + meta_bytes;
    const uint64_t batch = st.bytes / per_file;
    if (batch == 0) return CC_EINVAL;
    const uint32_t slices = chunk_bytes / slice_bytes;
    const uint64_t pages_per_chunk = chunk_bytes / page_bytes;
    if (batch * pages_per_chunk + batch * (3 + (uint64_t)slices) > st.bytes / 256) return CC_EINVAL;
    EpilogueLaunch epi = {};
    const bool use_epi =
        epilogue_geometry(c.get(), (uint32_t)pages_per_chunk, page_bytes, slice_bytes / page_bytes, &epi);
    FoldLaunch f1 = {}, f2 = {};
    f1.per_group = slice_bytes / page_bytes;
    f1.m_unit = xpow((uint64_t)page_bytes << 3);
    for (int t = 0; t < 6; t++) f1.m_tree[t] = xpow(((uint64_t)page_bytes * (f1.per_group / 64) << t) << 3);
    f2.per_group = slices;
    f2.m_unit = xpow((uint64_t)slice_bytes << 3);
    for (int t = 0; t < 6; t++) f2.m_tree[t] = xpow(((uint64_t)slice_bytes * (slices / 64) << t) << 3);
    const uint32_t m_chunk = xpow((uint64_t)chunk_bytes << 3);
    const uint32_t threads = io_threads ? (io_threads > 64 ? 64 : io_threads) : default_io_threads();

    auto take = [&](int s) {
        return [&, s](uint64_t f, uint64_t nb) {
            const uint32_t* r = st.hcrc[s];
            for (uint64_t i = 0; i < nb; i++) {
                cc_file_result& fr = h_results[f + i];
                if (fr.status != 0) continue;
                fr.meta_crc = r[i];
                fr.file_crc = r[nb + nb * slices + i];
                if (h_slice_crcs) memcpy(h_slice_crcs + (f + i) * slices, r + nb + i * slices, slices * 4);
            }
        };
    };
    int slot = 0;
    hipError_t e;
    for (uint64_t first = 0; first < n_files; first += batch) {
        const uint64_t nb = (n_files - first < batch) ? n_files - first : batch;
        if ((rc = ring.drain(slot, take(slot)))) return rc;  // slot's previous batch done: its staging is free
        unsigned char* hstage = static_cast<unsigned char*>(st.host[slot]);
        // open + size check serially (cheap), then the reads as ~2 MiB pieces
        // pulled by the io threads (a batch holds only a few 16 MiB files)
        std::vector<int> fds(nb, -1);
        std::vector<std::atomic<int>> fst(nb);
        for (uint64_t i = 0; i < nb; i++) {
            const char* p = paths[first + i];
            int status = 0;
            const int fd = p ? open(p, O_RDONLY | O_CLOEXEC) : -1;
            if (fd < 0) status = p ? -errno : CC_EINVAL;
            struct stat sb;
            if (!status && fstat(fd, &sb) != 0) status = -errno;
            if (!status && (uint64_t)sb.st_size != per_file) status = CC_EFORMAT;  // CSChunkFile::Open's FileFormatError
            fds[i] = fd;
            fst[i].store(status);
        }
        const uint64_t pieces = (chunk_bytes + kReadPiece - 1) / kReadPiece;
        const uint64_t items = nb * (1 + pieces);
        hipStream_t s = st.stream[slot];
        hipStream_t cs = st.copy;  // every H2D of the call, FIFO
        unsigned char* ddata = static_cast<unsigned char*>(st.dev[slot]);
        unsigned char* dmeta = ddata + nb * (uint64_t)chunk_bytes;
        // a file's data goes to the device as soon as its last piece is read
        // (the reader that finishes it enqueues the copy on the FIFO copy
        // stream; the slot's kernels wait for the batch's copies by event), so
        // the DMA starts a file into the batch.  8 native readers alone move
        // 74 GiB/s beside a saturated H2D (scripts/file_read_probe.cpp,
        // profiles/file_read_probe_r05.jsonl): the reads are not the limit, the
        // copy schedule was (scripts/trace_files.py host timelines,
        // profiles/scan_files_trace_r05.txt: whole-batch copies on the two slot
        // streams 37.8 GiB/s; FIFO copy stream 48.0; per-file copies from the
        // readers on it 49.4)
        std::vector<std::atomic<uint32_t>> left(nb);
        for (uint64_t i = 0; i < nb; i++) left[i].store((uint32_t)(1 + pieces));
        std::atomic<int> herr{(int)hipSuccess};
        std::atomic<uint64_t> next{0};
        auto reader = [&]() {
            for (uint64_t it; (it = next.fetch_add(1)) < items;) {
                const uint64_t i = it / (1 + pieces), k = it % (1 + pieces);
                if (!fst[i].load(std::memory_order_relaxed)) {
                    int r;
                    if (k == 0) {
                        r = read_full(fds[i], hstage + nb * (uint64_t)chunk_bytes + i * (uint64_t)meta_bytes,
                                      meta_bytes, 0);
                    } else {
                        const uint64_t off = (k - 1) * kReadPiece;
                        const uint64_t len = chunk_bytes - off < kReadPiece ? chunk_bytes - off : kReadPiece;
                        r = read_full(fds[i], hstage + i * (uint64_t)chunk_bytes + off, len,
                                      (off_t)(meta_bytes + off));
                    }
                    if (r) {
                        int zero = 0;
                        fst[i].compare_exchange_strong(zero, r);
                    }
                }
                // the file's last item: its data (if it was read whole) leaves now
                if (left[i].fetch_sub(1) == 1 && fst[i].load() == 0) {
                    const hipError_t ce = hipMemcpyAsync(ddata + i * (uint64_t)chunk_bytes,
                                                         hstage + i * (uint64_t)chunk_bytes, chunk_bytes,
                                                         hipMemcpyHostToDevice, cs);
                    int ok = (int)hipSuccess;
                    if (ce != hipSuccess) herr.compare_exchange_strong(ok, (int)ce);
                }
            }
        };
        const int dev = c->device;
        c->readers.run((uint32_t)(items < threads ? items : threads), [&](uint32_t k) {
            if (k) (void)hipSetDevice(dev);  // pool threads enqueue copies on this device's stream
            reader();
        });
        for (uint64_t i = 0; i < nb; i++)
            if (fds[i] >= 0) close(fds[i]);  // before any early return below
        if ((e = (hipError_t)herr.load()) != hipSuccess) return ring.fail(map_err(e));
        for (uint64_t i = 0; i < nb; i++) {
            cc_file_result& fr = h_results[first + i];
            fr = cc_file_result{fst[i].load(), 0, 0, 0};
            if (fr.status) {  // keep the batch well-defined; its CRCs are discarded
                memset(hstage + i * (uint64_t)chunk_bytes, 0, chunk_bytes);
                memset(hstage + nb * (uint64_t)chunk_bytes + i * (uint64_t)meta_bytes, 0, meta_bytes);
                if ((e = hipMemcpyAsync(ddata + i * (uint64_t)chunk_bytes, hstage + i * (uint64_t)chunk_bytes,
                                        chunk_bytes, hipMemcpyHostToDevice, cs)) != hipSuccess)
                    return ring.fail(map_err(e));
            }
        }
        // the batch's metapages: one copy
        if ((e = hipMemcpyAsync(dmeta, hstage + nb * (uint64_t)chunk_bytes, nb * (uint64_t)meta_bytes,
                                hipMemcpyHostToDevice, cs)) != hipSuccess ||
            (e = hipEventRecord(st.copied[slot], cs)) != hipSuccess || (e = hipStreamWaitEvent(s, st.copied[slot], 0)) != hipSuccess)
            return ring.fail(map_err(e));
        uint32_t* res = st.dcrc[slot];
        uint32_t* d_pages = res + nb * (3 + (uint64_t)slices);
        uint32_t* d_meta = res;
        uint32_t* d_slices = res + nb;
        uint32_t* d_file = res + nb + nb * slices;
        uint32_t* d_data = d_file + nb;
        PageLaunch a = {};
        a.pages = reinterpret_cast<const uint32_t*>(ddata);
        a.n_pages = nb * pages_per_chunk;
        a.words_per_lane = page_bytes / kWaveBytes;
        a.image = c->image;
        a.kconst = kconst_for(page_bytes);
        a.out = d_pages;
        geometry_for(c.get(), a.n_pages, &a);
        if ((e = launch_page_crc(a, s)) != hipSuccess) return ring.fail(map_err(e));
        a.pages = reinterpret_cast<const uint32_t*>(dmeta);
        a.n_pages = nb;
        a.words_per_lane = meta_bytes / kWaveBytes;
        a.kconst = kconst_for(meta_bytes);
        a.out = d_meta;
        geometry_for(c.get(), nb, &a);
        if ((e = launch_page_crc(a, s)) != hipSuccess) return ring.fail(map_err(e));
        if (use_epi) {
            EpilogueLaunch ea = epi;
            ea.page_crcs = d_pages;
            ea.meta_crcs = d_meta;
            ea.n_chunks = nb;
            ea.slice_crcs = d_slices;
            ea.file_crcs = d_file;
            if ((e = launch_epilogue(ea, s)) != hipSuccess) return ring.fail(map_err(e));
        } else {
            f1.crcs = d_pages;
            f1.n_groups = nb * slices;
            f1.out = d_slices;
            if ((e = launch_fold(f1, s)) != hipSuccess) return ring.fail(map_err(e));
            f2.crcs = d_slices;
            f2.n_groups = nb;
            f2.out = d_data;
            if ((e = launch_fold(f2, s)) != hipSuccess) return ring.fail(map_err(e));
            if ((e = launch_combine(d_meta, d_data, m_chunk, nb, d_file, s)) != hipSuccess)
                return ring.fail(map_err(e));
        }
        if ((e = hipMemcpyAsync(st.hcrc[slot], res, nb * (2 + (uint64_t)slices) * 4, hipMemcpyDeviceToHost, s)) !=
            hipSuccess)
            return ring.fail(map_err(e));
        if ((e = arm_slot(st, slot, s)) != hipSuccess) return ring.fail(map_err(e));
        ring.first[slot] = first;
        ring.n[slot] = nb;
        slot ^= 1;
    }
    if ((rc = ring.drain(slot, take(slot)))) return rc;
    return ring.drain(slot ^ 1, take(slot ^ 1));
}

}  // extern "C"
