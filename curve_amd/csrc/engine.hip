// curve_amd/csrc/engine.hip -- C ABI of the device path: per-device contexts
// (LDS image, CU count, pinned staging), argument checking, error mapping.
//
// Threading: the reference calls its CRC primitive from raft apply threads and
// brpc bthread workers.  Device contexts are created once under a
// mutex; *_dev calls are lock-free after that (they only enqueue).  The
// blocking *_host call serialises on a per-device submission lock.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <errno.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/curve_crc.h"
#include "gf2.h"
#include "kernels.h"

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
};

struct DevCtx {
    bool ready = false;
    int cus = 256;
    void* image = nullptr;
    std::mutex submit;  // serialises *_host calls on this device
    Staging st;
    std::unordered_map<uint64_t, void*> epi_tables;  // epilogue product tables per (page_bytes, q)
    std::unordered_map<void*, uint32_t> work_gen;    // partial-write generation per work buffer
    std::unordered_map<void*, uint64_t> work_pages;
};

std::mutex g_mu;
std::vector<DevCtx*> g_ctx;
cc_opts g_opts = {4096u, 4u << 20, 256ull << 20};

int map_err(hipError_t e) {
    if (e == hipSuccess) return CC_OK;
    if (e == hipErrorOutOfMemory) return CC_ENOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice || e == hipErrorNoBinaryForGpu ||
        e == hipErrorInsufficientDriver)
        return CC_ENODEV;
    return CC_EHIP;
}

// Context of the calling thread's current device, created on first use.
int get_ctx(DevCtx** out) {
    int dev = -1, n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return CC_ENODEV;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return CC_ENODEV;
    std::lock_guard<std::mutex> lk(g_mu);
    if ((int)g_ctx.size() < n) g_ctx.resize(n, nullptr);
    if (!g_ctx[dev]) g_ctx[dev] = new DevCtx();
    DevCtx* c = g_ctx[dev];
    if (!c->ready) {
        hipDeviceProp_t prop;
        hipError_t e = hipGetDeviceProperties(&prop, dev);
        if (e != hipSuccess) return map_err(e);
        c->cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
        std::vector<uint32_t> img(kLdsBytes / 4);
        build_lds_image(img.data());
        e = hipMalloc(&c->image, kLdsBytes);
        if (e != hipSuccess) return map_err(e);
        e = hipMemcpy(c->image, img.data(), kLdsBytes, hipMemcpyHostToDevice);
        if (e != hipSuccess) return map_err(e);
        e = upload_x2k(x2k().t);
        if (e != hipSuccess) return map_err(e);
        static uint32_t xinv[kXinvEntries];
        uint32_t r = xinv_bytes(0);
        for (uint32_t t = 0; t < kXinvEntries; t++, r = div_x8(r)) xinv[t] = r;  // x^(-8t)
        e = upload_xinv(xinv);
        if (e != hipSuccess) return map_err(e);
        c->ready = true;
    }
    *out = c;
    return CC_OK;
}

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
#ifndef CC_MAX_TSHIFT
#define CC_MAX_TSHIFT 6
#endif
    uint32_t ts = CC_MAX_TSHIFT;
    while (ts > 0 && (n_pages >> ts) < waves) ts--;
    const uint64_t tiles = (n_pages + (1ull << ts) - 1) >> ts;
    const uint64_t need = (tiles + kWavesPerBlock - 1) / kWavesPerBlock;
    a->blocks = (int)(need < (uint64_t)c->cus ? (need ? need : 1) : (uint64_t)c->cus);
    a->tile_shift = ts;
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
    }
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

hipError_t arm_slot(Staging& st, int slot, hipStream_t s) {
    hipError_t e = hipEventRecord(st.done[slot], s);
    if (e != hipSuccess) return e;
    SlotSignal& sg = st.sig[slot];
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

hipError_t park_slot(Staging& st, int slot) {
    SlotSignal& sg = st.sig[slot];
    {
        std::unique_lock<std::mutex> lk(sg.m);
        sg.cv.wait(lk, [&] { return sg.fired; });
    }
    return hipEventSynchronize(st.done[slot]);  // already complete: returns its status
}

bool is_pinned(const void* p) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeHost;
}

void staging_free(Staging& st) {
    for (int i = 0; i < 2; i++) {
        if (st.stream[i]) hipStreamSynchronize(st.stream[i]);
        if (st.host[i]) hipHostFree(st.host[i]);
        if (st.dev[i]) hipFree(st.dev[i]);
        if (st.dcrc[i]) hipFree(st.dcrc[i]);
        if (st.hcrc[i]) hipHostFree(st.hcrc[i]);
        if (st.stream[i]) hipStreamDestroy(st.stream[i]);
        if (st.done[i]) hipEventDestroy(st.done[i]);
        st.host[i] = st.dev[i] = nullptr;
        st.dcrc[i] = st.hcrc[i] = nullptr;
        st.stream[i] = nullptr;
        st.done[i] = nullptr;
        st.sig[i].fired = true;
    }
    st.ready = false;
    st.bytes = 0;
}

}  // namespace
}  // namespace cc

using namespace cc;

extern "C" {

const char* cc_version(void) { return "libcurvecrc 0.1 (gfx950)"; }

const char* cc_strerror(int code) {
    switch (code) {
        case CC_OK: return "ok";
        case CC_EINVAL: return "invalid argument";
        case CC_ENODEV: return "no usable HIP device";
        case CC_ENOMEM: return "out of memory";
        case CC_EHIP: return "HIP runtime error";
        case CC_ECORRUPT: return "checksum mismatch";
        case CC_ECOMM: return "RCCL communication error";
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
    DevCtx* c = nullptr;
    int rc = get_ctx(&c);
    if (rc) return rc;
    return map_err(launch_read_probe(d_buf, bytes, d_sink, 2 * c->cus, static_cast<hipStream_t>(stream)));
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
    DevCtx* c = nullptr;
    return get_ctx(&c);
}

int cc_engine_fini(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    int cur = -1;
    (void)hipGetDevice(&cur);
    for (size_t d = 0; d < g_ctx.size(); d++) {
        DevCtx* c = g_ctx[d];
        if (!c) continue;
        if (hipSetDevice((int)d) == hipSuccess) {
            staging_free(c->st);
            if (c->image) hipFree(c->image);
            for (auto& kv : c->epi_tables)
                if (kv.second) hipFree(kv.second);
        }
        delete c;
        g_ctx[d] = nullptr;
    }
    if (cur >= 0) (void)hipSetDevice(cur);
    return CC_OK;
}

int cc_page_crc_dev(const void* d_pages, uint64_t n_pages, uint32_t page_bytes, uint32_t* d_out, void* stream) {
    if (!page_size_ok(page_bytes)) return CC_EINVAL;
    if (n_pages == 0) return CC_OK;
    if (!d_pages || !d_out || ((uintptr_t)d_pages & 3u)) return CC_EINVAL;
    DevCtx* c = nullptr;
    int rc = get_ctx(&c);
    if (rc) return rc;
    PageLaunch a = {};
    a.pages = static_cast<const uint32_t*>(d_pages);
    a.n_pages = n_pages;
    a.words_per_lane = page_bytes / kWaveBytes;
    a.image = c->image;
    a.kconst = kconst_for(page_bytes);
    a.out = d_out;
    geometry_for(c, n_pages, &a);
    return map_err(launch_page_crc(a, static_cast<hipStream_t>(stream)));
}

int cc_page_verify_list_dev(const void* d_pages, uint64_t n_pages, uint32_t page_bytes, const uint32_t* d_expected,
                            uint64_t* d_bad_count, uint64_t* d_first_bad, uint64_t* d_bad_pages,
                            uint64_t max_bad_pages, void* stream) {
    if (!page_size_ok(page_bytes)) return CC_EINVAL;
    if (n_pages == 0) return CC_OK;
    if (!d_pages || !d_expected || !d_bad_count || !d_first_bad || ((uintptr_t)d_pages & 3u)) return CC_EINVAL;
    if (max_bad_pages && !d_bad_pages) return CC_EINVAL;
    DevCtx* c = nullptr;
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
    geometry_for(c, n_pages, &a);
    return map_err(launch_page_verify(a, static_cast<hipStream_t>(stream)));
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
    DevCtx* c = nullptr;
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
    DevCtx* c = nullptr;
    int rc = get_ctx(&c);
    if (rc) return rc;
    return map_err(launch_shift(d_crcs, d_shift_bytes, n, d_out, static_cast<hipStream_t>(stream)));
}

int cc_crc_ranges_dev(const void* d_buf, const cc_range* d_ranges, uint64_t n, uint32_t* d_out, void* stream) {
    if (n == 0) return CC_OK;
    if (!d_buf || !d_ranges || !d_out) return CC_EINVAL;
    DevCtx* c = nullptr;
    int rc = get_ctx(&c);
    if (rc) return rc;
#ifndef CC_RANGE_GRID_MULT
#define CC_RANGE_GRID_MULT 1  // workgroups per CU launched for a range batch (> 1: hardware re-balances waves)
#endif
    const uint64_t need = (n + kWavesPerBlock - 1) / kWavesPerBlock;
    const uint64_t cap = (uint64_t)c->cus * CC_RANGE_GRID_MULT;
    const int blocks = (int)(need < cap ? need : cap);
    return map_err(launch_range_crc(static_cast<const unsigned char*>(d_buf),
                                    reinterpret_cast<const RangeDesc*>(d_ranges), n, c->image, d_out, blocks,
                                    static_cast<hipStream_t>(stream)));
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
    // (page_bytes, q) and kept on the device
    const uint64_t key = ((uint64_t)page_bytes << 32) | q;
    std::lock_guard<std::mutex> lk(g_mu);
    void*& dev = c->epi_tables[key];
    if (!dev) {
        uint32_t m[10];
        m[0] = xpow((uint64_t)page_bytes << 3);
        for (int k = 0; k < 8; k++) m[1 + k] = xpow(((uint64_t)page_bytes * q << k) << 3);
        m[9] = xpow((uint64_t)pages_per_chunk * page_bytes << 3);
        std::vector<uint32_t> h(10 * 1024);
        for (int t = 0; t < 10; t++)
            for (uint32_t k = 0; k < 4; k++)
                for (uint32_t b = 0; b < 256; b++) h[t * 1024 + k * 256 + b] = mulmod(m[t], b << (8 * k));
        if (hipMalloc(&dev, h.size() * 4) != hipSuccess) {
            dev = nullptr;
            return false;
        }
        if (hipMemcpy(dev, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
            hipFree(dev);  // never leave a half-initialised table in the cache
            dev = nullptr;
            return false;
        }
    }
    a->mtab = static_cast<const uint32_t*>(dev);
    return true;
}
}  // namespace
}  // namespace cc

int cc_xpow8_dev(const uint64_t* d_nbytes, uint64_t n, uint32_t* d_out, void* stream) {
    if (n == 0) return CC_OK;
    if (!d_nbytes || !d_out) return CC_EINVAL;
    DevCtx* c = nullptr;
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
    DevCtx* c = nullptr;
    int rc = get_ctx(&c);
    if (rc) return rc;
    EpilogueLaunch a = {};
    if (!epilogue_geometry(c, pages_per_chunk, page_bytes, pages_per_slice, &a)) return CC_EINVAL;
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
    DevCtx* c = nullptr;
    int rc = get_ctx(&c);
    if (rc) return rc;
    return map_err(launch_combine(d_a, d_b, xpow(len_b << 3), n, d_out, static_cast<hipStream_t>(stream)));
}

int cc_digest_dev(const uint32_t* d_file_crcs, const uint64_t* d_after_bytes, const uint32_t* d_group,
                  uint64_t n_files, uint32_t* d_digest, void* stream) {
    if (n_files == 0) return CC_OK;
    if (!d_file_crcs || !d_after_bytes || !d_group || !d_digest) return CC_EINVAL;
    DevCtx* c = nullptr;
    int rc = get_ctx(&c);
    if (rc) return rc;
    return map_err(launch_digest(d_file_crcs, d_after_bytes, d_group, n_files, d_digest,
                                 static_cast<hipStream_t>(stream)));
}

// Host in / host out.  Two-slot pipeline: while slot i's pages are copied in
// and hashed on stream i, the CPU fills slot i^1 (pageable input) or -- when
// the caller's buffer is already pinned (chunk files pread into pinned memory)
// -- the DMA reads it directly.
int cc_page_crc_host(const void* h_pages, uint64_t n_pages, uint32_t page_bytes, uint32_t* h_out) {
    if (!page_size_ok(page_bytes)) return CC_EINVAL;
    if (n_pages == 0) return CC_OK;
    if (!h_pages || !h_out) return CC_EINVAL;
    DevCtx* c = nullptr;
    int rc = get_ctx(&c);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(c->submit);
    if ((rc = staging_init(c))) return rc;
    Staging& st = c->st;
    const bool pinned = is_pinned(h_pages);
    const uint64_t per_slot = st.bytes / page_bytes;
    const unsigned char* src = static_cast<const unsigned char*>(h_pages);
    uint64_t done = 0;
    uint64_t pending_first[2] = {0, 0}, pending_n[2] = {0, 0};
    int slot = 0;
    hipError_t e = hipSuccess;
    while (done < n_pages) {
        const uint64_t n = (n_pages - done < per_slot) ? n_pages - done : per_slot;
        // reclaim this slot: wait for its previous batch and copy its CRCs out
        if (pending_n[slot]) {
            if ((e = park_slot(st, slot)) != hipSuccess) return map_err(e);
            memcpy(h_out + pending_first[slot], st.hcrc[slot], pending_n[slot] * 4);
            pending_n[slot] = 0;
        }
        const void* hsrc = src + done * page_bytes;
        if (!pinned) {
            memcpy(st.host[slot], hsrc, n * page_bytes);
            hsrc = st.host[slot];
        }
        if ((e = hipMemcpyAsync(st.dev[slot], hsrc, n * page_bytes, hipMemcpyHostToDevice, st.stream[slot])) !=
            hipSuccess)
            return map_err(e);
        PageLaunch a = {};
        a.pages = static_cast<const uint32_t*>(st.dev[slot]);
        a.n_pages = n;
        a.words_per_lane = page_bytes / kWaveBytes;
        a.image = c->image;
        a.kconst = kconst_for(page_bytes);
        a.out = st.dcrc[slot];
        geometry_for(c, n, &a);
        if ((e = launch_page_crc(a, st.stream[slot])) != hipSuccess) return map_err(e);
        if ((e = hipMemcpyAsync(st.hcrc[slot], st.dcrc[slot], n * 4, hipMemcpyDeviceToHost, st.stream[slot])) !=
            hipSuccess)
            return map_err(e);
        if ((e = arm_slot(st, slot, st.stream[slot])) != hipSuccess) return map_err(e);
        pending_first[slot] = done;
        pending_n[slot] = n;
        done += n;
        slot ^= 1;
    }
    for (int k = 0; k < 2; k++) {
        if (!pending_n[slot]) {
            slot ^= 1;
            continue;
        }
        if ((e = park_slot(st, slot)) != hipSuccess) return map_err(e);
        memcpy(h_out + pending_first[slot], st.hcrc[slot], pending_n[slot] * 4);
        pending_n[slot] = 0;
        slot ^= 1;
    }
    return CC_OK;
}

uint64_t cc_update_work_bytes(uint64_t n_pages, uint64_t n_updates, uint32_t max_len, uint32_t page_bytes) {
    (void)n_updates;
    (void)max_len;
    if (page_bytes == 0) return 0;
    return (n_pages * 4 + 255) & ~255ull;  // one generation tag per page
}

int cc_apply_updates_dev(void* d_pool, uint64_t pool_bytes, uint32_t page_bytes, const void* d_src,
                         const cc_update* d_updates, uint64_t n_updates, const uint64_t* h_batch_ends,
                         uint32_t n_batches, uint32_t max_len, uint32_t* d_page_crcs, void* d_work,
                         uint64_t work_bytes, void* stream) {
    if (!page_size_ok(page_bytes) || page_bytes / kWaveBytes > 32) return CC_EINVAL;
    if (n_updates == 0) return CC_OK;
    if (!d_pool || !d_src || !d_updates || !d_page_crcs || !d_work || max_len == 0) return CC_EINVAL;
    if (pool_bytes % page_bytes || ((uintptr_t)d_pool & 3u) || ((uintptr_t)d_src & 3u)) return CC_EINVAL;
    const uint64_t n_pages = pool_bytes / page_bytes;
    if (work_bytes < cc_update_work_bytes(n_pages, n_updates, max_len, page_bytes)) return CC_EINVAL;
    DevCtx* c = nullptr;
    int rc = get_ctx(&c);
    if (rc) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e;
    // generation tags: a work buffer seen for the first time (or after 2^32-1
    // calls) is zeroed once; afterwards each call just bumps its tag
    uint32_t gen;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        uint32_t& g = c->work_gen[d_work];
        if (g == 0 || g == 0xFFFFFFFFu || c->work_pages[d_work] != n_pages) {
            if ((e = hipMemsetAsync(d_work, 0, n_pages * 4, s)) != hipSuccess) return map_err(e);
            g = 0;
            c->work_pages[d_work] = n_pages;
        }
        gen = ++g;
    }
    UpdateLaunch a = {};
    a.pool = static_cast<unsigned char*>(d_pool);
    a.src = static_cast<const unsigned char*>(d_src);
    a.upd = reinterpret_cast<const UpdateDesc*>(d_updates);
    a.n_updates = n_updates;
    a.page_bytes = page_bytes;
    a.flags = static_cast<uint32_t*>(d_work);
    a.gen = gen;
    a.n_pages = n_pages;
    a.image = c->image;
    a.kconst = kconst_for(page_bytes);
    a.page_crcs = d_page_crcs;
    const uint64_t tiles = (n_pages + 63) / 64;
    const uint64_t need = (tiles + kWavesPerBlock - 1) / kWavesPerBlock;
    a.blocks = (int)(need < (uint64_t)c->cus ? (need ? need : 1) : (uint64_t)c->cus);
    // batches in order (stream-ordered kernels), then ONE recompute pass
    uint64_t first = 0;
    const uint32_t nb = h_batch_ends ? n_batches : 1u;
    for (uint32_t b = 0; b < nb; b++) {
        const uint64_t last = h_batch_ends ? h_batch_ends[b] : n_updates;
        if (last < first || last > n_updates) return CC_EINVAL;
        UpdateLaunch ab = a;
        ab.upd = a.upd + first;
        ab.n_updates = last - first;
        if ((e = launch_apply_updates(ab, s)) != hipSuccess) return map_err(e);
        first = last;
    }
    if (first != n_updates) return CC_EINVAL;
    return map_err(launch_page_list_crc(a, s));
}

namespace {
inline bool log_page_ok(uint32_t page_bytes) {
    const uint32_t m = page_bytes / kWaveBytes;
    return page_bytes % kWaveBytes == 0 && m >= 1 && m <= 32 && (m & (m - 1)) == 0;
}
inline uint32_t log_slots(uint32_t max_len, uint32_t page_bytes) { return (max_len - 1) / page_bytes + 2; }
inline uint64_t align256(uint64_t x) { return (x + 255) & ~255ull; }
}  // namespace

uint64_t cc_apply_log_work_bytes(uint64_t n_updates, uint32_t max_len, uint32_t page_bytes) {
    if (!log_page_ok(page_bytes) || max_len == 0 || n_updates == 0) return 0;
    const uint64_t nk = n_updates * log_slots(max_len, page_bytes);
    if (nk >= (1ull << 31)) return 0;
    const size_t temp = log_sort_temp_bytes(nk);
    if (!temp) return 0;
    return 5 * align256(nk * 4) + 256 + align256(temp);
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
    if (n_pages >= kNoPiece) return CC_EINVAL;  // page index must fit a 32-bit key below kNoPiece
    const uint64_t need = cc_apply_log_work_bytes(n_updates, max_len, page_bytes);
    if (need == 0 || work_bytes < need) return CC_EINVAL;
    DevCtx* c = nullptr;
    int rc = get_ctx(&c);
    if (rc) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    LogLaunch a = {};
    a.pool = static_cast<unsigned char*>(d_pool);
    a.pool_bytes = pool_bytes;
    a.src = static_cast<const unsigned char*>(d_src);
    a.upd = reinterpret_cast<const UpdateDesc*>(d_log);
    a.n_updates = n_updates;
    a.page_bytes = page_bytes;
    a.max_len = max_len;
    a.slots = log_slots(max_len, page_bytes);
    const uint64_t nk = n_updates * a.slots;
    unsigned char* w = static_cast<unsigned char*>(d_work);
    a.keys = reinterpret_cast<uint32_t*>(w);
    uint32_t* skeys = reinterpret_cast<uint32_t*>(w + align256(nk * 4));
    a.vals = reinterpret_cast<uint32_t*>(w + 2 * align256(nk * 4));
    uint32_t* svals = reinterpret_cast<uint32_t*>(w + 3 * align256(nk * 4));
    a.heads = reinterpret_cast<uint32_t*>(w + 4 * align256(nk * 4));
    a.head_count = reinterpret_cast<uint32_t*>(w + 5 * align256(nk * 4));
    void* temp = w + 5 * align256(nk * 4) + 256;
    a.skeys = skeys;
    a.svals = svals;
    a.n_keys = nk;
    a.image = c->image;
    a.kconst = kconst_for(page_bytes);
    a.page_crcs = d_page_crcs;
    a.delta = delta;
    // sort only the bits a page index can have, + 1 so kNoPiece sorts last
    int end_bit = 1;
    while (end_bit < 32 && (1ull << end_bit) < n_pages) end_bit++;
    if (end_bit < 32) end_bit++;
    // at most n_keys page runs: a wave per run up to one 8-wave block per CU
    const uint64_t blocks = (nk + kLogWaves - 1) / kLogWaves;
    a.blocks = (int)(blocks < (uint64_t)c->cus ? (blocks ? blocks : 1) : (uint64_t)c->cus);
    hipError_t e;
    if ((e = launch_log_expand(a, s)) != hipSuccess) return map_err(e);
    if ((e = log_sort(temp, work_bytes - 5 * align256(nk * 4) - 256, a.keys, skeys, a.vals, svals, nk, end_bit,
                      s)) != hipSuccess)
        return map_err(e);
    if ((e = launch_log_heads(a, s)) != hipSuccess) return map_err(e);
    return map_err(launch_log_pages(a, s));
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

uint64_t cc_verify_reads_work_bytes(uint64_t n_reads) {
    if (n_reads == 0 || n_reads >= (1ull << 31)) return 0;
    const size_t temp = scan_temp_bytes(n_reads);
    if (!temp) return 0;
    return 2 * align256(n_reads * 8) + align256(temp);
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
    DevCtx* c = nullptr;
    int rc = get_ctx(&c);
    if (rc) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    unsigned char* w = static_cast<unsigned char*>(d_work);
    ReadVerifyLaunch a = {};
    a.pool = static_cast<const uint32_t*>(d_pool);
    a.pool_bytes = pool_bytes;
    a.page_bytes = page_bytes;
    a.reads = reinterpret_cast<const RangeDesc*>(d_reads);
    a.n_reads = n_reads;
    a.counts = reinterpret_cast<uint64_t*>(w);
    a.start = reinterpret_cast<uint64_t*>(w + align256(n_reads * 8));
    void* temp = w + 2 * align256(n_reads * 8);
    a.page_crcs = d_page_crcs;
    a.bad_per_read = d_bad_per_read;
    a.bad_total = reinterpret_cast<unsigned long long*>(d_bad_total);
    a.image = c->image;
    a.kconst = kconst_for(page_bytes);
    a.blocks = c->cus;  // every wave takes an equal share of the (device-computed) page slots
    hipError_t e;
    if ((e = launch_read_counts(a, s)) != hipSuccess) return map_err(e);
    if ((e = exclusive_scan_u64(temp, work_bytes - 2 * align256(n_reads * 8), a.counts, a.start, n_reads, s)) !=
        hipSuccess)
        return map_err(e);
    return map_err(launch_read_verify(a, s));
}

// Streaming scan.  Each staging slot holds a batch of whole chunks (data and
// metapages in separate device regions) plus the per-chunk results; a batch is
// {H2D data+meta, page kernel over data, page kernel over metapages, fold to
// slices, fold to chunk data CRC, combine to file CRC, D2H results} on the
// slot's stream, so consecutive batches on the two streams overlap copy and
// compute.
int cc_scan_host(const cc_chunk_src* chunks, uint64_t n_chunks, uint32_t chunk_bytes, uint32_t meta_bytes,
                 uint32_t page_bytes, uint32_t slice_bytes, uint32_t* h_meta_crcs, uint32_t* h_slice_crcs,
                 uint32_t* h_file_crcs) {
    if (n_chunks == 0) return CC_OK;
    if (!chunks || !page_size_ok(page_bytes) || !page_size_ok(meta_bytes) || chunk_bytes == 0 ||
        slice_bytes == 0 || chunk_bytes % slice_bytes || slice_bytes % page_bytes)
        return CC_EINVAL;
    DevCtx* c = nullptr;
    int rc = get_ctx(&c);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(c->submit);
    if ((rc = staging_init(c))) return rc;
    Staging& st = c->st;
    const uint64_t per_chunk_dev = (uint64_t)chunk_bytes + meta_bytes;
    const uint64_t batch = st.bytes / per_chunk_dev;
    if (batch == 0) return CC_EINVAL;  // staging smaller than one chunk file
    const uint32_t slices = chunk_bytes / slice_bytes;
    const uint64_t pages_per_chunk = chunk_bytes / page_bytes;
    // per-slot device result region (carved from dcrc, sized per/256*4 bytes):
    // page CRCs [batch*pages_per_chunk] | meta [batch] | slices [batch*slices] | data [batch] | file [batch]
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
                         epilogue_geometry(c, (uint32_t)pages_per_chunk, page_bytes, slice_bytes / page_bytes, &epi);

    const bool pinned0 = is_pinned(chunks[0].data) && is_pinned(chunks[0].meta);
    uint64_t pend_first[2] = {0, 0}, pend_n[2] = {0, 0};
    hipError_t e = hipSuccess;
    auto drain = [&](int s) -> int {
        if (!pend_n[s]) return CC_OK;
        hipError_t ee = park_slot(st, s);
        if (ee != hipSuccess) return map_err(ee);
        const uint32_t* r = st.hcrc[s];
        const uint64_t nb = pend_n[s], f = pend_first[s];
        const uint32_t* rm = r;
        const uint32_t* rs = r + nb;
        const uint32_t* rf = r + nb + nb * slices;
        if (h_meta_crcs) memcpy(h_meta_crcs + f, rm, nb * 4);
        if (h_slice_crcs) memcpy(h_slice_crcs + f * slices, rs, nb * slices * 4);
        if (h_file_crcs) memcpy(h_file_crcs + f, rf, nb * 4);
        pend_n[s] = 0;
        return CC_OK;
    };
    int slot = 0;
    for (uint64_t first = 0; first < n_chunks; first += batch) {
        const uint64_t nb = (n_chunks - first < batch) ? n_chunks - first : batch;
        if ((rc = drain(slot))) return rc;
        unsigned char* ddata = static_cast<unsigned char*>(st.dev[slot]);
        unsigned char* dmeta = ddata + nb * (uint64_t)chunk_bytes;
        unsigned char* hstage = static_cast<unsigned char*>(st.host[slot]);
        hipStream_t s = st.stream[slot];
        for (uint64_t i = 0; i < nb; i++) {
            const cc_chunk_src& cs = chunks[first + i];
            if (!cs.data || !cs.meta) return CC_EINVAL;
            const void* sd = cs.data;
            const void* sm = cs.meta;
            if (!pinned0) {
                memcpy(hstage + i * (uint64_t)chunk_bytes, cs.data, chunk_bytes);
                memcpy(hstage + nb * (uint64_t)chunk_bytes + i * (uint64_t)meta_bytes, cs.meta, meta_bytes);
                continue;
            }
            if ((e = hipMemcpyAsync(ddata + i * (uint64_t)chunk_bytes, sd, chunk_bytes, hipMemcpyHostToDevice, s)) !=
                hipSuccess)
                return map_err(e);
            if ((e = hipMemcpyAsync(dmeta + i * (uint64_t)meta_bytes, sm, meta_bytes, hipMemcpyHostToDevice, s)) !=
                hipSuccess)
                return map_err(e);
        }
        if (!pinned0 && (e = hipMemcpyAsync(ddata, hstage, nb * per_chunk_dev, hipMemcpyHostToDevice, s)) != hipSuccess)
            return map_err(e);
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
        geometry_for(c, a.n_pages, &a);
        if ((e = launch_page_crc(a, s)) != hipSuccess) return map_err(e);
        a.pages = reinterpret_cast<const uint32_t*>(dmeta);
        a.n_pages = nb;
        a.words_per_lane = meta_bytes / kWaveBytes;
        a.kconst = k_meta;
        a.out = d_meta;
        geometry_for(c, nb, &a);
        if ((e = launch_page_crc(a, s)) != hipSuccess) return map_err(e);
        if (use_epi) {  // one fused launch: slices + file CRCs
            EpilogueLaunch ea = epi;
            ea.page_crcs = d_pages;
            ea.meta_crcs = d_meta;
            ea.n_chunks = nb;
            ea.slice_crcs = d_slices;
            ea.file_crcs = d_file;
            if ((e = launch_epilogue(ea, s)) != hipSuccess) return map_err(e);
        } else {
            f1.crcs = d_pages;
            f1.n_groups = nb * slices;
            f1.out = d_slices;
            if ((e = launch_fold(f1, s)) != hipSuccess) return map_err(e);
            f2.crcs = d_slices;
            f2.n_groups = nb;
            f2.out = d_data;
            if ((e = launch_fold(f2, s)) != hipSuccess) return map_err(e);
            if ((e = launch_combine(d_meta, d_data, m_chunk, nb, d_file, s)) != hipSuccess) return map_err(e);
        }
        if ((e = hipMemcpyAsync(st.hcrc[slot], res, nb * (2 + (uint64_t)slices) * 4, hipMemcpyDeviceToHost, s)) !=
            hipSuccess)
            return map_err(e);
        if ((e = arm_slot(st, slot, s)) != hipSuccess) return map_err(e);
        pend_first[slot] = first;
        pend_n[slot] = nb;
        slot ^= 1;
    }
    if ((rc = drain(slot))) return rc;
    if ((rc = drain(slot ^ 1))) return rc;
    return CC_OK;
}

// Native file scan.  Batch layout in a staging slot = the pageable layout of
// cc_scan_host (data of the batch's files back to back, then their metapages),
// so one H2D per batch; files that fail get status != 0 and their slots are
// zero-filled (their CRCs are discarded).
namespace {
constexpr uint64_t kReadPiece = 2ull << 20;  // io work item

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

int cc_scan_files(const char* const* paths, uint64_t n_files, uint32_t chunk_bytes, uint32_t meta_bytes,
                  uint32_t page_bytes, uint32_t slice_bytes, uint32_t io_threads, uint32_t* h_slice_crcs,
                  cc_file_result* h_results) {
    if (n_files == 0) return CC_OK;
    if (!paths || !h_results || !page_size_ok(page_bytes) || !page_size_ok(meta_bytes) || chunk_bytes == 0 ||
        slice_bytes == 0 || chunk_bytes % slice_bytes || slice_bytes % page_bytes)
        return CC_EINVAL;
    DevCtx* c = nullptr;
    int rc = get_ctx(&c);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(c->submit);
    if ((rc = staging_init(c))) return rc;
    Staging& st = c->st;
    const uint64_t per_file = (uint64_t)chunk_bytes + meta_bytes;
    const uint64_t batch = st.bytes / per_file;
    if (batch == 0) return CC_EINVAL;
    const uint32_t slices = chunk_bytes / slice_bytes;
    const uint64_t pages_per_chunk = chunk_bytes / page_bytes;
    if (batch * pages_per_chunk + batch * (3 + (uint64_t)slices) > st.bytes / 256) return CC_EINVAL;
    EpilogueLaunch epi = {};
    const bool use_epi = epilogue_geometry(c, (uint32_t)pages_per_chunk, page_bytes, slice_bytes / page_bytes, &epi);
    FoldLaunch f1 = {}, f2 = {};
    f1.per_group = slice_bytes / page_bytes;
    f1.m_unit = xpow((uint64_t)page_bytes << 3);
    for (int t = 0; t < 6; t++) f1.m_tree[t] = xpow(((uint64_t)page_bytes * (f1.per_group / 64) << t) << 3);
    f2.per_group = slices;
    f2.m_unit = xpow((uint64_t)slice_bytes << 3);
    for (int t = 0; t < 6; t++) f2.m_tree[t] = xpow(((uint64_t)slice_bytes * (slices / 64) << t) << 3);
    const uint32_t m_chunk = xpow((uint64_t)chunk_bytes << 3);
    const uint32_t threads = io_threads ? (io_threads > 64 ? 64 : io_threads) : 8;

    uint64_t pend_first[2] = {0, 0}, pend_n[2] = {0, 0};
    auto drain = [&](int s) -> int {
        if (!pend_n[s]) return CC_OK;
        hipError_t ee = park_slot(st, s);
        if (ee != hipSuccess) return map_err(ee);
        const uint32_t* r = st.hcrc[s];
        const uint64_t nb = pend_n[s], f = pend_first[s];
        for (uint64_t i = 0; i < nb; i++) {
            cc_file_result& fr = h_results[f + i];
            if (fr.status != 0) continue;
            fr.meta_crc = r[i];
            fr.file_crc = r[nb + nb * slices + i];
            if (h_slice_crcs) memcpy(h_slice_crcs + (f + i) * slices, r + nb + i * slices, slices * 4);
        }
        pend_n[s] = 0;
        return CC_OK;
    };
    int slot = 0;
    hipError_t e;
    for (uint64_t first = 0; first < n_files; first += batch) {
        const uint64_t nb = (n_files - first < batch) ? n_files - first : batch;
        if ((rc = drain(slot))) return rc;  // slot's previous batch done: its staging is free
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
            if (!status && (uint64_t)sb.st_size != per_file) status = CC_EINVAL;
            fds[i] = fd;
            fst[i].store(status);
        }
        const uint64_t pieces = (chunk_bytes + kReadPiece - 1) / kReadPiece;
        const uint64_t items = nb * (1 + pieces);
        std::atomic<uint64_t> next{0};
        auto reader = [&]() {
            for (uint64_t it; (it = next.fetch_add(1)) < items;) {
                const uint64_t i = it / (1 + pieces), k = it % (1 + pieces);
                if (fst[i].load(std::memory_order_relaxed)) continue;
                int r;
                if (k == 0) {
                    r = read_full(fds[i], hstage + nb * (uint64_t)chunk_bytes + i * (uint64_t)meta_bytes, meta_bytes, 0);
                } else {
                    const uint64_t off = (k - 1) * kReadPiece;
                    const uint64_t len = chunk_bytes - off < kReadPiece ? chunk_bytes - off : kReadPiece;
                    r = read_full(fds[i], hstage + i * (uint64_t)chunk_bytes + off, len, (off_t)(meta_bytes + off));
                }
                if (r) {
                    int zero = 0;
                    fst[i].compare_exchange_strong(zero, r);
                }
            }
        };
        {
            std::vector<std::thread> pool;
            const uint32_t nt = (uint32_t)(items < threads ? items : threads);
            for (uint32_t t = 1; t < nt; t++) pool.emplace_back(reader);
            reader();
            for (auto& th : pool) th.join();
        }
        for (uint64_t i = 0; i < nb; i++) {
            if (fds[i] >= 0) close(fds[i]);
            cc_file_result& fr = h_results[first + i];
            fr = cc_file_result{fst[i].load(), 0, 0, 0};
            if (fr.status) {  // keep the batch well-defined; its CRCs are discarded
                memset(hstage + i * (uint64_t)chunk_bytes, 0, chunk_bytes);
                memset(hstage + nb * (uint64_t)chunk_bytes + i * (uint64_t)meta_bytes, 0, meta_bytes);
            }
        }
        hipStream_t s = st.stream[slot];
        unsigned char* ddata = static_cast<unsigned char*>(st.dev[slot]);
        unsigned char* dmeta = ddata + nb * (uint64_t)chunk_bytes;
        if ((e = hipMemcpyAsync(ddata, hstage, nb * per_file, hipMemcpyHostToDevice, s)) != hipSuccess)
            return map_err(e);
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
        geometry_for(c, a.n_pages, &a);
        if ((e = launch_page_crc(a, s)) != hipSuccess) return map_err(e);
        a.pages = reinterpret_cast<const uint32_t*>(dmeta);
        a.n_pages = nb;
        a.words_per_lane = meta_bytes / kWaveBytes;
        a.kconst = kconst_for(meta_bytes);
        a.out = d_meta;
        geometry_for(c, nb, &a);
        if ((e = launch_page_crc(a, s)) != hipSuccess) return map_err(e);
        if (use_epi) {
            EpilogueLaunch ea = epi;
            ea.page_crcs = d_pages;
            ea.meta_crcs = d_meta;
            ea.n_chunks = nb;
            ea.slice_crcs = d_slices;
            ea.file_crcs = d_file;
            if ((e = launch_epilogue(ea, s)) != hipSuccess) return map_err(e);
        } else {
            f1.crcs = d_pages;
            f1.n_groups = nb * slices;
            f1.out = d_slices;
            if ((e = launch_fold(f1, s)) != hipSuccess) return map_err(e);
            f2.crcs = d_slices;
            f2.n_groups = nb;
            f2.out = d_data;
            if ((e = launch_fold(f2, s)) != hipSuccess) return map_err(e);
            if ((e = launch_combine(d_meta, d_data, m_chunk, nb, d_file, s)) != hipSuccess) return map_err(e);
        }
        if ((e = hipMemcpyAsync(st.hcrc[slot], res, nb * (2 + (uint64_t)slices) * 4, hipMemcpyDeviceToHost, s)) !=
            hipSuccess)
            return map_err(e);
        if ((e = arm_slot(st, slot, s)) != hipSuccess) return map_err(e);
        pend_first[slot] = first;
        pend_n[slot] = nb;
        slot ^= 1;
    }
    if ((rc = drain(slot))) return rc;
    if ((rc = drain(slot ^ 1))) return rc;
    return CC_OK;
}

}  // extern "C"
