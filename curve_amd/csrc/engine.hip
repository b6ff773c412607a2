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

#include <mutex>
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

struct Staging {
    bool ready = false;
    size_t bytes = 0;            // per slot
    void* host[2] = {nullptr, nullptr};
    void* dev[2] = {nullptr, nullptr};
    uint32_t* dcrc[2] = {nullptr, nullptr};
    uint32_t* hcrc[2] = {nullptr, nullptr};
    hipStream_t stream[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
};

struct DevCtx {
    bool ready = false;
    int cus = 256;
    void* image = nullptr;
    std::mutex submit;  // serialises *_host calls on this device
    Staging st;
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
    }
    st = Staging();
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
        default: return "unknown error";
    }
}

int cc_lds_image(void* out, size_t bytes) {
    if (!out || bytes < kLdsBytes) return CC_EINVAL;
    build_lds_image(static_cast<uint32_t*>(out));
    return CC_OK;
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

int cc_page_verify_dev(const void* d_pages, uint64_t n_pages, uint32_t page_bytes, const uint32_t* d_expected,
                       uint64_t* d_bad_count, uint64_t* d_first_bad, void* stream) {
    if (!page_size_ok(page_bytes)) return CC_EINVAL;
    if (n_pages == 0) return CC_OK;
    if (!d_pages || !d_expected || !d_bad_count || !d_first_bad || ((uintptr_t)d_pages & 3u)) return CC_EINVAL;
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
    a.bad_count = reinterpret_cast<unsigned long long*>(d_bad_count);
    a.first_bad = reinterpret_cast<unsigned long long*>(d_first_bad);
    geometry_for(c, n_pages, &a);
    return map_err(launch_page_verify(a, static_cast<hipStream_t>(stream)));
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
            if ((e = hipEventSynchronize(st.done[slot])) != hipSuccess) return map_err(e);
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
        if ((e = hipEventRecord(st.done[slot], st.stream[slot])) != hipSuccess) return map_err(e);
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
        if ((e = hipEventSynchronize(st.done[slot])) != hipSuccess) return map_err(e);
        memcpy(h_out + pending_first[slot], st.hcrc[slot], pending_n[slot] * 4);
        pending_n[slot] = 0;
        slot ^= 1;
    }
    return CC_OK;
}

}  // extern "C"
