// curve_amd/host/scan_op_bench.cpp -- bench and test harness (not product):
// ScanChunkRequest-shaped CRC calls from T threads at once, timed natively
// (no interpreter between the calls).
//
// The reference hashes one scan op per raft-applied ScanChunkRequest: the 4 KiB
// metapage or one 4 MiB data slice, `crc = CRC32(readBuffer, size)`
// (src/chunkserver/op_request.cpp:776-794, :847), on the write apply pool,
// wconcurrentapply.size = 10 threads (conf/chunkserver.conf:183; scan ops are
// queued there, op_request.cpp:179-187).  A chunk is 5 ops at scanSize 4 MiB
// (scan_manager_test.cpp:107-142).
//
// sob_run: thread t runs `calls` ops over its own buffer bufs[t], op i being
// (op_off[i % n_ops], op_len[i % n_ops]), in one of three modes:
//   0  CPU: crc32c_value (libcurvecrc's CPU primitive, the drop-in for CRC32)
//   1  GPU: cc_page_crc_host over the op's pages + cc_fold_host
//   2  routed: cchost::ScanOpCrc (chunkserver_host: below kCpuHashMax on the CPU
//      primitive, else mode 1) -- what the integration recipe runs
// Per call: latency (us) and the CRC; per run: wall seconds from a common start
// to the last thread's end, the calling threads' summed CPU seconds, and the
// whole process's CPU seconds over the same window (the HIP runtime's own
// threads included: what a GPU call really costs the host).
#include <pthread.h>
#include <stdint.h>
#include <time.h>

#include <atomic>
#include <thread>
#include <vector>

#include "../../include/curve_crc.h"
#include "chunkserver_host.h"

namespace {
double now_s(clockid_t id) {
    timespec ts;
    clock_gettime(id, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}
}  // namespace

extern "C" int sob_run(uint32_t threads, const void* const* bufs, const uint64_t* op_off, const uint64_t* op_len,
                       uint32_t n_ops, uint32_t calls, int mode, double* lat_us, uint32_t* crcs, double* out) {
    if (!threads || !bufs || !op_off || !op_len || !n_ops || !lat_us || !crcs || !out || mode < 0 || mode > 2)
        return CC_EINVAL;
    std::atomic<uint32_t> ready{0};
    std::atomic<bool> go{false};
    std::atomic<int> first_err{0};
    std::vector<double> cpu(threads, 0.0), end(threads, 0.0);
    double start = 0.0;
    auto body = [&](uint32_t t) {
        const unsigned char* base = static_cast<const unsigned char*>(bufs[t]);
        std::vector<uint32_t> pages;
        ready.fetch_add(1);
        while (!go.load(std::memory_order_acquire)) std::this_thread::yield();  // before the timed window
        const double c0 = now_s(CLOCK_THREAD_CPUTIME_ID);
        for (uint32_t i = 0; i < calls; i++) {
            const unsigned char* p = base + op_off[i % n_ops];
            const uint64_t n = op_len[i % n_ops];
            const double t0 = now_s(CLOCK_MONOTONIC);
            uint32_t crc = 0;
            int rc = CC_OK;
            if (mode == 0) {
                crc = crc32c_value(p, n);
            } else if (mode == 1) {
                pages.resize(n / 4096);
                rc = cc_page_crc_host(p, n / 4096, 4096, pages.data());
                if (rc == CC_OK) crc = cc_fold_host(pages.data(), n / 4096, 4096);
            } else {
                rc = cchost::ScanOpCrc(reinterpret_cast<const char*>(p), n, &crc) ? CC_OK : CC_EHIP;
            }
            lat_us[(uint64_t)t * calls + i] = (now_s(CLOCK_MONOTONIC) - t0) * 1e6;
            crcs[(uint64_t)t * calls + i] = crc;
            if (rc != CC_OK) {
                int z = 0;
                first_err.compare_exchange_strong(z, rc);
                break;
            }
        }
        cpu[t] = now_s(CLOCK_THREAD_CPUTIME_ID) - c0;
        end[t] = now_s(CLOCK_MONOTONIC);
    };
    std::vector<std::thread> ts;
    for (uint32_t t = 0; t < threads; t++) ts.emplace_back(body, t);
    while (ready.load() < threads) std::this_thread::yield();
    const double p0 = now_s(CLOCK_PROCESS_CPUTIME_ID);
    start = now_s(CLOCK_MONOTONIC);
    go.store(true, std::memory_order_release);
    for (auto& th : ts) th.join();
    const double p1 = now_s(CLOCK_PROCESS_CPUTIME_ID);
    double last = start, cpu_sum = 0.0;
    for (uint32_t t = 0; t < threads; t++) {
        if (end[t] > last) last = end[t];
        cpu_sum += cpu[t];
    }
    out[0] = last - start;
    out[1] = cpu_sum;
    out[2] = p1 - p0;
    return first_err.load();
}
