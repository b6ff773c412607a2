// curve_amd/csrc/reader_pool.h -- the persistent io threads of cc_scan_files
// (engine.hip), kept in a header of its own so the host-only thread-sanitizer
// stress test (tests/native/reader_pool_stress.cpp) builds it without HIP.
#pragma once
#include <stdint.h>

#include <condition_variable>
#include <functional>
#include <mutex>
#include <system_error>
#include <thread>
#include <vector>

namespace cc {

// Persistent reader threads of cc_scan_files, one pool per device context:
// created on first use (grown to the largest io_threads asked), parked on a
// condition variable between batches, joined when the context is freed.  A
// batch runs `fn(0)` on the caller and `fn(1..n-1)` on pool threads, and
// returns when all have returned (round 4 spawned and joined a std::thread
// set per 7-file batch: the spawns alone cost more as io_threads grew).
class ReaderPool {
   public:
    ~ReaderPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        go_.notify_all();
        for (auto& t : threads_) t.join();
    }
    // run fn(k) for k in [0, m): k = 0 on the calling thread, m <= n (fewer
    // when the system refuses a new thread: the callers' fn take their work
    // from a shared counter, so any m >= 1 does it all).  Returns m.  fn must
    // not throw (cc_scan_files' readers call C functions only).
    template <class F>
    uint32_t run(uint32_t n, F&& fn) {
        std::lock_guard<std::mutex> one(run_mu_);  // one batch at a time per pool
        const uint32_t helpers = n > 1 ? grow(n - 1) : 0u;
        std::function<void(uint32_t)> job = fn;
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &job;
            want_ = helpers;
            taken_ = 0;
            left_ = helpers;
            gen_++;
        }
        if (helpers) go_.notify_all();
        fn(0);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return left_ == 0; });
        job_ = nullptr;
        return helpers + 1;
    }

   private:
    // pool threads available for a batch wanting n helpers (creation stops at
    // the first refusal, e.g. a thread limit; those made so far are kept)
    uint32_t grow(uint32_t n) {
        try {
            while (threads_.size() < n) threads_.emplace_back([this] { loop(); });
        } catch (const std::system_error&) {
        }
        return threads_.size() < n ? (uint32_t)threads_.size() : n;
    }
    void loop() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            go_.wait(lk, [&] { return stop_ || (gen_ != seen && taken_ < want_); });
            if (stop_) return;
            if (taken_ >= want_) {  // this generation is fully staffed
                seen = gen_;
                continue;
            }
            const uint32_t k = 1 + taken_++;
            seen = gen_;
            std::function<void(uint32_t)>* job = job_;
            lk.unlock();
            (*job)(k);
            lk.lock();
            if (--left_ == 0) done_.notify_one();
        }
    }
    std::mutex run_mu_, mu_;
    std::condition_variable go_, done_;
    std::vector<std::thread> threads_;
    std::function<void(uint32_t)>* job_ = nullptr;
    uint64_t gen_ = 0;
    uint32_t want_ = 0, taken_ = 0, left_ = 0;
    bool stop_ = false;
};

}  // namespace cc
