// tests/native/reader_pool_stress.cpp -- the persistent io threads of
// cc_scan_files (curve_amd/csrc/reader_pool.h) under stress, built host-only with
// -fsanitize=thread by tests/test_sanitize.py: batches of 1..24 participants
// back to back (the pool grows on demand), every participant index run exactly
// once per batch, every work item taken exactly once, a batch never returning
// before its last participant, and pools created and destroyed while idle.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../curve_amd/csrc/reader_pool.h"

#define CHECK(c)                                                         \
    do {                                                                 \
        if (!(c)) {                                                      \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            std::exit(1);                                                \
        }                                                                \
    } while (0)

int main() {
    uint64_t seed = 0x9E3779B97F4A7C15ull;
    auto rnd = [&]() {
        seed ^= seed << 13;
        seed ^= seed >> 7;
        seed ^= seed << 17;
        return seed;
    };
    for (int pools = 0; pools < 8; pools++) {
        cc::ReaderPool pool;
        for (int batch = 0; batch < 400; batch++) {
            const uint32_t n = 1 + (uint32_t)(rnd() % 24);
            const uint64_t items = 1 + rnd() % 200;
            std::vector<std::atomic<int>> ran(n), taken(items);
            for (auto& x : ran) x.store(0);
            for (auto& x : taken) x.store(0);
            std::atomic<uint64_t> next{0};
            std::vector<uint64_t> plain(items, 0);  // written by the workers, read after run(): needs run()'s ordering
            const uint32_t m = pool.run(n, [&](uint32_t k) {
                CHECK(k < n);
                ran[k].fetch_add(1);
                for (uint64_t it; (it = next.fetch_add(1)) < items;) {
                    taken[it].fetch_add(1);
                    plain[it] = it * 3 + 1;
                }
            });
            CHECK(m == n);  // no thread refused here
            for (uint32_t k = 0; k < n; k++) CHECK(ran[k].load() == 1);
            for (uint64_t i = 0; i < items; i++) CHECK(taken[i].load() == 1 && plain[i] == i * 3 + 1);
        }
    }
    std::printf("reader_pool_stress: ok\n");
    return 0;
}
