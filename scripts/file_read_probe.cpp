// scripts/file_read_probe.cpp -- where can cc_scan_files' host side go?  (diagnostic)
//
// Page-cache-resident chunk files (16 MiB + 4 KiB) copied into pinned staging
// (hipHostMalloc) by T threads, four ways:
//   pread     2 MiB pread()s (what cc_scan_files does)
//   mmap_cpy  mmap(MAP_POPULATE) of the file + memcpy
//   mmap_nt   mmap(MAP_POPULATE) + AVX2 non-temporal stores (no read-for-ownership
//             of the staging lines)
// each alone and while a second pinned buffer streams H2D on the GPU (the
// overlap cc_scan_files runs: batch i+1's reads beside batch i's copy).
// Prints one JSON line per case.
//   hipcc -O3 -mavx2 -std=c++17 scripts/file_read_probe.cpp -o build/file_read_probe
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

static const size_t kFile = (16u << 20) + 4096, kPiece = 2u << 20, kBatch = 7;

static void nt_copy(void* dst, const void* src, size_t n) {
    char* d = static_cast<char*>(dst);
    const char* s = static_cast<const char*>(src);
    size_t i = 0;
    for (; i + 128 <= n; i += 128) {
        __m256i a = _mm256_loadu_si256((const __m256i*)(s + i));
        __m256i b = _mm256_loadu_si256((const __m256i*)(s + i + 32));
        __m256i c = _mm256_loadu_si256((const __m256i*)(s + i + 64));
        __m256i e = _mm256_loadu_si256((const __m256i*)(s + i + 96));
        _mm256_stream_si256((__m256i*)(d + i), a);
        _mm256_stream_si256((__m256i*)(d + i + 32), b);
        _mm256_stream_si256((__m256i*)(d + i + 64), c);
        _mm256_stream_si256((__m256i*)(d + i + 96), e);
    }
    memcpy(d + i, s + i, n - i);
    _mm_sfence();
}

int main(int argc, char** argv) {
    const int nfiles = argc > 1 ? atoi(argv[1]) : 128;
    const char* dir = getenv("TMPDIR") ? getenv("TMPDIR") : "/tmp";
    std::vector<std::string> paths;
    {
        std::vector<char> body(kFile);
        for (size_t i = 0; i < kFile; i++) body[i] = (char)(i * 2654435761u >> 13);
        for (int f = 0; f < nfiles; f++) {
            std::string p = std::string(dir) + "/frp_" + std::to_string(getpid()) + "_" + std::to_string(f);
            const int fd = open(p.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
            body[0] = (char)f;
            if (fd < 0 || write(fd, body.data(), kFile) != (ssize_t)kFile) return 2;
            close(fd);
            paths.push_back(p);
        }
    }
    void* stage = nullptr;
    void* dma_src = nullptr;
    void* dma_dst = nullptr;
    if (hipHostMalloc(&stage, kBatch * kFile, hipHostMallocDefault) != hipSuccess) return 3;
    if (hipHostMalloc(&dma_src, 128u << 20, hipHostMallocDefault) != hipSuccess) return 3;
    if (hipMalloc(&dma_dst, 128u << 20) != hipSuccess) return 3;
    memset(stage, 1, kBatch * kFile);
    memset(dma_src, 2, 128u << 20);
    hipStream_t st;
    (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);

    auto run = [&](int mode, int threads) {
        // items: every file in pieces, into its slot of a 7-file batch
        const size_t pieces = (kFile + kPiece - 1) / kPiece;
        std::atomic<size_t> next{0};
        const size_t items = (size_t)nfiles * pieces;
        auto worker = [&]() {
            int cur_fd = -1, cur_f = -1;
            char* map = nullptr;
            for (size_t it; (it = next.fetch_add(1)) < items;) {
                const size_t f = it / pieces, k = it % pieces;
                const size_t off = k * kPiece, len = kFile - off < kPiece ? kFile - off : kPiece;
                char* dst = static_cast<char*>(stage) + (f % kBatch) * kFile + off;
                if (mode == 0) {
                    const int fd = open(paths[f].c_str(), O_RDONLY);
                    size_t got = 0;
                    while (got < len) {
                        ssize_t r = pread(fd, dst + got, len - got, off + got);
                        if (r <= 0) break;
                        got += r;
                    }
                    close(fd);
                } else {
                    if ((int)f != cur_f) {
                        if (map) munmap(map, kFile);
                        if (cur_fd >= 0) close(cur_fd);
                        cur_fd = open(paths[f].c_str(), O_RDONLY);
                        map = static_cast<char*>(mmap(nullptr, kFile, PROT_READ, MAP_SHARED | MAP_POPULATE, cur_fd, 0));
                        cur_f = (int)f;
                    }
                    if (mode == 1)
                        memcpy(dst, map + off, len);
                    else
                        nt_copy(dst, map + off, len);
                }
            }
            if (map) munmap(map, kFile);
            if (cur_fd >= 0) close(cur_fd);
        };
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (int t = 0; t < threads; t++) th.emplace_back(worker);
        for (auto& x : th) x.join();
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    };
    const char* names[3] = {"pread", "mmap_cpy", "mmap_nt"};
    for (int dma = 0; dma < 2; dma++) {
        std::atomic<bool> stop{false};
        std::atomic<uint64_t> moved{0};
        std::thread pump;
        if (dma) {
            pump = std::thread([&]() {
                while (!stop.load()) {
                    (void)hipMemcpyAsync(dma_dst, dma_src, 128u << 20, hipMemcpyHostToDevice, st);
                    (void)hipStreamSynchronize(st);
                    moved += 128u << 20;
                }
            });
            std::this_thread::sleep_for(std::chrono::milliseconds(100));
        }
        for (int mode = 0; mode < 3; mode++)
            for (int threads : {1, 2, 4, 8, 12, 16}) {
                run(mode, threads);  // warm
                double best = 1e9, sum = 0;
                const int reps = 3;
                const uint64_t m0 = moved.load();
                const auto w0 = std::chrono::steady_clock::now();
                for (int r = 0; r < reps; r++) {
                    const double el = run(mode, threads);
                    best = el < best ? el : best;
                    sum += el;
                }
                const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count();
                const double gib = (double)nfiles * kFile / (1u << 30);
                printf("{\"mode\": \"%s\", \"threads\": %d, \"with_h2d\": %d, \"GiBps_best\": %.2f, \"GiBps_mean\": %.2f"
                       ", \"h2d_GiBps\": %.2f}\n",
                       names[mode], threads, dma, gib / best, gib * reps / sum,
                       dma ? (double)(moved.load() - m0) / (1u << 30) / wall : 0.0);
                fflush(stdout);
            }
        if (dma) {
            stop = true;
            pump.join();
        }
    }
    for (auto& p : paths) unlink(p.c_str());
    return 0;
}
