// scripts/h2d_cpu_probe.cpp -- diagnostic: the calling thread's CPU time inside
// one hipMemcpyAsync host->device call, by size and host-buffer kind
// (hipHostMalloc, malloc + hipHostRegister), and of the completion waits.
// build: hipcc -O2 -o build/h2d_cpu_probe scripts/h2d_cpu_probe.cpp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double cpu_us() {
    timespec t;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}
static double wall_us() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    const size_t max = 16u << 20;
    void *hm = nullptr, *dev = nullptr;
    CK(hipHostMalloc(&hm, max, hipHostMallocDefault));
    void* reg = aligned_alloc(4096, max);
    memset(reg, 1, max);
    memset(hm, 1, max);
    CK(hipHostRegister(reg, max, hipHostRegisterDefault));
    CK(hipMalloc(&dev, max));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const size_t sizes[] = {4096, 1u << 20, 4u << 20, 16u << 20};
    for (int kind = 0; kind < 2; kind++) {
        void* src = kind ? reg : hm;
        for (size_t n : sizes) {
            double c_call = 0, w_call = 0, c_sync = 0, w_total = 0;
            const int reps = 60;
            for (int r = 0; r < reps + 5; r++) {
                const double w0 = wall_us(), c0 = cpu_us();
                CK(hipMemcpyAsync(dev, src, n, hipMemcpyHostToDevice, s));
                const double w1 = wall_us(), c1 = cpu_us();
                CK(hipStreamSynchronize(s));
                const double w2 = wall_us(), c2 = cpu_us();
                if (r >= 5) {
                    c_call += c1 - c0;
                    w_call += w1 - w0;
                    c_sync += c2 - c1;
                    w_total += w2 - w0;
                }
            }
            printf("{\"host\": \"%s\", \"bytes\": %zu, \"call_cpu_us\": %.1f, \"call_wall_us\": %.1f, "
                   "\"sync_cpu_us\": %.1f, \"total_wall_us\": %.1f, \"GBps\": %.1f}\n",
                   kind ? "malloc+hipHostRegister" : "hipHostMalloc", n, c_call / reps, w_call / reps,
                   c_sync / reps, w_total / reps, n / (w_total / reps) / 1e3);
        }
    }
    return 0;
}
