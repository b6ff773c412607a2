// scripts/hbm_probe.hip -- read-only HBM bandwidth probe (diagnostic, not product).
//
// Measures what a pure streaming read achieves on this MI355X with the same
// launch shape as the page-CRC kernel (one 1024-thread block per CU, grid
// stride) and with several load widths, so the page kernel's roofline
// fraction can be read against a measured ceiling and FETCH_SIZE can be
// calibrated on a known byte count.  Each variant XOR-reduces what it reads
// (one store per wave) so nothing is dead-code eliminated.
//
// build: hipcc -O3 --offload-arch=gfx950 -o build/hbm_probe scripts/hbm_probe.hip
// run:   build/hbm_probe [GiB=16] [reps=10]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

// W = dwords per lane per load (1, 2, 4); U = loads in flight per lane per step; NT = nontemporal.
template <int W, int U, bool NT>
__global__ __launch_bounds__(1024) void read_kernel(const uint32_t* __restrict__ p, uint64_t n_dw,
                                                    uint32_t* __restrict__ out) {
    const uint64_t lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
    const uint64_t waves = (uint64_t)gridDim.x * 16;
    const uint64_t step_dw = 64ull * W * U;  // dwords per wave per step
    uint32_t acc = 0;
    for (uint64_t base = wave * step_dw; base + step_dw <= n_dw; base += waves * step_dw) {
        uint32_t v[U * W];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t* q = p + base + (uint64_t)u * 64 * W + lane * W;
            if (W == 4) {
                u32x4 t = NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(q))
                             : *reinterpret_cast<const u32x4*>(q);
                v[u * W + 0] = t.x; v[u * W + 1] = t.y; v[u * W + 2] = t.z; v[u * W + 3] = t.w;
            } else if (W == 2) {
                u32x2 t = NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(q))
                             : *reinterpret_cast<const u32x2*>(q);
                v[u * W + 0] = t.x; v[u * W + 1] = t.y;
            } else {
                v[u] = NT ? __builtin_nontemporal_load(q) : *q;
            }
        }
#pragma unroll
        for (int i = 0; i < U * W; i++) acc ^= v[i];
    }
    acc ^= __shfl_xor(acc, 32);
    if (lane == 0) out[wave] = acc;
}

template <int W, int U, bool NT>
void run(const char* name, const uint32_t* d, uint64_t n_dw, uint32_t* out, int blocks, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL((read_kernel<W, U, NT>), dim3(blocks), dim3(1024), 0, 0, d, n_dw, out);
    CK(hipDeviceSynchronize());
    float best = 1e30f, tot = 0;
    for (int r = 0; r < reps; r++) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((read_kernel<W, U, NT>), dim3(blocks), dim3(1024), 0, 0, d, n_dw, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
        tot += ms;
    }
    const double bytes = (double)n_dw * 4;
    printf("{\"probe\":\"%s\",\"blocks\":%d,\"bytes\":%.0f,\"ms_avg\":%.4f,\"ms_best\":%.4f,\"GBps_avg\":%.1f,\"GBps_best\":%.1f}\n",
           name, blocks, bytes, tot / reps, best, bytes / (tot / reps) / 1e6, bytes / best / 1e6);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 16.0;
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    const uint64_t n_dw = (uint64_t)(gib * (1ull << 30)) / 4;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    uint32_t* d;
    uint32_t* out;
    CK(hipMalloc(&d, n_dw * 4));
    CK(hipMalloc(&out, 1u << 24));
    CK(hipMemset(d, 0x5A, n_dw * 4));
    printf("{\"device\":\"%s\",\"cus\":%d,\"gib\":%.1f}\n", prop.gcnArchName, cus, gib);
    run<1, 16, true>("dword_x16_nt", d, n_dw, out, cus, reps);
    run<1, 16, false>("dword_x16", d, n_dw, out, cus, reps);
    run<2, 8, true>("dwordx2_x8_nt", d, n_dw, out, cus, reps);
    run<4, 4, true>("dwordx4_x4_nt", d, n_dw, out, cus, reps);
    run<4, 4, false>("dwordx4_x4", d, n_dw, out, cus, reps);
    run<4, 8, false>("dwordx4_x8", d, n_dw, out, cus, reps);
    run<4, 4, false>("dwordx4_x4_2xgrid", d, n_dw, out, 2 * cus, reps);
    run<1, 16, true>("dword_x16_nt_2xgrid", d, n_dw, out, 2 * cus, reps);
    CK(hipFree(d));
    CK(hipFree(out));
    return 0;
}
