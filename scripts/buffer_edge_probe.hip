// Probe: clipped-descriptor stores/loads with base = page + a and voffset =
// 4*lane - a (wrapping) + imm 256*j.  Which (a, dword) combinations land?
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
constexpr uint32_t kFlags = 0x00020000u;
__global__ void k(unsigned char* page, uint32_t a, uint32_t nr, uint32_t* loads) {
    const uint32_t lane = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(page + a, 0, nr, kFlags);
    const uint32_t vo = 4u * lane - a;
#pragma unroll
    for (int j = 0; j < 16; j++) __builtin_amdgcn_raw_buffer_store_b32(1u, rc, vo + 256u * j, 0, 0);
}
__global__ void kl(const unsigned char* src, uint32_t a, uint32_t nr, uint32_t* out) {
    const uint32_t lane = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(src) + a, 0, nr, kFlags);
    const uint32_t vo = 4u * lane - a;
#pragma unroll
    for (int j = 0; j < 16; j++) out[lane + 64 * j] = __builtin_amdgcn_raw_buffer_load_b32(rc, vo + 256u * j, 0, 0);
}
int main() {
    unsigned char *d, *s;
    uint32_t* o;
    if (hipMalloc(&d, 8192) != hipSuccess || hipMalloc(&s, 8192) != hipSuccess || hipMalloc(&o, 4096) != hipSuccess) return 1;
    uint32_t hs[1024];
    for (int i = 0; i < 1024; i++) hs[i] = 0x1000 + i;
    (void)hipMemcpy(s, hs, 4096, hipMemcpyHostToDevice);
    const uint32_t as[] = {256, 260, 264, 268, 272, 276, 1028, 4, 8, 12, 16, 100, 3000};
    for (uint32_t a : as) {
        const uint32_t nr = 1024;
        (void)hipMemset(d, 0, 8192);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, a, nr, o);
        uint32_t h[1024];
        (void)hipMemcpy(h, d, 4096, hipMemcpyDeviceToHost);
        int miss = 0, extra = 0, first_miss = -1;
        for (int i = 0; i < 1024; i++) {
            const bool want = 4u * i >= a && 4u * i < a + nr;
            if (want && !h[i]) { miss++; if (first_miss < 0) first_miss = i; }
            if (!want && h[i]) extra++;
        }
        hipLaunchKernelGGL(kl, dim3(1), dim3(64), 0, 0, s, a, nr, o);
        uint32_t hl[1024];
        (void)hipMemcpy(hl, o, 4096, hipMemcpyDeviceToHost);
        int lmiss = 0, lbad = 0, lfirst = -1;
        for (int i = 0; i < 1024; i++) {
            const bool want = 4u * i >= a && 4u * i < a + nr;
            if (want && hl[i] != hs[i]) { lmiss++; if (lfirst < 0) lfirst = i; }
            if (!want && hl[i]) lbad++;
        }
        printf("a=%u: store missing %d (first dword %d) extra %d | load wrong %d (first %d) extra %d\n", a, miss,
               first_miss, extra, lmiss, lfirst, lbad);
    }
    return 0;
}
