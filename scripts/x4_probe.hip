// scripts/x4_probe.hip -- two gfx950 facts the dwordx4 write-log layout relies on:
//  1. v_permlane32_swap / v_permlane16_swap: the 4x4 (row a of 16 lanes) x (dword c)
//     transpose of kernels.hip's log path (two stages, four swaps per 4 registers);
//  2. raw buffer_load_dwordx4 at byte offsets that are not 4- or 16-byte aligned.
// Build: hipcc --offload-arch=gfx950 -O2 scripts/x4_probe.hip -o build/x4_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

__global__ void transpose_probe(uint32_t* out) {
    const uint32_t lane = threadIdx.x;
    uint32_t r[4];
    for (int c = 0; c < 4; c++) r[c] = (lane << 8) | c;  // value = (lane, c)
    auto s0 = __builtin_amdgcn_permlane32_swap(r[0], r[2], false, false);
    auto s1 = __builtin_amdgcn_permlane32_swap(r[1], r[3], false, false);
    r[0] = s0[0]; r[2] = s0[1]; r[1] = s1[0]; r[3] = s1[1];
    auto t0 = __builtin_amdgcn_permlane16_swap(r[0], r[1], false, false);
    auto t1 = __builtin_amdgcn_permlane16_swap(r[2], r[3], false, false);
    r[0] = t0[0]; r[1] = t0[1]; r[2] = t1[0]; r[3] = t1[1];
    for (int s = 0; s < 4; s++) out[s * 64 + lane] = r[s];
}

__global__ void x4_probe(const unsigned char* buf, uint32_t shift, uint32_t* out) {
    const uint32_t lane = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(buf), 0, 4096, 0x00020000u);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, 16u * lane + shift, 0, 0);
    for (int c = 0; c < 4; c++) out[lane * 4 + c] = v[c];
}

int main() {
    uint32_t* d;
    hipMalloc(&d, 4096 * 4);
    hipLaunchKernelGGL(transpose_probe, dim3(1), dim3(64), 0, 0, d);
    uint32_t h[256];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    int bad = 0;
    for (uint32_t s = 0; s < 4; s++)
        for (uint32_t L = 0; L < 64; L++) {
            const uint32_t r = L / 16, b = L % 16;       // output lane (row r, b)
            const uint32_t want = ((16 * s + b) << 8) | r;  // input (a = s, b) component c = r
            if (h[s * 64 + L] != want) bad++;
        }
    printf("{\"transpose_mismatches\": %d", bad);
    unsigned char* buf;
    hipMalloc(&buf, 8192);
    unsigned char hb[8192];
    for (int i = 0; i < 8192; i++) hb[i] = (unsigned char)(i * 7 + 3);
    hipMemcpy(buf, hb, 8192, hipMemcpyHostToDevice);
    for (uint32_t shift : {0u, 1u, 2u, 3u, 4u, 5u, 12u, 13u}) {
        hipLaunchKernelGGL(x4_probe, dim3(1), dim3(64), 0, 0, buf, shift, d);
        uint32_t o[256];
        hipMemcpy(o, d, sizeof o, hipMemcpyDeviceToHost);
        int wrong = 0;
        for (uint32_t L = 0; L < 64; L++)
            for (uint32_t c = 0; c < 4; c++) {
                uint32_t want;
                memcpy(&want, hb + 16 * L + shift + 4 * c, 4);
                if (16 * L + shift + 4 * c + 4 > 4096) want = 0;
                if (o[L * 4 + c] != want) wrong++;
            }
        printf(", \"x4_shift%u_wrong\": %d", shift, wrong);
    }
    printf("}\n");
    return 0;
}
