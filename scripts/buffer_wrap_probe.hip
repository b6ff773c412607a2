// Second probe of the buffer unit's range check (raw buffer, stride 0), for
// the write-log kernel's addressing: (1) is voffset + instruction offset
// summed in 32 bits (a "negative" voffset plus a positive immediate wrapping
// back into range), (2) does soffset take part in the range check, and (3) do
// stores follow the same rules?  Build:
//   hipcc --offload-arch=gfx950 -O2 -o build/buffer_wrap_probe scripts/buffer_wrap_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr uint32_t kFlags = 0x00020000u;

// each case: (voffset, soffset, imm) -> loaded value (nr = 1024, buf[i] = 0x1000 + i dwords)
__global__ void probe_load(const uint32_t* buf, uint32_t* out) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(buf), 0, 1024, kFlags);
    const uint32_t t = threadIdx.x;
    uint32_t v = 0xDEADBEEFu;
    switch (t) {
        case 0: v = __builtin_amdgcn_raw_buffer_load_b32(r, 0xFFFFFF00u, 0, 0); break;                     // -256
        case 1: v = __builtin_amdgcn_raw_buffer_load_b32(r, 0xFFFFFF00u + 256u, 0, 0); break;              // folded by the compiler: 0
        case 2: v = __builtin_amdgcn_raw_buffer_load_b32(r, 0xFFFFFF00u, 0, 0); break;
        case 3: v = __builtin_amdgcn_raw_buffer_load_b32(r, 16, 2000, 0); break;                            // soffset past nr
        case 4: v = __builtin_amdgcn_raw_buffer_load_b32(r, 16, 0x80000000u, 0); break;                     // soffset huge
        case 5: v = __builtin_amdgcn_raw_buffer_load_b32(r, 2000, 0, 0); break;                             // voffset past nr
        case 6: v = __builtin_amdgcn_raw_buffer_load_b32(r, 16, 512, 0); break;                             // soffset inside
        default: break;
    }
    out[t] = v;
}

// the immediate must reach the instruction: pass voffset opaque, add imm inside
__global__ void probe_imm(const uint32_t* buf, const uint32_t* voffs, uint32_t* out) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(buf), 0, 1024, kFlags);
    const uint32_t t = threadIdx.x;
    const uint32_t vo = voffs[t];
    // immediate offsets 256 and 1024 as instruction offsets (vo opaque to the compiler)
    out[2 * t] = __builtin_amdgcn_raw_buffer_load_b32(r, vo + 256u, 0, 0);
    out[2 * t + 1] = __builtin_amdgcn_raw_buffer_load_b32(r, vo + 1024u, 0, 0);
}

__global__ void probe_store(uint32_t* buf, const uint32_t* voffs, uint32_t so) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(buf, 0, 1024, kFlags);
    const uint32_t t = threadIdx.x;
    __builtin_amdgcn_raw_buffer_store_b32(0xC0DE0000u | t, r, voffs[t] + 256u, so, 0);
}

int main() {
    uint32_t h[1024];
    for (int i = 0; i < 1024; i++) h[i] = 0x1000u + (uint32_t)i;
    uint32_t *d, *o, *vo;
    if (hipMalloc(&d, 4096 * 2) != hipSuccess || hipMalloc(&o, 4096) != hipSuccess || hipMalloc(&vo, 4096) != hipSuccess)
        return 1;
    if (hipMemcpy(d, h, 4096, hipMemcpyHostToDevice) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe_load, dim3(1), dim3(8), 0, 0, d, o);
    uint32_t ho[64];
    if (hipMemcpy(ho, o, 8 * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("{\"load\": {\"vo=-256\": \"0x%08x\", \"vo=-256+256(folded)\": \"0x%08x\", \"soff=2000,vo=16\": \"0x%08x\", "
           "\"soff=2^31,vo=16\": \"0x%08x\", \"vo=2000\": \"0x%08x\", \"soff=512,vo=16\": \"0x%08x\"}",
           ho[0], ho[1], ho[3], ho[4], ho[5], ho[6]);
    // voffsets: -256 (-> +256 imm = 0), -252 (-> 4), -4 (-> 252), 0 (-> 256)
    const uint32_t hv[4] = {0xFFFFFF00u, 0xFFFFFF04u, 0xFFFFFFFCu, 0u};
    if (hipMemcpy(vo, hv, sizeof hv, hipMemcpyHostToDevice) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe_imm, dim3(1), dim3(4), 0, 0, d, vo, o);
    if (hipMemcpy(ho, o, 8 * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf(", \"imm\": [");
    for (int t = 0; t < 4; t++)
        printf("%s{\"voffset\": \"0x%08x\", \"+256\": \"0x%08x\", \"+1024\": \"0x%08x\"}", t ? ", " : "", hv[t], ho[2 * t],
               ho[2 * t + 1]);
    printf("]");
    // stores: voffset + 256 with the same voffsets; soffset 0 then 2000
    for (int pass = 0; pass < 2; pass++) {
        if (hipMemcpy(d, h, 4096, hipMemcpyHostToDevice) != hipSuccess) return 1;
        hipLaunchKernelGGL(probe_store, dim3(1), dim3(4), 0, 0, d, vo, pass ? 2000u : 0u);
        uint32_t back[1024];
        if (hipMemcpy(back, d, 4096, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        printf(", \"store_soff%d\": [", pass ? 2000 : 0);
        int first = 1;
        for (int i = 0; i < 1024; i++)
            if (back[i] != h[i]) {
                printf("%s{\"dword\": %d, \"value\": \"0x%08x\"}", first ? "" : ", ", i, back[i]);
                first = 0;
            }
        printf("]");
    }
    printf("}\n");
    return 0;
}
