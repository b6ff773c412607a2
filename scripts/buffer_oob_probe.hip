// Probe of the buffer unit's range check on this GPU (raw buffer, stride 0):
// does a dword load whose START is inside num_records but whose END is past it
// return the data, zero, or a partial dword?  And does the instruction's
// immediate offset take part in the check?  Build:
//   hipcc --offload-arch=gfx950 -O2 -o build/buffer_oob_probe scripts/buffer_oob_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void probe(const unsigned char* buf, uint32_t nr, uint32_t* out) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(buf), 0, nr, 0x00020000u);
    const uint32_t t = threadIdx.x;  // byte offset t (0..23) as voffset
    out[t] = __builtin_amdgcn_raw_buffer_load_b32(r, t, 0, 0);
    // offsets that wrap when 4 is added in 32 bits (0xFFFFFFFC..0xFFFFFFFF), 0x80000000,
    // and -256..-1 style negatives: OOB only if the unit checks without 32-bit wrap
    if (t < 8) {
        const uint32_t big[8] = {0xFFFFFFFCu, 0xFFFFFFFDu, 0xFFFFFFFEu, 0xFFFFFFFFu,
                                 0x80000000u, 0xFFFFFF00u, 0xFFFFFFF8u, 0x7FFFFFFCu};
        out[32 + t] = __builtin_amdgcn_raw_buffer_load_b32(r, big[t], 0, 0);
    }
}

int main() {
    unsigned char h[64];
    for (int i = 0; i < 64; i++) h[i] = (unsigned char)(0x10 + i);
    unsigned char* d;
    uint32_t* o;
    if (hipMalloc(&d, 64) != hipSuccess || hipMalloc(&o, 64 * 4) != hipSuccess) return 1;
    if (hipMemcpy(d, h, 64, hipMemcpyHostToDevice) != hipSuccess) return 1;
    if (hipMemset(o, 0xAB, 64 * 4) != hipSuccess) return 1;
    const uint32_t nr = 10;
    hipLaunchKernelGGL(probe, dim3(1), dim3(24), 0, 0, d, nr, o);
    uint32_t ho[64];
    if (hipMemcpy(ho, o, sizeof ho, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("{\"num_records\": %u, \"loads\": [", nr);
    for (int t = 0; t < 24; t++) printf("%s{\"offset\": %d, \"value\": \"0x%08x\"}", t ? ", " : "", t, ho[t]);
    printf("], \"wrap_probe\": [");
    const char* names[8] = {"0xFFFFFFFC", "0xFFFFFFFD", "0xFFFFFFFE", "0xFFFFFFFF", "0x80000000", "0xFFFFFF00",
                            "0xFFFFFFF8", "0x7FFFFFFC"};
    for (int t = 0; t < 8; t++) printf("%s{\"offset\": \"%s\", \"value\": \"0x%08x\"}", t ? ", " : "", names[t], ho[32 + t]);
    printf("]}\n");
    return 0;
}
