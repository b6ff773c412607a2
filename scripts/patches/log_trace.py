#!/usr/bin/env python3
"""Timing-trace build of log_apply_kernel (NOT the shipped kernel): patches a COPY
of kernels.hip so lane 0 of every wave records, with s_memrealtime (100 MHz), the
time it starts, leaves its insert tiles, leaves the LDS fill, passes the
workgroup's wait for every inserted tile, and ends, plus its XCD, into a
__device__ array read back by cc_log_trace_read().
usage: log_trace.py KERNELS_HIP   (scripts/log_trace.py runs it)"""
import sys

p = sys.argv[1]
s = open(p).read()


def rep(old, new):
    global s
    assert old in s, old[:80]
    s = s.replace(old, new, 1)


rep("""    for (uint64_t t = (uint64_t)blockIdx.x * WV + wave; t < n_tiles; t += (uint64_t)gridDim.x * WV)
        insert_tile(a, t, tag, lane);
    fill_lds<64 * WV>(tab, static_cast<const uint4*>(a.image));
    if (wave == 0) wait_inserted(a, tag, n_tiles, ctr, lane);
    __syncthreads();""", """    uint64_t* tr = g_log_trace + 8 * (blockIdx.x * WV + wave);
    const uint64_t tr0 = __builtin_amdgcn_s_memrealtime();
    for (uint64_t t = (uint64_t)blockIdx.x * WV + wave; t < n_tiles; t += (uint64_t)gridDim.x * WV)
        insert_tile(a, t, tag, lane);
    const uint64_t tr1 = __builtin_amdgcn_s_memrealtime();
    fill_lds<64 * WV>(tab, static_cast<const uint4*>(a.image));
    const uint64_t tr2 = __builtin_amdgcn_s_memrealtime();
    if (wave == 0) wait_inserted(a, tag, n_tiles, ctr, lane);
    __syncthreads();
    const uint64_t tr3 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        tr[0] = tr0;
        tr[1] = tr1;
        tr[2] = tr2;
        tr[3] = tr3;
        tr[4] = tr3;
        tr[5] = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u;
    }""")
rep("""    log_pages_body<M, Delta>(a, tab);
}""", """    log_pages_body<M, Delta>(a, tab);
    if ((threadIdx.x & 63u) == 0)
        g_log_trace[8 * (blockIdx.x * log_waves(M, Delta) + (threadIdx.x >> 6)) + 4] = __builtin_amdgcn_s_memrealtime();
}""")
rep("""    const uint32_t first = hb0 + (uint32_t)((uint64_t)Hb * wprefix(wave) / wsum);""",
    """    const uint32_t first = hb0 + (uint32_t)((uint64_t)Hb * wprefix(wave) / wsum);
    if (lane == 0) g_log_trace[8 * (blockIdx.x * WV + wave) + 6] = H - first;""")
rep("""__device__ __forceinline__ uint32_t page_hash(""", """__device__ uint64_t g_log_trace[8 * 8192];
__device__ __forceinline__ uint32_t page_hash(""")
s += """
extern "C" int cc_log_trace_read(void* dst, size_t bytes) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(cc::g_log_trace), bytes) == hipSuccess ? 0 : -1;
}
"""
open(p, "w").write(s)
