#!/usr/bin/env python3
"""Timing-trace build of range_flat_kernel (NOT the shipped kernel): patches a COPY
of kernels.hip so every wave records, with s_memrealtime (100 MHz), the time it
enters the kernel, has published its tile counts, has filled LDS, has every
tile count, the time it starts its first item (after the LDS fill and the tile-count wait), the time it
leaves the static pieces, and its end, plus its XCD, blocks hashed and dynamic
chunks pulled, into a __device__ array read back by cc_range_trace_read().
usage: range_trace.py KERNELS_HIP   (scripts/gpu_wal_trace.sh builds and runs it)"""
import sys

p = sys.argv[1]
s = open(p).read()


def rep(old, new):
    global s
    assert old in s, old[:80]
    s = s.replace(old, new, 1)


rep("""    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t W = (uint64_t)gridDim.x * kFlatWaves;""", """    const uint64_t tr_entry = __builtin_amdgcn_s_memrealtime();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t W = (uint64_t)gridDim.x * kFlatWaves;""")
rep("""    fill_lds<64 * kFlatWaves>(tab, static_cast<const uint4*>(a.image));
    const unsigned char* __restrict__ buf = a.buf;""", """    const uint64_t tr_pub = __builtin_amdgcn_s_memrealtime();
    fill_lds<64 * kFlatWaves>(tab, static_cast<const uint4*>(a.image));
    const uint64_t tr_fill = __builtin_amdgcn_s_memrealtime();
    const unsigned char* __restrict__ buf = a.buf;""")
rep("""    wait_tiles<kTpl>(tb, a.tiles, tag, lane, [&](uint32_t t) { return range_tile_count(a, t, lane, false); });""",
    """    wait_tiles<kTpl>(tb, a.tiles, tag, lane, [&](uint32_t t) { return range_tile_count(a, t, lane, false); });
    const uint64_t tr_wait = __builtin_amdgcn_s_memrealtime();""")
rep("""
    // work items: static pieces item < rounds, then dynamic chunks until the counter runs out
#pragma unroll 1
    for (uint32_t item = 0;; item++) {""", """
    const uint64_t tr_t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t tr_ts = 0, tr_blocks = 0, tr_dyn = 0;

    // work items: static pieces item < rounds, then dynamic chunks until the counter runs out
#pragma unroll 1
    for (uint32_t item = 0;; item++) {
        if (item == rounds) tr_ts = __builtin_amdgcn_s_memrealtime();""")
rep("""            if (c >= n_dyn) break;
            b0 = Bs + c * kRangeDynBlocks;""", """            if (c >= n_dyn) break;
            tr_dyn++;
            b0 = Bs + c * kRangeDynBlocks;""")
rep("""        uint64_t left = b1 - b0;  // blocks not yet issued""", """        uint64_t left = b1 - b0;  // blocks not yet issued
        tr_blocks += left;""")
# the end of the kernel: the last closing brace of range_flat_kernel
k = s.index("__global__ __launch_bounds__(64 * kFlatWaves) void range_flat_kernel(")
e = s.index("\n}\n", k)
s = s[:e] + """
    if (lane == 0) {
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u;
        uint64_t* r = g_range_trace + 8 * (blockIdx.x * kFlatWaves + wave);
        r[0] = tr_t0;
        r[1] = tr_ts;
        r[2] = t1;
        r[3] = (uint64_t)xcc | tr_blocks << 8 | tr_dyn << 40;
        r[4] = tr_entry;
        r[5] = tr_pub;
        r[6] = tr_fill;
        r[7] = tr_wait;
    }""" + s[e:]
rep("""constexpr int kFlatWaves = 8;""", """constexpr int kFlatWaves = 8;
__device__ uint64_t g_range_trace[8 * 8192];""")
s += """
extern "C" int cc_range_trace_read(void* dst, size_t bytes) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(cc::g_range_trace), bytes) == hipSuccess ? 0 : -1;
}
"""
open(p, "w").write(s)
