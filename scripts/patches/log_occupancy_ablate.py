#!/usr/bin/env python3
"""Occupancy ablation of the write log's page pass (timing only, WRONG CRCs by
design): the 160 KiB LDS image shrunk to 8 KiB (every table lookup masked into
it, same instruction count) so that more than one workgroup fits a CU, then
WAVES waves a workgroup and BLOCKS_PER_CU workgroups a CU.  Compares 16 waves
in one workgroup (the shipped occupancy) with 2 x 10 = 20 waves, to see whether
the write log would gain from an LDS image small enough for two workgroups.
usage: log_occupancy_ablate.py KERNELS_HIP WAVES BLOCKS_PER_CU"""
import os
import sys

p, waves, bpc = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
s = open(p).read()


def rep(old, new, count=1):
    global s
    assert s.count(old) == count, (old[:70], s.count(old))
    s = s.replace(old, new)


rep("""__device__ __forceinline__ uint32_t lds_u32(const uint32_t* tab, uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(tab) + byte_addr);""",
    """__device__ __forceinline__ uint32_t lds_u32(const uint32_t* tab, uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(tab) + (byte_addr & 0x1FFCu));""")
rep("""template <int M, bool Delta>
__global__ __launch_bounds__(64 * log_waves(M, Delta)) void log_pages_kernel(LogLaunch a) {
    __shared__ uint32_t tab[kLdsBytes / 4];""", """template <int M, bool Delta>
__global__ __launch_bounds__(64 * log_waves(M, Delta), MINW) void log_pages_kernel(LogLaunch a) {
    __shared__ uint32_t tab[8192 / 4];""".replace("MINW", str(-(-waves * bpc // 4))))
# the fill: 8 KiB only
s = s.replace("fill_lds<64 * WV>(tab, static_cast<const uint4*>(a.image));",
              "{ for (uint32_t i = threadIdx.x; i < 8192 / 16; i += 64 * WV) reinterpret_cast<uint4*>(tab)[i] = static_cast<const uint4*>(a.image)[i]; __syncthreads(); }")
rep("""            hipLaunchKernelGGL((log_pages_kernel<MM, false>), dim3(a.blocks), dim3(64 * log_waves(MM, false)), 0, \\""",
    """            hipLaunchKernelGGL((log_pages_kernel<MM, false>), dim3(a.blocks * %d), dim3(64 * log_waves(MM, false)), 0, \\""" % bpc)
open(p, "w").write(s)
h = os.path.join(os.path.dirname(p), "kernels.h")
t = open(h).read()
old = "constexpr int kLogWavesFull = 16;"
assert t.count(old) == 1
t = t.replace(old, "constexpr int kLogWavesFull = %d;" % waves)
open(h, "w").write(t)
