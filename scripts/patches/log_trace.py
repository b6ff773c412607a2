#!/usr/bin/env python3
"""Timing-trace build of log_pages_kernel (NOT the shipped kernel): patches a COPY
of kernels.hip so lane 0 of every wave records, with s_memrealtime (100 MHz), the
time its LDS fill ends and the time it ends, its XCD, the pages it rehashed and
the tails it took from other waves, into a __device__ array read back by
cc_log_trace_read().  (The round-4 one-launch write log, scripts/patches/
log_fused_r04.diff, was traced the same way: profiles/write_log_fused_ab_r04.txt.)
usage: log_trace.py KERNELS_HIP   (scripts/log_trace.py runs it)"""
import sys

p = sys.argv[1]
s = open(p).read()


def rep(old, new):
    global s
    assert s.count(old) == 1, old[:80]
    s = s.replace(old, new, 1)


rep("""    fill_lds<64 * WV>(tab, static_cast<const uint4*>(a.image));
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);""", """    fill_lds<64 * WV>(tab, static_cast<const uint4*>(a.image));
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t tr0 = __builtin_amdgcn_s_memrealtime();
    uint32_t tr_pages = 0, tr_steals = 0;""")
rep("""            if (lane == 0) a.page_crcs[pg] = crc;
            return more;""", """            if (lane == 0) a.page_crcs[pg] = crc;
            tr_pages++;
            return more;""")
rep("""            if (!step(B, S1, pB, pgB, h + 1, ocB, A, S0, pA, pgA, ocA)) break;
        }
    }
    group_next<WV>(a.nx, tab);
}""", """            if (!step(B, S1, pB, pgB, h + 1, ocB, A, S0, pA, pgA, ocA)) break;
        }
    }
    if (lane == 0) {
        uint64_t* tr = g_log_trace + 8 * (blockIdx.x * WV + wave);
        tr[0] = tr0;
        tr[1] = tr0;
        tr[2] = tr0;
        tr[3] = tr0;
        tr[4] = __builtin_amdgcn_s_memrealtime();
        tr[5] = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u;
        tr[6] = tr_pages;
        tr[7] = tr_steals;
    }
    group_next<WV>(a.nx, tab);
}""")
rep("""__device__ __forceinline__ uint32_t page_hash(""", """__device__ uint64_t g_log_trace[8 * 8192];
__device__ __forceinline__ uint32_t page_hash(""")
s += """
extern "C" int cc_log_trace_read(void* dst, size_t bytes) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(cc::g_log_trace), bytes) == hipSuccess ? 0 : -1;
}
"""
open(p, "w").write(s)
