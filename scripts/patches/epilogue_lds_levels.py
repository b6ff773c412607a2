#!/usr/bin/env python3
"""A/B build of the fused scan epilogue (NOT the shipped kernel): the in-wave
combine levels 0-5 look up their product tables in LDS (copied with the Horner
table: 28 KiB a block) instead of global memory, and thread 0 loads the
chunk's metapage CRC, copyset and shift before the fold, not after.
usage: epilogue_lds_levels.py KERNELS_HIP"""
import sys

p = sys.argv[1]
s = open(p).read()


def rep(old, new):
    global s
    assert s.count(old) == 1, old[:80]
    s = s.replace(old, new, 1)


rep("""    __shared__ uint32_t mt[1024];  // x^(8 page_bytes) product table (Horner), copied once per block
    __shared__ uint32_t part[4];
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    for (uint32_t i = t; i < 1024; i += 256) mt[i] = a.mtab[i];
    __syncthreads();""", """    __shared__ uint32_t mt[7 * 1024];  // Horner table + combine levels 0..5, copied once per block
    __shared__ uint32_t part[4];
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    for (uint32_t i = t; i < 7 * 1024; i += 256) mt[i] = a.mtab[i];
    __syncthreads();""")
rep("""        const uint32_t* p = a.page_crcs + c * a.pages_per_chunk + (uint64_t)t * a.q;""",
    """        const uint32_t* p = a.page_crcs + c * a.pages_per_chunk + (uint64_t)t * a.q;
        uint32_t meta = 0, grp = 0, aft = 0;
        if (t == 0) {
            meta = a.meta_crcs[c];
            if (a.digest) {
                grp = a.group[c];
                aft = a.after_mult[c];
            }
        }""")
rep("""            if ((lane & ((2u << k) - 1u)) == 0) s = mul_tab(lvl + 1024 * k, s) ^ other;""",
    """            if ((lane & ((2u << k) - 1u)) == 0) s = mul_tab(mt + 1024 * (k + 1), s) ^ other;""")
rep("""            const uint32_t file = mul_tab(chk, a.meta_crcs[c]) ^ data;
            if (a.file_crcs) a.file_crcs[c] = file;
            if (a.digest) atomicXor(a.digest + a.group[c], mulmod_dev(a.after_mult[c], file));""",
    """            const uint32_t file = mul_tab(chk, meta) ^ data;
            if (a.file_crcs) a.file_crcs[c] = file;
            if (a.digest) atomicXor(a.digest + grp, mulmod_dev(aft, file));""")
open(p, "w").write(s)
