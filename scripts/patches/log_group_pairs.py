#!/usr/bin/env python3
"""A/B build: the page kernel's tail grouping claims TWO chunks per counter
take, so half as many (the earliest-finishing) workgroups do the next batch's
inserts.  usage: log_group_pairs.py KERNELS_HIP"""
import sys

p = sys.argv[1]
s = open(p).read()
old = """    for (uint32_t r = 0; r < nx.rounds; r++) {
        if (threadIdx.x == 0) tab[T] = (uint32_t)atomicAdd(nx.take, 1ull);  // (< 2^32 chunks: n_pieces < 2^31)
        __syncthreads();
        const uint64_t c = tab[T];
        if (c >= chunks) break;  // uniform
        insert_piece(nx, c * T + threadIdx.x, tab, used);  // ends with a barrier: tab[T] free again
    }"""
new = """    for (uint32_t r = 0; r + 2 <= nx.rounds; r += 2) {
        if (threadIdx.x == 0) tab[T] = (uint32_t)atomicAdd(nx.take, 1ull);
        __syncthreads();
        const uint64_t c = 2ull * tab[T];
        if (c >= chunks) break;  // uniform
        insert_piece(nx, c * T + threadIdx.x, tab, used);
        if (c + 1 < chunks) insert_piece(nx, (c + 1) * T + threadIdx.x, tab, used);
    }"""
assert s.count(old) == 1
s = s.replace(old, new)
open(p, "w").write(s)
