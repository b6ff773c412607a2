#!/usr/bin/env python3
"""A/B build: the page kernel's tail grouping claims K chunks per counter take
(K = 1 shipped), so fewer, earlier-finishing workgroups do the next batch's
inserts.  usage: log_group_k.py KERNELS_HIP K"""
import sys

p, k = sys.argv[1], int(sys.argv[2])
s = open(p).read()
old = """    for (uint32_t r = 0; r < nx.rounds; r++) {
        if (threadIdx.x == 0) tab[T] = (uint32_t)atomicAdd(nx.take, 1ull);  // (< 2^32 chunks: n_pieces < 2^31)
        __syncthreads();
        const uint64_t c = tab[T];
        if (c >= chunks) break;  // uniform
        insert_piece(nx, c * T + threadIdx.x, tab, used);  // ends with a barrier: tab[T] free again
    }"""
new = """    for (uint32_t r = 0; r + K <= nx.rounds; r += K) {
        if (threadIdx.x == 0) tab[T] = (uint32_t)atomicAdd(nx.take, 1ull);
        __syncthreads();
        const uint64_t c = (uint64_t)K * tab[T];
        if (c >= chunks) break;  // uniform
        for (uint32_t i = 0; i < K && c + i < chunks; i++) insert_piece(nx, (c + i) * T + threadIdx.x, tab, used);
    }""".replace("K", str(k))
assert s.count(old) == 1
s = s.replace(old, new)
open(p, "w").write(s)
