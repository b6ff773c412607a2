#!/usr/bin/env python3
"""A/B build: the verify-on-read kernel with THREE pages' loads in flight while
one is hashed (a ring of four register sets) instead of two.
usage: rv_depth3.py KERNELS_HIP"""
import sys

p = sys.argv[1]
s = open(p).read()
old = """            uint32_t A[M], B[M], Cq[M];
            uint32_t oA, oB, oC;
            uint64_t gA = page_at(ks, oA), gB = page_at(ks + 1 < ke ? ks + 1 : ks, oB), gC = gB;
            oC = oB;
            uint32_t sA = stored_crc(gA), sB = stored_crc(gB), sC = sB;
            load_page<M>(A, pages + gA * (64u * M));
            load_page<M>(B, pages + gB * (64u * M));
            // hash X (page k: stored CRC sx, owner lane ox); page k+2's loads go into Y
            auto step = [&](uint32_t (&X)[M], uint32_t sx, uint32_t ox, uint32_t k, uint32_t (&Y)[M], uint64_t& gy,
                            uint32_t& sy, uint32_t& oy) {
                const bool more = k + 1 < ke;
                gy = page_at(k + 2 < ke ? k + 2 : ke - 1, oy);  // clamped: same loads every step"""
new = """            uint32_t A[M], B[M], Cq[M], Dq[M];
            uint32_t oA, oB, oC, oD;
            uint64_t gA = page_at(ks, oA), gB = page_at(ks + 1 < ke ? ks + 1 : ks, oB),
                     gC = page_at(ks + 2 < ke ? ks + 2 : ke - 1, oC), gD = gC;
            oD = oC;
            uint32_t sA = stored_crc(gA), sB = stored_crc(gB), sC = stored_crc(gC), sD = sC;
            load_page<M>(A, pages + gA * (64u * M));
            load_page<M>(B, pages + gB * (64u * M));
            load_page<M>(Cq, pages + gC * (64u * M));
            auto step = [&](uint32_t (&X)[M], uint32_t sx, uint32_t ox, uint32_t k, uint32_t (&Y)[M], uint64_t& gy,
                            uint32_t& sy, uint32_t& oy) {
                const bool more = k + 1 < ke;
                gy = page_at(k + 3 < ke ? k + 3 : ke - 1, oy);  // clamped: same loads every step"""
assert s.count(old) == 1
s = s.replace(old, new)
old2 = """            for (uint32_t k = ks;; k += 3) {
                if (!step(A, sA, oA, k, Cq, gC, sC, oC)) break;
                if (!step(B, sB, oB, k + 1, A, gA, sA, oA)) break;
                if (!step(Cq, sC, oC, k + 2, B, gB, sB, oB)) break;
            }"""
new2 = """            for (uint32_t k = ks;; k += 4) {
                if (!step(A, sA, oA, k, Dq, gD, sD, oD)) break;
                if (!step(B, sB, oB, k + 1, A, gA, sA, oA)) break;
                if (!step(Cq, sC, oC, k + 2, B, gB, sB, oB)) break;
                if (!step(Dq, sD, oD, k + 3, Cq, gC, sC, oC)) break;
            }"""
assert s.count(old2) == 1
s = s.replace(old2, new2)
open(p, "w").write(s)
