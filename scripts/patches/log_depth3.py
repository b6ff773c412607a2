#!/usr/bin/env python3
"""A/B build: the write log's page pass with THREE register sets -- pages k+1
and k+2 loading while page k is merged, stored and hashed -- instead of two.
(Round 3 measured a third page slower when it cost the kernel 4 of its 16
waves; since round 4 the full-mode kernel holds 100 VGPRs, so a third set of
16 + 6 fits the 128 that 16 waves allow.)
usage: log_depth3.py KERNELS_HIP"""
import sys

p = sys.argv[1]
s = open(p).read()


def rep(old, new):
    global s
    assert s.count(old) == 1, (old[:80], s.count(old))
    s = s.replace(old, new)


rep("""        uint32_t A[M], B[M];
        constexpr bool kRowSel = !Delta;""", """        uint32_t A[M], B[M], C3[M];
        constexpr bool kRowSel = !Delta;""")
rep("""        Src S0, S1;""", """        Src S0, S1, S2;""")
rep("""            const uint32_t h1 = more ? hh + 1 : hh;
            pgy = __builtin_amdgcn_readlane(key, h1);
            py = head_piece(h1);
            load_next(Y, py, pgy, h1, ocy);""", """            const uint32_t h1 = hh + 2 < cnt ? hh + 2 : cnt - 1;  // two pages ahead (clamped)
            pgy = __builtin_amdgcn_readlane(key, h1);
            py = head_piece(h1);
            load_next(Y, py, pgy, h1, ocy);""")
rep("""        uint32_t pgA = __builtin_amdgcn_readlane(key, 0), pgB = pgA;
        uint32_t ocA = 0, ocB = 0;
        Piece pA = head_piece(0), pB = pA;
        load_next(A, pA, pgA, 0, ocA);
        fetch(S0, pA);
        for (uint32_t h = 0;; h += 2) {
            if (!step(A, S0, pA, pgA, h, ocA, B, S1, pB, pgB, ocB)) break;
            if (!step(B, S1, pB, pgB, h + 1, ocB, A, S0, pA, pgA, ocA)) break;
        }""", """        const uint32_t one = cnt > 1 ? 1u : 0u;
        uint32_t pgA = __builtin_amdgcn_readlane(key, 0), pgB = __builtin_amdgcn_readlane(key, one), pgC = pgB;
        uint32_t ocA = 0, ocB = 0, ocC = 0;
        Piece pA = head_piece(0), pB = head_piece(one), pC = pB;
        load_next(A, pA, pgA, 0, ocA);
        fetch(S0, pA);
        load_next(B, pB, pgB, one, ocB);
        fetch(S1, pB);
        for (uint32_t h = 0;; h += 3) {
            if (!step(A, S0, pA, pgA, h, ocA, C3, S2, pC, pgC, ocC)) break;
            if (!step(B, S1, pB, pgB, h + 1, ocB, A, S0, pA, pgA, ocA)) break;
            if (!step(C3, S2, pC, pgC, h + 2, ocC, B, S1, pB, pgB, ocB)) break;
        }""")
open(p, "w").write(s)
