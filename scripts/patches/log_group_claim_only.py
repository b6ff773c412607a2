#!/usr/bin/env python3
"""Timing ablation (WRONG results by design): the page kernel's tail grouping
keeps its barrier and its one claim round trip per workgroup but inserts
nothing, so every other page kernel of a queue has no heads.  Compared by page
kernel duration (the full ones) with the shipped tail grouping, it splits the
grouping's cost into the claim itself and the inserts.  usage: log_group_claim_only.py KERNELS_HIP"""
import sys

p = sys.argv[1]
s = open(p).read()
old = """        if (c >= chunks) break;  // uniform
        insert_piece(nx, c * T + threadIdx.x, tab, used);"""
assert s.count(old) == 1
s = s.replace(old, """        if (c >= chunks || true) break;  // ablation: claim, never insert
        insert_piece(nx, c * T + threadIdx.x, tab, used);""")
open(p, "w").write(s)
