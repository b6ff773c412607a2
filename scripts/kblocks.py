#!/usr/bin/env python3
"""Basic blocks of one kernel in build/csrc/kernels.s (make asm) with their
instruction mix: kblocks.py SUBSTRING [FIRST_LINE LAST_LINE]"""
import collections
import re
import sys

s = open("build/csrc/kernels.s").read()
m = [m for m in re.finditer(r"\n(_Z\S+):\s*;.*?\n(.*?)\n\.Lfunc_end", s, re.S) if sys.argv[1] in m.group(1)][0]
lines = [l.strip() for l in m.group(2).split("\n")]


def cat(op):
    if op.startswith(("s_waitcnt", "s_nop")):
        return op[:9]
    if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
        return "lane"
    if op.startswith("s_"):
        return "S"
    if op.startswith("v_"):
        return "V"
    if op.startswith(("buffer_", "global_", "scratch_")):
        return "M"
    if op.startswith("ds_"):
        return "L"
    return op


blk, name = collections.Counter(), "entry"
start = 0
lo = int(sys.argv[2]) if len(sys.argv) > 2 else 0
hi = int(sys.argv[3]) if len(sys.argv) > 3 else len(lines)
for i, l in enumerate(lines + [".LBBend:"]):
    if re.match(r"\.LBB\d+_\d+:|\.LBBend:", l):
        if lo <= start < hi and sum(blk.values()):
            print(f"{start:5d} {name:14s} n={sum(blk.values()):4d} " + " ".join(f"{k}={v}" for k, v in sorted(blk.items())))
        blk, name, start = collections.Counter(), l.split(":")[0], i
        continue
    if not l or l.startswith((";", ".")):
        continue
    blk[cat(l.split()[0])] += 1
