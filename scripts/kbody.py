#!/usr/bin/env python3
"""Instruction census of one kernel in build/csrc/kernels.s (make asm):
kbody.py SUBSTRING [--grep PATTERN]  -> counts by class, optionally the matching lines"""
import re
import sys

s = open("build/csrc/kernels.s").read()
pat = sys.argv[1]
g = sys.argv[sys.argv.index("--grep") + 1] if "--grep" in sys.argv else None
for m in re.finditer(r"\n(_Z\S+):\s*;.*?\n(.*?)\n\.Lfunc_end", s, re.S):
    if pat not in m.group(1):
        continue
    body = [l.strip() for l in m.group(2).split("\n") if l.strip() and not l.strip().startswith((";", "."))]
    ins = [l for l in body if not l.endswith(":")]
    cls = {}
    for l in ins:
        op = l.split()[0]
        k = op.split("_")[0] + "_" + (op.split("_")[1] if "_" in op else "")
        cls[k] = cls.get(k, 0) + 1
    print(m.group(1)[:80], "instructions", len(ins))
    print("  ", sorted(cls.items(), key=lambda x: -x[1])[:14])
    if g:
        for i, l in enumerate(body):
            if re.search(g, l):
                print("   ", i, l)
