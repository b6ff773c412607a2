#!/usr/bin/env python3
"""Static instruction mix + register use of kernels in build/csrc/kernels.s
(make asm).  usage: asm_mix.py SUBSTRING [SUBSTRING ...]"""
import collections
import re
import sys

s = open("build/csrc/kernels.s").read()
names = re.findall(r"^(_Z\S+):(?: |$)", s, re.M)
for want in sys.argv[1:]:
    for name in [n for n in names if want in n]:
        i = s.index(name + ":")
        j = s.index(".Lfunc_end", i)
        c = collections.Counter()
        for line in s[i:j].split("\n"):
            line = line.strip()
            if not line or line.startswith((".", ";")) or line.endswith(":"):
                continue
            c[line.split()[0]] += 1
        cat = collections.Counter()
        for op, n in c.items():
            cat[op.split("_")[0]] += n
        k = s.index(".name:           " + name)
        regs = dict(re.findall(r"\.(vgpr_count|vgpr_spill_count|sgpr_spill_count):\s+(\d+)", s[k - 1200:k + 1200]))
        print(name, sum(c.values()), dict(cat.most_common(6)), regs)
