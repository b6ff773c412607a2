#!/usr/bin/env python3
"""Register / LDS / scratch use of the kernels in build/csrc/kernels.s (make asm),
filtered by a substring of the mangled name: kregs.py [substring ...]"""
import re
import sys

s = open("build/csrc/kernels.s").read()
pats = sys.argv[1:] or [""]
for blk in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", s, re.S):
    name, b = blk.group(1), blk.group(2)
    if not any(p in name for p in pats):
        continue
    g = lambda k: re.search(r"\." + k + r"\s+(\S+)", b).group(1)  # noqa: E731
    print(f"{name[:72]:72s} vgpr {g('amdhsa_next_free_vgpr'):>4} sgpr {g('amdhsa_next_free_sgpr'):>4} "
          f"lds {g('amdhsa_group_segment_fixed_size'):>6} scratch {g('amdhsa_private_segment_fixed_size')}")
