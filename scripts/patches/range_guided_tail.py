#!/usr/bin/env python3
"""Variant build: the WAL / range kernel's dynamic tail in two chunk sizes -- the
tail's first part in kRangeDynBlocks-block chunks (16, shipped), its last 1/DIV
in SMALL-block chunks, so the last chunks a wave takes are short and the waves
end closer together (the round-6 trace: waves end over ~30 us, a 16-block chunk
is ~19 us of one wave's work).
usage: make_variant.sh NAME py scripts/patches/range_guided_tail.py SMALL DIV"""
import sys

hip, small, div = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
s = open(hip).read()
old_n = "    const uint64_t n_dyn = (B - Bs + kRangeDynBlocks - 1) / kRangeDynBlocks;\n"
new_n = (f"    const uint64_t Dsm = (B - Bs) / {div}, Bbig = B - Dsm;  // small chunks over [Bbig, B)\n"
         "    const uint64_t n_big = (Bbig - Bs + kRangeDynBlocks - 1) / kRangeDynBlocks;\n"
         f"    const uint64_t n_dyn = n_big + (Dsm + {small} - 1) / {small};\n")
old_b = ("            b0 = Bs + c * kRangeDynBlocks;\n"
         "            b1 = b0 + kRangeDynBlocks < B ? b0 + kRangeDynBlocks : B;\n")
new_b = ("            if (c < n_big) {\n"
         "                b0 = Bs + c * kRangeDynBlocks;\n"
         "                b1 = b0 + kRangeDynBlocks < Bbig ? b0 + kRangeDynBlocks : Bbig;\n"
         "            } else {\n"
         f"                b0 = Bbig + (c - n_big) * {small};\n"
         f"                b1 = b0 + {small} < B ? b0 + {small} : B;\n"
         "            }\n")
assert s.count(old_n) == 1 and s.count(old_b) == 1
s = s.replace(old_n, new_n).replace(old_b, new_b)
open(hip, "w").write(s)
