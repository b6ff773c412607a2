#!/usr/bin/env python3
"""A/B build of range_flat_kernel (NOT the shipped kernel): a guided dynamic
tail -- the first part of the tail in kRangeDynBlocks-block chunks, the last
1/FRAC of it in SMALL-block chunks, so the final pulls even out finer.
usage: range_guided_tail.py KERNELS_HIP FRAC SMALL"""
import sys

p, frac, small = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
s = open(p).read()


def rep(old, new):
    global s
    assert s.count(old) == 1, old[:80]
    s = s.replace(old, new, 1)


rep("""    const uint64_t n_dyn = (B - Bs + kRangeDynBlocks - 1) / kRangeDynBlocks;""",
    f"""    // guided tail: big chunks first, the last 1/{frac} of the tail in {small}-block chunks
    const uint64_t Bd = B - Bs, Bsmall = Bd / {frac}, Bbig = Bd - Bsmall;
    const uint64_t n_big = (Bbig + kRangeDynBlocks - 1) / kRangeDynBlocks;
    const uint64_t n_dyn = n_big + (Bsmall + {small} - 1) / {small};""")
rep("""            b0 = Bs + c * kRangeDynBlocks;
            b1 = b0 + kRangeDynBlocks < B ? b0 + kRangeDynBlocks : B;""",
    f"""            if (c < n_big) {{
                b0 = Bs + c * kRangeDynBlocks;
                b1 = b0 + kRangeDynBlocks < Bs + Bbig ? b0 + kRangeDynBlocks : Bs + Bbig;
            }} else {{
                b0 = Bs + Bbig + (c - n_big) * {small};
                b1 = b0 + {small} < B ? b0 + {small} : B;
            }}""")
open(p, "w").write(s)
