#!/usr/bin/env python3
"""Variant build: kRangeTiles (kernels.h, beside the COPY of kernels.hip that
make_variant.sh passes) = N -- the range tiles the WAL and verify-on-read
kernels count, poll and search (1024 shipped; the engine's scratch follows).
A comment is added to kernels.hip so make_variant.sh sees an edit.
usage: make_variant.sh NAME py scripts/patches/range_tiles.py N"""
import os
import sys

hip, n = sys.argv[1], int(sys.argv[2])
assert n % 64 == 0 and n >= 64
h = os.path.join(os.path.dirname(hip), "kernels.h")
s = open(h).read()
old = "constexpr uint32_t kRangeTiles = 1024;"
assert s.count(old) == 1
open(h, "w").write(s.replace(old, f"constexpr uint32_t kRangeTiles = {n};"))
open(hip, "a").write(f"\n// variant: kRangeTiles = {n}\n")
