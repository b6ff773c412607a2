#!/usr/bin/env python3
"""Verify-on-read tail constants for a variant build: DIV (1/DIV of the slots dynamic), HEADS
(tail counters, per XCD when 8), SLOTS (pages per dynamic chunk).
usage: rv_tail_consts.py KERNELS_HIP DIV HEADS SLOTS"""
import sys

p, div, heads, slots = sys.argv[1:5]
s = open(p).read()


def rep(o, n):
    global s
    assert s.count(o) == 1, o
    s = s.replace(o, n)


rep("constexpr uint64_t kRvDynDiv = 16;", "constexpr uint64_t kRvDynDiv = %s;" % div)
rep("constexpr uint32_t kRvHeads = 1;", "constexpr uint32_t kRvHeads = %s;" % heads)
rep("constexpr uint64_t kRvDynSlots = 32;", "constexpr uint64_t kRvDynSlots = %s;" % slots)
open(p, "w").write(s)
