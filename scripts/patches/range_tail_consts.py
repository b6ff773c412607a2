#!/usr/bin/env python3
"""WAL range kernel tail constants for a variant build: DIV (1/DIV of the blocks dynamic), HEADS (tail counters, per XCD when 8), BLOCKS (blocks per dynamic chunk).  usage: range_tail_consts.py KERNELS_HIP DIV HEADS BLOCKS"""
import sys
p=sys.argv[1]; div=sys.argv[2]; heads=sys.argv[3]; blk=sys.argv[4]
s=open(p).read()
def rep(o,n):
    global s
    assert s.count(o)==1,o
    s=s.replace(o,n)
rep("constexpr uint64_t kRangeDynDiv = 32;", "constexpr uint64_t kRangeDynDiv = %s;" % div)
rep("constexpr uint32_t kRangeHeads = 1;", "constexpr uint32_t kRangeHeads = %s;" % heads)
rep("constexpr uint64_t kRangeDynBlocks = 16;", "constexpr uint64_t kRangeDynBlocks = %s;" % blk)
open(p,'w').write(s)
