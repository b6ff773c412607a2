#!/usr/bin/env python3
"""Which HIP runtime a process ends up with, by load order: `lib` loads libcurvecrc
(through curve_amd._lib.lib()) before importing torch, `torch` the other way;
then a page-list probe and a page CRC call, and the HIP / HSA runtimes mapped.
usage: load_order_probe.py lib|torch"""
import sys, numpy as np
sys.path.insert(0, '.')
first = sys.argv[1]
if first == "lib":
    from curve_amd import _lib
    _lib.lib()
import torch
from curve_amd import crc as C
dev = torch.device("cuda", 0)
pool = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
pages = torch.arange(10, dtype=torch.int64, device=dev)
out = torch.zeros(10, dtype=torch.int32, device=dev)
try:
    C.page_list_probe(pool, pages, 10, out)
    torch.cuda.synchronize()
    print(first, "probe ok")
except Exception as e:
    print(first, "probe failed", e)
try:
    print(first, "page_crc", int(C.page_crc(pool, 4096)[0]))
except Exception as e:
    print(first, "page_crc failed", e)
import os
print(first, sorted(set(l.split()[-1] for l in open('/proc/self/maps') if 'amdhip64' in l or 'hsa-runtime' in l)))
