#!/usr/bin/env python3
"""Minimal driver for rocprofv3 passes over the page kernels: N compute launches
and N verify launches over a device-resident pool (default 1024 x 16 MiB)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from curve_amd import crc as C  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--gib", type=float, default=16.0)
p.add_argument("--n", type=int, default=3)
a = p.parse_args()
dev = torch.device("cuda", 0)
nb = int(a.gib * (1 << 30)) // 4096 * 4096
d = torch.empty(nb, dtype=torch.uint8, device=dev).random_(0, 256)
out = torch.empty(nb // 4096, dtype=torch.int32, device=dev)
for _ in range(a.n):
    C.page_crc(d, 4096, out=out)
for _ in range(a.n):
    cnt = C.page_verify(d, out, 4096)
torch.cuda.synchronize()
assert int(cnt[0]) == 0
print("ok", nb, "bytes x", a.n)
