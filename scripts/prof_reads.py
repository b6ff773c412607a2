#!/usr/bin/env python3
"""Drive cc_verify_reads_dev alone (bench leg shape: 65,536 random page-aligned
reads of 4-128 KiB over a 16 GiB pool, reads resident on the device) for
rocprofv3 traces and library A/B (--lib)."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from curve_amd import crc as C  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--gib", type=int, default=16)
p.add_argument("--reads", type=int, default=65536)
p.add_argument("--reps", type=int, default=8)
p.add_argument("--lib", default=None, help="libcurvecrc variant to load instead of the in-tree one")
a = p.parse_args()
if a.lib:
    from curve_amd import _lib
    # relative to the repo root (the profilers run these from /tmp)
    _lib.LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), a.lib)
dev = torch.device("cuda", 0)
pb = 4096
pool = torch.empty(a.gib << 30, dtype=torch.uint8, device=dev).random_(0, 256)
crcs = C.page_crc(pool, pb)
n_pages = pool.numel() // pb
rng = np.random.default_rng(0xEAD)
bad = torch.zeros(a.reads, dtype=torch.int32, device=dev)
total = torch.zeros(1, dtype=torch.int64, device=dev)
s = torch.cuda.current_stream()
ms, pages = [], 0
for k in range(a.reps + 1):
    npg = rng.integers(1, 33, a.reads)
    first = rng.integers(0, n_pages - 32, a.reads)
    d = torch.from_numpy(np.stack([first * pb, npg * pb], axis=1).reshape(-1).astype(np.int64)).to(dev)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    C.verify_read_records(pool, crcs, d, a.reads, bad, total, pb)
    e1.record(s)
    torch.cuda.synchronize()
    if k:
        ms.append(e0.elapsed_time(e1))
        pages += int(npg.sum())
ok = int(total.item()) == 0
med = sorted(ms)[len(ms) // 2]
print("verify_reads ms per batch:", [round(x, 4) for x in ms], "median", round(med, 4),
      "GiB/s", round(pages / len(ms) * pb / 2**30 / (med * 1e-3), 1), "clean", ok)
