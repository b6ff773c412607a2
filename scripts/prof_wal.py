#!/usr/bin/env python3
"""Drive cc_crc_ranges_dev alone in the bench's WAL-replay shape (65,536 entries,
data 1-128 KiB, 4 KiB-aligned slots after a 28-byte header, over a 16 GiB pool)
for rocprofv3 traces and library A/B (--lib)."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from curve_amd import crc as C  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--gib", type=int, default=16)
p.add_argument("--entries", type=int, default=65536)
p.add_argument("--reps", type=int, default=8)
p.add_argument("--lib", default=None, help="libcurvecrc variant to load instead of the in-tree one")
p.add_argument("--fixed", type=int, default=0, help="every entry this many bytes (balance probe)")
p.add_argument("--sorted", action="store_true", help="entries in decreasing size order (balance probe)")
a = p.parse_args()
if a.lib:
    from curve_amd import _lib
    # relative to the repo root (the profilers run these from /tmp)
    _lib.LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), a.lib)
dev = torch.device("cuda", 0)
pool = torch.empty(a.gib << 30, dtype=torch.uint8, device=dev).random_(0, 256)
rng = np.random.default_rng(0x3A1)
n = a.entries
real = rng.integers(1024, (128 << 10) + 1, n).astype(np.uint64)
if a.fixed:
    real[:] = a.fixed
if a.sorted:
    real = np.sort(real)[::-1].copy()
slot = (28 + real + 4095) // 4096 * 4096
start = np.concatenate([[0], np.cumsum(slot)[:-1]]).astype(np.uint64) + 4096
offs = start + 28
rec = np.empty((n, 2), dtype=np.uint64)
rec[:, 0], rec[:, 1] = offs, real
d_rec = torch.from_numpy(rec.view(np.uint8).reshape(-1)).to(dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
L = C.lib()
s = torch.cuda.current_stream()
ms = []
for k in range(a.reps + 1):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    C.check(L.cc_crc_ranges_dev(pool.data_ptr(), d_rec.data_ptr(), n, out.data_ptr(), C._stream_handle(s)),
            "cc_crc_ranges_dev")
    e1.record(s)
    torch.cuda.synchronize()
    if k:
        ms.append(e0.elapsed_time(e1))
got = C.as_u32(out)
ok = all(int(got[i]) == C.CRC32(pool[int(offs[i]):int(offs[i] + real[i])].cpu().numpy().tobytes())
         for i in (0, 1, n // 2, n - 1))
med = sorted(ms)[len(ms) // 2]
print("crc_ranges ms per batch:", [round(x, 4) for x in ms], "median", round(med, 4),
      "GB/s", round(float(real.sum()) / (med * 1e-3) / 1e9, 1), "spot_ok", ok)
