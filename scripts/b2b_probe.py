#!/usr/bin/env python3
"""Diagnostic: per-call event times of cc_crc_ranges_dev in the bench's WAL
shape, synchronised between calls vs enqueued back to back."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from curve_amd import crc as C  # noqa: E402

dev = torch.device("cuda", 0)
pool = torch.empty(16 << 30, dtype=torch.uint8, device=dev).random_(0, 256)
rng = np.random.default_rng(0x3A1)
n = 65536
real = rng.integers(1024, (128 << 10) + 1, n).astype(np.uint64)
slot = (28 + real + 4095) // 4096 * 4096
offs = np.concatenate([[0], np.cumsum(slot)[:-1]]).astype(np.uint64) + 4096 + 28
rec = np.empty((n, 2), dtype=np.uint64)
rec[:, 0], rec[:, 1] = offs, real
d_rec = torch.from_numpy(rec.view(np.uint8).reshape(-1)).to(dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
L = C.lib()


def call():
    C.check(L.cc_crc_ranges_dev(pool.data_ptr(), d_rec.data_ptr(), n, out.data_ptr(), C._stream_handle(s)), "x")


for _ in range(30):
    call()
for mode in ("sync", "b2b", "sync", "b2b"):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(12)]
    for e0, e1 in ev:
        e0.record(s)
        call()
        e1.record(s)
        if mode == "sync":
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    ms = [round(a.elapsed_time(b), 4) for a, b in ev]
    gaps = [round(ev[i][1].elapsed_time(ev[i + 1][0]), 4) for i in range(len(ev) - 1)]
    print(mode, "ms", ms, "mean", round(float(np.mean(ms)), 4), "gaps", gaps[:6], flush=True)
