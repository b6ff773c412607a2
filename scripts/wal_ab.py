#!/usr/bin/env python3
"""Interleaved in-process A/B of cc_crc_ranges_dev across libcurvecrc builds, in
the bench's WAL-replay shape (65,536 entries, data 1-128 KiB, 4 KiB-aligned slots
after a 28-byte header, over a 16 GiB pool).  Each build gets its own ctypes
handle; rounds alternate the order; every build's output is compared with the
first build's on every round.  usage: wal_ab.py [--fixed BYTES] LIB.so [LIB.so ...]
(--fixed: every entry that many data bytes, the balance probe of equal sizes)"""
import ctypes
import os
import sys

import numpy as np
import torch

argv = sys.argv[1:]
fixed = 0
if "--fixed" in argv:
    i = argv.index("--fixed")
    fixed = int(argv[i + 1])
    del argv[i:i + 2]
args = [x for x in argv if not x.startswith("--")]
dev = torch.device("cuda", 0)
pool = torch.empty(16 << 30, dtype=torch.uint8, device=dev).random_(0, 256)
rng = np.random.default_rng(0x3A1)
n = 65536
real = rng.integers(1024, (128 << 10) + 1, n).astype(np.uint64)
if fixed:
    real[:] = fixed
slot = (28 + real + 4095) // 4096 * 4096
offs = np.concatenate([[0], np.cumsum(slot)[:-1]]).astype(np.uint64) + 4096 + 28
rec = np.empty((n, 2), dtype=np.uint64)
rec[:, 0], rec[:, 1] = offs, real
d_rec = torch.from_numpy(rec.view(np.uint8).reshape(-1)).to(dev)
s = torch.cuda.current_stream()
libs = {}
for path in args:
    L = ctypes.CDLL(os.path.abspath(path))
    L.cc_crc_ranges_dev.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                    ctypes.c_void_p]
    libs[path] = (L, torch.empty(n, dtype=torch.int32, device=dev))


def call(path):
    L, out = libs[path]
    rc = L.cc_crc_ranges_dev(pool.data_ptr(), d_rec.data_ptr(), n, out.data_ptr(), ctypes.c_void_p(s.cuda_stream))
    assert rc == 0, rc


for p in libs:
    call(p)
for _ in range(200):  # ~130 ms of sustained load: clocks up
    call(args[0])
torch.cuda.synchronize()
ms = {p: [] for p in libs}
same = {p: True for p in libs}
order = list(libs)
data_bytes = float(real.sum())
for r in range(30):
    for p in (order if r % 2 == 0 else order[::-1]):
        call(p)  # queued ahead: the timed calls start behind work
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(4):
            call(p)
        e1.record(s)
        torch.cuda.synchronize()
        ms[p].append(e0.elapsed_time(e1) / 4)
    for p in libs:
        same[p] &= bool(torch.equal(libs[p][1], libs[order[0]][1]))
for p, v in ms.items():
    med = sorted(v)[len(v) // 2]
    print(f"wal{' fixed %d' % fixed if fixed else ''} {os.path.basename(p)}: median {med:.4f} ms min {min(v):.4f} mean {np.mean(v):.4f} "
          f"frac {(data_bytes + 4 * n) / (med * 1e-3) / 8e12:.4f} same_as_first {same[p]}", flush=True)
