#!/usr/bin/env python3
"""Interleaved in-process A/B of cc_verify_reads_dev across libcurvecrc builds
in the bench's read-verify shape (65,536 reads of 4-128 KiB over a 16 GiB pool,
records resident in HBM).  usage: reads_ab.py LIB.so [LIB.so ...]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from curve_amd import crc as C  # noqa: E402

dev = torch.device("cuda", 0)
pb = 4096
pool = torch.empty(16 << 30, dtype=torch.uint8, device=dev).random_(0, 256)
crcs = C.page_crc(pool, pb)
n = 65536
rng = np.random.default_rng(0xEAD)
npg = rng.integers(1, 33, n)
first = rng.integers(0, (16 << 30) // pb - 32, n)
d_reads = torch.from_numpy(np.stack([first * pb, npg * pb], axis=1).reshape(-1).astype(np.int64)).to(dev)
s = torch.cuda.current_stream()
libs = {}
for path in sys.argv[1:]:
    L = ctypes.CDLL(os.path.abspath(path))
    L.cc_verify_reads_work_bytes.restype = ctypes.c_uint64
    L.cc_verify_reads_work_bytes.argtypes = [ctypes.c_uint64]
    L.cc_verify_reads_dev.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                      ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    need = L.cc_verify_reads_work_bytes(n)
    libs[path] = (L, torch.empty(need, dtype=torch.uint8, device=dev))
bad = torch.zeros(n, dtype=torch.int32, device=dev)
total = torch.zeros(1, dtype=torch.int64, device=dev)


def call(path):
    L, work = libs[path]
    rc = L.cc_verify_reads_dev(pool.data_ptr(), pool.numel(), pb, d_reads.data_ptr(), n, crcs.data_ptr(),
                               bad.data_ptr(), total.data_ptr(), work.data_ptr(), work.numel(),
                               ctypes.c_void_p(s.cuda_stream))
    assert rc == 0, rc


for p in libs:
    call(p)
for _ in range(40):
    call(sys.argv[1])
torch.cuda.synchronize()
ms = {p: [] for p in libs}
order = list(libs)
for r in range(20):
    for p in (order if r % 2 == 0 else order[::-1]):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(3):
            call(p)
        e1.record(s)
        torch.cuda.synchronize()
        ms[p].append(e0.elapsed_time(e1) / 3)
assert int(total.item()) == 0, "clean pool flagged"
alg = float(npg.sum()) * (pb + 4)
for p, v in ms.items():
    med = sorted(v)[len(v) // 2]
    print(f"{os.path.basename(p)}: median {med:.4f} ms min {min(v):.4f} frac {alg / (med * 1e-3) / 8e12:.4f}", flush=True)
