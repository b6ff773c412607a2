#!/usr/bin/env python3
"""A/B timing of libcurvecrc variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  Each variant .so is loaded with its
own ctypes handle; all run cc_page_crc_dev over the same device buffer.

usage: python scripts/ab_bench.py build/variants/libcurvecrc_*.so [--gib 16] [--rounds 7] [--reps 5]
"""
import argparse
import ctypes
import json
import os
import statistics

import torch

p = argparse.ArgumentParser()
p.add_argument("libs", nargs="+")
p.add_argument("--gib", type=float, default=16.0)
p.add_argument("--rounds", type=int, default=7)
p.add_argument("--reps", type=int, default=5)
p.add_argument("--page-bytes", type=int, default=4096)
p.add_argument("--verify", action="store_true")
a = p.parse_args()

dev = torch.device("cuda", 0)
nb = int(a.gib * (1 << 30)) // a.page_bytes * a.page_bytes
data = torch.empty(nb, dtype=torch.uint8, device=dev).random_(0, 256)
n = nb // a.page_bytes
outs, libs = {}, {}
for path in a.libs:
    L = ctypes.CDLL(os.path.abspath(path))
    L.cc_page_crc_dev.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    L.cc_page_verify_dev.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    libs[path] = L
    outs[path] = torch.empty(n, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
h = ctypes.c_void_p(s.cuda_stream)
cnt = torch.zeros(2, dtype=torch.int64, device=dev)


def launch(path):
    L = libs[path]
    if a.verify:
        rc = L.cc_page_verify_dev(ctypes.c_void_p(data.data_ptr()), n, a.page_bytes,
                                  ctypes.c_void_p(outs[path].data_ptr()), ctypes.c_void_p(cnt.data_ptr()),
                                  ctypes.c_void_p(cnt.data_ptr() + 8), h)
    else:
        rc = L.cc_page_crc_dev(ctypes.c_void_p(data.data_ptr()), n, a.page_bytes,
                               ctypes.c_void_p(outs[path].data_ptr()), h)
    assert rc == 0, rc


if a.verify:  # expected CRCs from the first variant's compute path
    L0 = libs[a.libs[0]]
    for path in a.libs:
        assert L0.cc_page_crc_dev(ctypes.c_void_p(data.data_ptr()), n, a.page_bytes,
                                  ctypes.c_void_p(outs[path].data_ptr()), h) == 0
for path in a.libs:  # warm + results
    launch(path)
for _ in range(20):  # clock ramp after idle
    launch(a.libs[0])
torch.cuda.synchronize()
ref = outs[a.libs[0]].clone()
times = {p_: [] for p_ in a.libs}
for r in range(a.rounds):
    for path in a.libs:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.reps):
            launch(path)
        e1.record(s)
        torch.cuda.synchronize()
        times[path].append(e0.elapsed_time(e1) / a.reps)
if a.verify:
    torch.cuda.synchronize()
    assert int(cnt[0]) == 0, "verify flagged clean pages"
for path in a.libs:
    same = bool(torch.equal(outs[path], ref)) if not a.verify else None
    ms = statistics.median(times[path])
    print(json.dumps({"lib": os.path.basename(path), "ms_median": round(ms, 4), "ms_min": round(min(times[path]), 4),
                      "GBps_alg": round(n * (a.page_bytes + 4) / ms / 1e6, 1), "same_as_first": same}))
