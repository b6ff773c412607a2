#!/usr/bin/env python3
"""Interleaved in-process A/B of the write-log traffic probe
(cc_apply_log_probe_dev) across libcurvecrc builds, in the bench's
partial-write shape (65,536 random 512 B-4 KiB writes over a 16 GiB pool):
per round one log is applied (in-tree build, untimed) and every build's probe
runs over that log's touched pages (idempotent right after the apply), in
alternating order, HIP events around each probe.  usage: probe_ab.py LIB.so [LIB.so ...]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from curve_amd import crc as C  # noqa: E402

argv = sys.argv[1:]
order_mode = "head"
if "--sorted" in argv:  # descriptors in page (address) order instead of head order
    order_mode = "sorted"
    argv.remove("--sorted")
args = argv
dev = torch.device("cuda", 0)
pb, U = 4096, 65536
pool = torch.empty(16 << 30, dtype=torch.uint8, device=dev).random_(0, 256)
crcs = C.page_crc(pool, pb)
src = torch.empty(U * pb, dtype=torch.uint8, device=dev).random_(0, 256)
rng = np.random.default_rng(11)
logs = []
for _ in range(8):
    dst, so, ln = rng.integers(0, pool.numel() - pb, U), rng.integers(0, U * pb - pb, U), rng.integers(512, 4097, U)
    d = C.log_probe_descs(dst, so, ln)
    if order_mode == "sorted":
        d = np.sort(d, order="page")
    logs.append((torch.from_numpy(C.log_records(dst, so, ln).view(np.uint8)).to(dev),
                 torch.from_numpy(d.view(np.uint8)).to(dev), d.size))
out = torch.empty(U * 2, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
libs = {}
for p in args:
    L = ctypes.CDLL(os.path.abspath(p))
    L.cc_apply_log_probe_dev.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    libs[p] = L


def probe(p, k):
    _, dd, n = logs[k % len(logs)]
    rc = libs[p].cc_apply_log_probe_dev(pool.data_ptr(), pool.numel(), src.data_ptr(), dd.data_ptr(), n,
                                        out.data_ptr(), ctypes.c_void_p(s.cuda_stream))
    assert rc == 0, rc


ms = {p: [] for p in libs}
order = list(libs)
for r in range(40):
    k = r % len(logs)
    C.apply_log(pool, crcs, src, logs[k][0], U, pb, pb)
    for p in (order if r % 2 == 0 else order[::-1]):
        probe(p, k)  # queued ahead
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(3):
            probe(p, k)
        e1.record(s)
        torch.cuda.synchronize()
        if r >= 4:
            ms[p].append(e0.elapsed_time(e1) / 3)
ok = bool(torch.equal(crcs, C.page_crc(pool, pb)))
for p, v in ms.items():
    print(f"probe ({order_mode} order) {os.path.basename(p)}: median {sorted(v)[len(v) // 2]:.4f} ms min {min(v):.4f} pool_consistent {ok}",
          flush=True)
