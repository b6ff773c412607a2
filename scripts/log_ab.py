#!/usr/bin/env python3
"""Interleaved in-process A/B of the write-log call (cc_apply_log_dev, and the
delta variant with --delta) across libcurvecrc builds, in the bench's
partial-write shape: 65,536 random 512 B-4 KiB writes over a 16 GiB pool.
Each build gets its own ctypes handle and work buffer; every build is then
checked once: after one more batch, the stored CRCs equal a fresh rehash.
usage: log_ab.py [--delta] [--n WRITES] LIB.so [LIB.so ...]   (--n: writes per log, default 65,536)"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from curve_amd import crc as C  # noqa: E402

argv = sys.argv[1:]
n_arg = None
if "--n" in argv:
    i = argv.index("--n")
    n_arg = int(argv[i + 1])
    del argv[i:i + 2]
args = [x for x in argv if not x.startswith("--")]
delta = "--delta" in sys.argv
fn = "cc_apply_log_delta_dev" if delta else "cc_apply_log_dev"
dev = torch.device("cuda", 0)
pb, U = 4096, n_arg or 65536
pool = torch.empty(16 << 30, dtype=torch.uint8, device=dev).random_(0, 256)
crcs = C.page_crc(pool, pb)
src = torch.empty(U * pb, dtype=torch.uint8, device=dev).random_(0, 256)
rng = np.random.default_rng(7)
logs = []
for _ in range(8):
    rec = C.log_records(rng.integers(0, pool.numel() - pb, U), rng.integers(0, U * pb - pb, U),
                        rng.integers(512, 4097, U))
    logs.append(torch.from_numpy(rec.view(np.uint8)).to(dev))
s = torch.cuda.current_stream()
libs = {}
for path in args:
    L = ctypes.CDLL(os.path.abspath(path))
    L.cc_apply_log_work_bytes.restype = ctypes.c_uint64
    L.cc_apply_log_work_bytes.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]
    getattr(L, fn).argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                               ctypes.c_void_p]
    need = L.cc_apply_log_work_bytes(U, pb, pb)
    libs[path] = (L, torch.empty(need, dtype=torch.uint8, device=dev))


def call(path, k):
    L, work = libs[path]
    rc = getattr(L, fn)(pool.data_ptr(), pool.numel(), pb, src.data_ptr(), logs[k % len(logs)].data_ptr(), U, pb,
                        crcs.data_ptr(), work.data_ptr(), work.numel(), ctypes.c_void_p(s.cuda_stream))
    assert rc == 0, rc


for p in libs:
    call(p, 0)
for k in range(60):
    call(args[0], k)
torch.cuda.synchronize()
ms = {p: [] for p in libs}
order = list(libs)
k = 0
for r in range(24):
    for p in (order if r % 2 == 0 else order[::-1]):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(4):
            call(p, k)
            k += 1
        e1.record(s)
        torch.cuda.synchronize()
        ms[p].append(e0.elapsed_time(e1) / 4)
ok = {}
for p in libs:
    call(p, k)
    k += 1
    ok[p] = bool(torch.equal(crcs, C.page_crc(pool, pb)))
for p, v in ms.items():
    med = sorted(v)[len(v) // 2]
    print(f"{'delta' if delta else 'full'} n={U} {os.path.basename(p)}: median {med:.4f} ms min {min(v):.4f} "
          f"crcs_consistent {ok[p]}", flush=True)
