#!/usr/bin/env python3
"""Interleaved in-process A/B of cc_crc_ranges_dev across libcurvecrc builds
(arguments LIB.so@name) in the bench's WAL-replay shape (65,536 entries, data
1-128 KiB, 28-byte header, 4 KiB slots) and at one fixed entry size; all
outputs must agree entry for entry.  (It also drove the round-2 comparison of
the flat and size-sorted schedules through CC_RANGE_SCHED, since removed with
the sorted schedule; the variable is now ignored.)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from curve_amd import crc as C  # noqa: E402

dev = torch.device("cuda", 0)
pool = torch.empty(16 << 30, dtype=torch.uint8, device=dev).random_(0, 256)
L = C.lib()
s = torch.cuda.current_stream()


def shape(fixed):
    rng = np.random.default_rng(0x3A1)
    n = 65536
    real = rng.integers(1024, (128 << 10) + 1, n).astype(np.uint64)
    if fixed:
        real[:] = fixed
    slot = (28 + real + 4095) // 4096 * 4096
    offs = np.concatenate([[0], np.cumsum(slot)[:-1]]).astype(np.uint64) + 4096 + 28
    rec = np.empty((n, 2), dtype=np.uint64)
    rec[:, 0], rec[:, 1] = offs, real
    return n, torch.from_numpy(rec.view(np.uint8).reshape(-1)).to(dev), int(real.sum())


VARIANTS = sys.argv[1:] or ["flat", "sorted"]  # [LIB.so@]flat[:rounds] | [LIB.so@]sorted
LIBS = {}
for v in VARIANTS:
    if "@" in v:
        import ctypes
        path = v.split("@")[0]
        if path not in LIBS:
            LIBS[path] = ctypes.CDLL(os.path.abspath(path))
            for fn in ("cc_crc_ranges_dev",):
                getattr(LIBS[path], fn).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                    ctypes.c_void_p, ctypes.c_void_p]


def run(n, d_rec, out, variant):
    lib = LIBS[variant.split("@")[0]] if "@" in variant else L
    sched = variant.split("@")[-1]
    os.environ["CC_RANGE_SCHED"] = sched.split(":")[0]
    os.environ["CC_RANGE_ROUNDS"] = sched.split(":")[1] if ":" in sched else "1"
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    C.check(lib.cc_crc_ranges_dev(pool.data_ptr(), d_rec.data_ptr(), n, out.data_ptr(), C._stream_handle(s)),
            "cc_crc_ranges_dev")
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


for fixed in (0, 66 << 10):
    n, d_rec, nbytes = shape(fixed)
    outs = {k: torch.empty(n, dtype=torch.int32, device=dev) for k in VARIANTS}
    for k in outs:
        run(n, d_rec, outs[k], k)
    for _ in range(30):  # clock ramp after idle (the bench's trace shows ~7 slow launches)
        run(n, d_rec, outs[VARIANTS[0]], VARIANTS[0])
    same = all(bool(torch.equal(outs[k], outs[VARIANTS[0]])) for k in VARIANTS)
    ms = {k: [] for k in outs}
    for r in range(int(os.environ.get("AB_ROUNDS", "10"))):
        for k in (VARIANTS if r % 2 == 0 else VARIANTS[::-1]):
            ms[k].append(run(n, d_rec, outs[k], k))
    for k, v in ms.items():
        med = sorted(v)[len(v) // 2]
        print(sorted(round(x, 4) for x in v))
        print(f"{'fixed 66 KiB' if fixed else 'random 1-128 KiB'} {k}: median {med:.4f} ms "
              f"min {min(v):.4f} {nbytes / (med * 1e-3) / 1e9:.1f} GB/s frac {nbytes / (med * 1e-3) / 8e12:.4f}"
              f" agree {same}", flush=True)
