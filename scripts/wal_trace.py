#!/usr/bin/env python3
"""Per-wave timeline of range_flat_kernel in the bench's WAL-replay shape, from a
trace build (scripts/patches/range_trace.py; never the shipped library): when each
wave enters the kernel, starts its first item, leaves its static pieces and ends,
by XCD (times from the earliest entry), and the prologue's parts (tile counts,
LDS fill, the wait for every tile count).
usage: wal_trace.py LIB.so [--calls N]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), sys.argv[1])
calls = int(sys.argv[sys.argv.index("--calls") + 1]) if "--calls" in sys.argv else 3
L = ctypes.CDLL(lib)
L.cc_crc_ranges_dev.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
L.cc_range_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
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
res = []
for c in range(40 + calls):
    assert L.cc_crc_ranges_dev(pool.data_ptr(), d_rec.data_ptr(), n, out.data_ptr(), ctypes.c_void_p(s.cuda_stream)) == 0
    if c < 40:
        continue
    torch.cuda.synchronize()
    buf = np.zeros(8 * 8192, dtype=np.uint64)
    assert L.cc_range_trace_read(buf.ctypes.data, buf.nbytes) == 0
    t = buf.reshape(-1, 8)
    t = t[t[:, 2] != 0]
    t0 = t[:, 4].min()
    entry = (t[:, 4] - t0) / 100.0
    start = (t[:, 0] - t0) / 100.0  # us
    stat = (t[:, 1].astype(np.int64) - t0) / 100.0
    end = (t[:, 2] - t0) / 100.0
    xcc = (t[:, 3] & 15).astype(int)
    blocks = ((t[:, 3] >> 8) & ((1 << 32) - 1)).astype(np.int64)
    dyn = (t[:, 3] >> 40).astype(np.int64)
    q = lambda a: [round(float(x), 1) for x in np.percentile(a, [0, 1, 50, 99, 100])]
    per_x = {int(x): {"waves": int((xcc == x).sum()), "static_end_p50": round(float(np.median(stat[xcc == x])), 1),
                      "end_p50": round(float(np.median(end[xcc == x])), 1), "end_max": round(float(end[xcc == x].max()), 1),
                      "dyn_chunks": int(dyn[xcc == x].sum()),
                      "us_per_block_static": round(float(np.median((stat[xcc == x] - start[xcc == x]) /
                                                                   np.maximum(blocks[xcc == x] - 16 * dyn[xcc == x], 1))), 3)}
             for x in sorted(set(xcc))}
    res.append({"call": c - 40, "waves": int(len(t)), "entry_us_p0_1_50_99_100": q(entry),
                "prologue_us": q(start - entry), "count_us": q((t[:, 5] - t[:, 4]) / 100.0),
                "fill_us": q((t[:, 6] - t[:, 5]) / 100.0), "tile_wait_us": q((t[:, 7] - t[:, 6]) / 100.0),
                "search_us": q((t[:, 0].astype(np.int64) - t[:, 7].astype(np.int64)) / 100.0),
                "wait_done_us": q((t[:, 7] - t0) / 100.0), "start_us_p0_1_50_99_100": q(start),
                "static_end_us": q(stat), "end_us": q(end), "blocks_per_wave": q(blocks), "dyn_chunks_per_wave": q(dyn),
                "per_xcc": per_x})
print(json.dumps(res, indent=1))
