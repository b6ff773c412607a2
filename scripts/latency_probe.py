#!/usr/bin/env python3
"""Small-batch latency of the device calls a chunkserver makes per request:
verify-on-read for 1 / 16 / 256 reads, the write log for 1 / 16 / 256 writes,
and page CRCs of one 16 MiB chunk -- device time per call (HIP events around
back-to-back calls, records already resident) over a 16 GiB pool."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from curve_amd import _lib, crc as C  # noqa: E402

if len(sys.argv) > 1:  # a libcurvecrc variant to load instead of the in-tree one
    _lib.LIB_PATH = os.path.abspath(sys.argv[1])

dev = torch.device("cuda", 0)
pb = 4096
pool = torch.empty(16 << 30, dtype=torch.uint8, device=dev).random_(0, 256)
crcs = C.page_crc(pool, pb)
src = torch.empty(1 << 24, dtype=torch.uint8, device=dev).random_(0, 256)
s = torch.cuda.current_stream()
rng = np.random.default_rng(5)


def timed(fn, reps=50):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps * 1e3, 1)  # us


out = {}
for n in (1, 16, 256, 1024, 8192):
    first = rng.integers(0, (16 << 30) // pb - 32, n)
    npg = rng.integers(1, 33, n)
    d_reads = torch.from_numpy(np.stack([first * pb, npg * pb], axis=1).reshape(-1).astype(np.int64)).to(dev)
    bad = torch.zeros(n, dtype=torch.int32, device=dev)
    total = torch.zeros(1, dtype=torch.int64, device=dev)
    out[f"verify_reads_{n}_us"] = timed(lambda: C.verify_read_records(pool, crcs, d_reads, n, bad, total, pb))
    assert int(total.item()) == 0
for n in (1, 16, 256):
    rec = C.log_records(rng.integers(0, pool.numel() - pb, n), rng.integers(0, src.numel() - pb, n),
                        rng.integers(512, 4097, n))
    d_log = torch.from_numpy(rec.view(np.uint8)).to(dev)
    out[f"apply_log_{n}_us"] = timed(lambda: C.apply_log(pool, crcs, src, d_log, n, 4096, pb))
out["page_crc_one_chunk_us"] = timed(lambda: C.page_crc(pool[:16 << 20], pb, out=crcs[:4096]))
assert torch.equal(crcs, C.page_crc(pool, pb))
print(json.dumps(out), flush=True)
