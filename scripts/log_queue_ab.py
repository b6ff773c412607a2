#!/usr/bin/env python3
"""Write-log queue A/B in the bench's partial-write shape (65,536 random
512 B-4 KiB writes per batch over a 16 GiB pool, 10 batches): the batches as
10 cc_apply_log_dev calls vs ONE cc_apply_logs_dev call (each page kernel also
groups the next batch), interleaved rounds, HIP events around the 10 batches,
per-batch ms.  Afterwards every page must verify.
usage: log_queue_ab.py [--rounds 20] [--delta]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from curve_amd import crc as C  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--rounds", type=int, default=20)
p.add_argument("--delta", action="store_true")
p.add_argument("--only", choices=("singles", "queue"), default=None, help="time one form only (kernel traces)")
a = p.parse_args()
dev = torch.device("cuda", 0)
pb, U, B = 4096, 65536, 10
pool = torch.empty(16 << 30, dtype=torch.uint8, device=dev).random_(0, 256)
crcs = C.page_crc(pool, pb)
src = torch.empty(U * pb, dtype=torch.uint8, device=dev).random_(0, 256)
rng = np.random.default_rng(0xC3)
batches = []
for _ in range(B):
    dst, so, ln = rng.integers(0, pool.numel() - pb, U), rng.integers(0, U * pb - pb, U), rng.integers(512, 4097, U)
    batches.append((src, torch.from_numpy(C.log_records(dst, so, ln).view(np.uint8)).to(dev), U))
s = torch.cuda.current_stream()


def singles():
    for sr, d_log, n in batches:
        C.apply_log(pool, crcs, sr, d_log, n, pb, pb, delta=a.delta)


def queue():
    C.apply_logs(pool, crcs, batches, pb, pb, delta=a.delta)


for f in (singles, queue, singles, queue):
    f()
torch.cuda.synchronize()
ms = {"singles": [], "queue": []} if a.only is None else {a.only: []}
for r in range(a.rounds):
    pairs = (("singles", singles), ("queue", queue)) if r % 2 == 0 else (("queue", queue), ("singles", singles))
    for name, f in (x for x in pairs if x[0] in ms):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        f()
        e1.record(s)
        torch.cuda.synchronize()
        ms[name].append(e0.elapsed_time(e1) / B)
bad = int(C.page_verify(pool, crcs, pb)[0])
for name, v in ms.items():
    print(f"{name}{' delta' if a.delta else ''}: per batch median {np.median(v):.4f} ms min {min(v):.4f} "
          f"mean {np.mean(v):.4f}", flush=True)
print(f"pages failing verify after: {bad}")
assert bad == 0
