#!/usr/bin/env python3
"""Drive cc_apply_log_dev alone (config-3 shape: 65,536 random 512 B-4 KiB
writes over a 16 GiB pool) for rocprofv3 kernel traces of the write-log path."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from curve_amd import crc as C  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--gib", type=int, default=16)
p.add_argument("--updates", type=int, default=65536)
p.add_argument("--reps", type=int, default=5)
p.add_argument("--lib", default=None, help="libcurvecrc variant to load instead of the in-tree one")
p.add_argument("--align", type=int, default=1, help="round dst/src offsets and lengths down to this")
p.add_argument("--delta", action="store_true", help="cc_apply_log_delta_dev (stored CRCs updated by linearity)")
p.add_argument("--span-gib", type=float, default=0, help="confine write destinations to the first SPAN GiB (locality probe)")
a = p.parse_args()
if a.lib:
    from curve_amd import _lib
    # relative to the repo root (the profilers run these from /tmp)
    _lib.LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), a.lib)
dev = torch.device("cuda", 0)
pool = torch.empty(a.gib << 30, dtype=torch.uint8, device=dev).random_(0, 256)
crcs = C.page_crc(pool, 4096)
U = a.updates
src = torch.empty(U * 4096, dtype=torch.uint8, device=dev).random_(0, 256)
rng = np.random.default_rng(1)
logs = []
for _ in range(a.reps + 1):
    al = a.align
    span = int(a.span_gib * (1 << 30)) if a.span_gib else pool.numel()
    rec = C.log_records(rng.integers(0, span - 4096, U) // al * al,
                        rng.integers(0, U * 4096 - 4096, U) // al * al, rng.integers(512, 4097, U) // al * al)
    logs.append(torch.from_numpy(rec.view(np.uint8)).to(dev))
s = torch.cuda.current_stream()
ms = []
for k, d_log in enumerate(logs):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    C.apply_log(pool, crcs, src, d_log, U, 4096, 4096, delta=a.delta)
    e1.record(s)
    torch.cuda.synchronize()
    if k:
        ms.append(e0.elapsed_time(e1))
ok = bool(torch.equal(crcs, C.page_crc(pool, 4096)))  # page CRCs consistent with the final bytes
print("apply_log%s ms per batch:" % (" delta" if a.delta else ""), [round(x, 4) for x in ms], "median", round(sorted(ms)[len(ms) // 2], 4),
      "crcs_consistent", ok)
