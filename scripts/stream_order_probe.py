#!/usr/bin/env python3
"""Does the ORDER in which 2,048 waves stream a contiguous buffer set the read
rate?  cc_page_list_probe_dev (verify-on-read's grid: 8 waves a CU, each wave an
equal contiguous share of its page list, two pages in flight) over the same
1,058,816 pages (4.1 GiB, the WAL leg's size) listed three ways:
  contiguous   -- wave w's share is one contiguous ~2 MiB run (the WAL kernel's
                  static pieces);
  tiles64      -- the buffer cut into 64-page (256 KiB) tiles dealt round robin,
                  wave w taking tiles w, w + W, ... (the page kernel's walk);
  tiles16      -- the same with 16-page (64 KiB) tiles.
usage: stream_order_probe.py [--rounds 20]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from curve_amd import crc as C  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--rounds", type=int, default=20)
a = p.parse_args()
dev = torch.device("cuda", 0)
pool = torch.empty(16 << 30, dtype=torch.uint8, device=dev).random_(0, 256)
W = torch.cuda.get_device_properties(dev).multi_processor_count * 8
n = 1058816 // (W * 64) * W * 64  # a whole number of 64-page tiles per wave (~the WAL leg's size)
base = np.arange(n, dtype=np.int64) + 4096


def tiled(t):
    per = n // W                       # pages per wave
    tiles = per // t                    # tiles per wave
    idx = np.empty(n, dtype=np.int64)
    for w in range(W):                  # wave w's share: tiles w, w + W, ... laid out consecutively
        tl = w + W * np.arange(tiles)
        idx[w * per:(w + 1) * per] = (tl[:, None] * t + np.arange(t)[None, :]).reshape(-1)
    return base[idx]


lists = {"contiguous": base, "tiles64": tiled(64), "tiles16": tiled(16)}
assert all(np.array_equal(np.sort(v), base) for v in lists.values())
dl = {k: torch.from_numpy(v).to(dev) for k, v in lists.items()}
out = torch.empty(n, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
for _ in range(30):
    for k in dl:
        C.page_list_probe(pool, dl[k], n, out)
torch.cuda.synchronize()
ms = {k: [] for k in dl}
for r in range(a.rounds):
    for k in (list(dl) if r % 2 == 0 else list(dl)[::-1]):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        C.page_list_probe(pool, dl[k], n, out)
        e1.record(s)
        torch.cuda.synchronize()
        ms[k].append(e0.elapsed_time(e1))
for k, v in ms.items():
    med = float(np.median(v))
    print(f"{k}: median {med:.4f} ms, {n * 4096 / (med * 1e-3) / 1e9:.1f} GB/s", flush=True)
