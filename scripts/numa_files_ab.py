#!/usr/bin/env python3
"""Does binding the process to its GPU's NUMA node help the host-fed paths at
N = 1?  One mode per process (the pinned staging and the page cache of the
files are placed when first touched, so a mode must own its whole process):
`bind` calls bench.bind_to_gpu_numa(0) before anything is allocated, `nobind`
does not.  Then: the chunk files written (page cache), cc_scan_files at the
default readers, `--passes` passes, and cc_page_crc_host over a 1 GiB pinned
buffer for 2 s.  Prints one JSON line.
usage: numa_files_ab.py bind|nobind [--files 128] [--passes 5]
       (run the two modes alternately, each in its own process)"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from curve_amd import crc as C  # noqa: E402

GiB = 1 << 30
p = argparse.ArgumentParser()
p.add_argument("mode", choices=("bind", "nobind"))
p.add_argument("--files", type=int, default=128)
p.add_argument("--passes", type=int, default=5)
a = p.parse_args()
torch.cuda.set_device(0)
out = {"mode": a.mode}
if a.mode == "bind":
    out["binding"] = bench.bind_to_gpu_numa(0)
out["cpus"] = len(os.sched_getaffinity(0))
d = tempfile.mkdtemp(prefix="cc_numa_", dir=os.environ.get("TMPDIR", "/tmp"))
try:
    rng = np.random.default_rng(3)
    body = rng.integers(0, 256, C.CHUNK_SIZE + C.META_PAGE_SIZE, dtype=np.uint8)
    paths = []
    for i in range(a.files):
        body[:8] = np.frombuffer(np.uint64(i).tobytes(), dtype=np.uint8)
        path = os.path.join(d, f"chunk_{i}")
        body.tofile(path)
        paths.append(path)
    C.scan_files(paths[:4])
    fb = a.files * (C.CHUNK_SIZE + C.META_PAGE_SIZE) / GiB
    each = []
    for _ in range(a.passes):
        t0 = time.perf_counter()
        st, _, _, _ = C.scan_files(paths)
        each.append(fb / (time.perf_counter() - t0))
        assert (st == 0).all()
    out["files_GiBps"] = round(float(np.median(each)), 2)
    out["files_each"] = [round(x, 2) for x in each]
finally:
    shutil.rmtree(d, ignore_errors=True)
h = torch.empty(GiB, dtype=torch.uint8, pin_memory=True)
h.random_(0, 256)
arr = h.numpy()
C.page_crc_host(arr, 4096)
t0, reps = time.perf_counter(), 0
while time.perf_counter() - t0 < 2.0:
    C.page_crc_host(arr, 4096)
    reps += 1
out["pinned_e2e_GiBps"] = round(reps / (time.perf_counter() - t0), 2)
print(json.dumps(out), flush=True)
