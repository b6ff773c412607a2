#!/usr/bin/env python3
"""cc_scan_files timeline (diagnostic): the trace build of the library
(scripts/make_variant.sh trace py scripts/patches/scan_files_trace.py)
writes per-batch host timestamps (loop start, drain done, the drained batch's
host function, reads done, enqueued) to /tmp/cc_scan_trace.txt; this runs
scan_files over 128 page-cache-resident chunk files with it (argv: labels of
the runs; round 5 took the copy-schedule variants through CC_AB_GROUP)."""
import os
import shutil
import sys
import tempfile
import time

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
from curve_amd import _lib  # noqa: E402
_lib.LIB_PATH = os.path.join(R, "build/variants/libcurvecrc_trace.so")
from curve_amd import crc as C  # noqa: E402

n = 128
d = tempfile.mkdtemp(prefix="cc_tr_", dir=os.environ.get("TMPDIR", "/tmp"))
body = np.random.default_rng(3).integers(0, 256, C.CHUNK_SIZE + C.META_PAGE_SIZE, dtype=np.uint8)
paths = []
for i in range(n):
    body[:8] = np.frombuffer(np.uint64(i).tobytes(), dtype=np.uint8)
    p = os.path.join(d, f"chunk_{i}")
    body.tofile(p)
    paths.append(p)
out = os.path.join(R, "gpurun_out")
os.makedirs(out, exist_ok=True)
for g in sys.argv[1:] or ["0"]:
    os.environ["CC_AB_GROUP"] = g
    C.scan_files(paths[:8], io_threads=8)
    for _ in range(2):
        if os.path.exists("/tmp/cc_scan_trace.txt"):
            os.unlink("/tmp/cc_scan_trace.txt")
        t0 = time.perf_counter()
        C.scan_files(paths, io_threads=8)
        el = time.perf_counter() - t0
    shutil.copy("/tmp/cc_scan_trace.txt", os.path.join(out, f"scan_trace_g{g}.txt"))
    print(g, round(n * (C.CHUNK_SIZE + C.META_PAGE_SIZE) / (1 << 30) / el, 2), "GiB/s", flush=True)
shutil.rmtree(d, ignore_errors=True)
