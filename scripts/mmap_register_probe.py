#!/usr/bin/env python3
"""Probe (diagnostic): can page-cache-resident chunk files reach the GPU without
a CPU copy?  mmap(MAP_SHARED) each file, hipHostRegister the mapping, DMA it
with hipMemcpyAsync, unregister -- vs the pread-into-pinned-staging path that
cc_scan_files uses.  Prints one JSON line with GiB/s for both.

usage: python scripts/mmap_register_probe.py [--files 64]
"""
import argparse
import ctypes
import json
import mmap
import os
import shutil
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from curve_amd import crc as C  # noqa: E402
from curve_amd import _lib  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--files", type=int, default=64)
a = p.parse_args()

_lib.lib()  # loads libamdhip64 through libcurvecrc
hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
GiB = float(1 << 30)
FILE = C.CHUNK_SIZE + C.META_PAGE_SIZE

dev = torch.device("cuda", 0)
d = tempfile.mkdtemp(prefix="cc_mmap_", dir=os.environ.get("TMPDIR", "/tmp"))
out = {"files": a.files, "file_bytes": FILE}
try:
    rng = np.random.default_rng(5)
    body = rng.integers(0, 256, FILE, dtype=np.uint8)
    paths = []
    for i in range(a.files):
        body[:8] = np.frombuffer(np.uint64(i).tobytes(), dtype=np.uint8)
        path = os.path.join(d, f"chunk_{i}")
        body.tofile(path)
        paths.append(path)
    dst = torch.empty(FILE, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    sh = ctypes.c_void_p(s.cuda_stream)
    rcs = set()
    t_reg = t_copy = 0.0
    t0 = time.perf_counter()
    for path in paths:
        fd = os.open(path, os.O_RDWR)
        mm = mmap.mmap(fd, FILE, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        buf = (ctypes.c_char * FILE).from_buffer(mm)
        addr = ctypes.addressof(buf)
        r0 = time.perf_counter()
        rc = hip.hipHostRegister(ctypes.c_void_p(addr), FILE, 0)
        r1 = time.perf_counter()
        rcs.add(rc)
        if rc == 0:
            hip.hipMemcpyAsync(ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(addr), FILE, 1, sh)
            hip.hipStreamSynchronize(sh)
            r2 = time.perf_counter()
            hip.hipHostUnregister(ctypes.c_void_p(addr))
            t_copy += r2 - r1
        t_reg += r1 - r0
        del buf
        mm.close()
        os.close(fd)
    el = time.perf_counter() - t0
    out["register_rcs"] = sorted(rcs)
    out["mmap_register_GiBps"] = round(a.files * FILE / GiB / el, 2)
    out["register_ms_per_file"] = round(t_reg / a.files * 1e3, 3)
    out["copy_ms_per_file"] = round(t_copy / a.files * 1e3, 3)
    # the shipped path for comparison: engine preads into pinned staging + scans
    C.scan_files(paths[:4])
    t0 = time.perf_counter()
    st, _, _, _ = C.scan_files(paths, io_threads=4)
    out["scan_files_GiBps"] = round(a.files * FILE / GiB / (time.perf_counter() - t0), 2)
finally:
    shutil.rmtree(d, ignore_errors=True)
print(json.dumps(out))
