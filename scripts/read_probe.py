"""Where does cc_scan_files' time go?  Times, on the same page-cache-resident
chunk files: threaded pread into a pageable buffer, into a pinned buffer, and
the engine's cc_scan_files at several io-thread counts.  Prints JSON lines.
Diagnostic only (not part of the product path)."""
import json
import os
import shutil
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from curve_amd import crc as C  # noqa: E402

GiB = 1 << 30
FILE = C.CHUNK_SIZE + C.META_PAGE_SIZE
PIECE = 2 << 20


def pread_all(paths, buf, threads):
    """buf: [batch, FILE] uint8; files read round-robin into batch slots."""
    batch = buf.shape[0]
    mv = [memoryview(buf[k]) for k in range(batch)]

    def job(args):
        i, off = args
        fd = os.open(paths[i], os.O_RDONLY)
        try:
            n = min(PIECE, FILE - off)
            got = os.preadv(fd, [mv[i % batch][off:off + n]], off)
            assert got == n
        finally:
            os.close(fd)

    items = [(i, off) for i in range(len(paths)) for off in range(0, FILE, PIECE)]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(job, items))
    return time.perf_counter() - t0


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    d = tempfile.mkdtemp(prefix="cc_probe_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        body = np.random.default_rng(1).integers(0, 256, FILE, dtype=np.uint8)
        paths = []
        for i in range(n):
            p = os.path.join(d, f"chunk_{i}")
            body.tofile(p)
            paths.append(p)
        total = n * FILE / GiB
        pageable = np.empty((8, FILE), dtype=np.uint8)
        pageable[:] = 1
        pinned = torch.empty((8, FILE), dtype=torch.uint8, pin_memory=True).numpy()
        pinned[:] = 1
        for t in (4, 8, 16, 32):
            el = pread_all(paths, pageable, t)
            print(json.dumps({"what": "pread->pageable", "threads": t, "GiBps": round(total / el, 2)}), flush=True)
            el = pread_all(paths, pinned, t)
            print(json.dumps({"what": "pread->pinned", "threads": t, "GiBps": round(total / el, 2)}), flush=True)
        C.scan_files(paths[:4])
        for t in (4, 8, 16, 32):
            t0 = time.perf_counter()
            st, _, _, _ = C.scan_files(paths, io_threads=t)
            el = time.perf_counter() - t0
            assert (st == 0).all()
            print(json.dumps({"what": "cc_scan_files", "threads": t, "GiBps": round(total / el, 2)}), flush=True)
        src = torch.from_numpy(pinned)
        dst = torch.empty_like(src, device="cuda")
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(8):
                dst.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
        print(json.dumps({"what": "H2D pinned", "GiBps": round(8 * 8 * FILE / GiB / el, 2)}), flush=True)
        print(json.dumps({"what": "env", "cpu_count": os.cpu_count(),
                          "affinity": len(os.sched_getaffinity(0)),
                          "tmp_fs": open("/proc/mounts").read().count(" /tmp ")}), flush=True)
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
