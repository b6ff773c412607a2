#!/usr/bin/env python3
"""Per-wave times of the write-log page kernel (the log_trace variant:
scripts/make_variant.sh ltrace py scripts/patches/log_trace.py) in the bench's
partial-write shape: 65,536 random 512 B-4 KiB writes over a 16 GiB pool.
Prints, over the grid's waves, when they end (us after the first wave's LDS
fill), by XCD and by age group, the pages each rehashed and the tails taken.
usage: log_trace.py LIB.so [--delta] [--out FILE.json]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from curve_amd import crc as C  # noqa: E402

args = [x for x in sys.argv[1:] if not x.startswith("--")]
delta = "--delta" in sys.argv
out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
fn = "cc_apply_log_delta_dev" if delta else "cc_apply_log_dev"
dev = torch.device("cuda", 0)
pb, U = 4096, 65536
pool = torch.empty(16 << 30, dtype=torch.uint8, device=dev).random_(0, 256)
crcs = C.page_crc(pool, pb)
src = torch.empty(U * pb, dtype=torch.uint8, device=dev).random_(0, 256)
rng = np.random.default_rng(7)
logs = []
for _ in range(8):
    rec = C.log_records(rng.integers(0, pool.numel() - pb, U), rng.integers(0, U * pb - pb, U),
                        rng.integers(512, 4097, U))
    logs.append(torch.from_numpy(rec.view(np.uint8)).to(dev))
L = ctypes.CDLL(os.path.abspath(args[0]))
L.cc_apply_log_work_bytes.restype = ctypes.c_uint64
L.cc_apply_log_work_bytes.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]
getattr(L, fn).argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                           ctypes.c_void_p]
L.cc_log_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
work = torch.empty(L.cc_apply_log_work_bytes(U, pb, pb), dtype=torch.uint8, device=dev)
s = torch.cuda.current_stream()
NW = 8 * 8192
host = np.zeros(NW, dtype=np.uint64)
res = []
for k in range(70):
    rc = getattr(L, fn)(pool.data_ptr(), pool.numel(), pb, src.data_ptr(), logs[k % 8].data_ptr(), U, pb,
                        crcs.data_ptr(), work.data_ptr(), work.numel(), ctypes.c_void_p(s.cuda_stream))
    assert rc == 0
    if k >= 60:  # clocks up: one launch at a time, each traced
        torch.cuda.synchronize()
        assert L.cc_log_trace_read(host.ctypes.data, host.nbytes) == 0
        t = host.reshape(-1, 8)
        t = t[t[:, 0] > 0]
        t0 = t[:, 0].min()
        us = lambda c: (t[:, c].astype(np.int64) - int(t0)) / 100.0  # noqa: E731
        row = {}
        for name, c in (("filled", 0), ("end", 4)):
            v = us(c)
            row[name] = [round(float(np.percentile(v, q)), 2) for q in (0, 50, 90, 100)]
        res.append(row)
        last = t.copy()
        host[:] = 0
        # leave the trace zero for the next launch
        torch.cuda.synchronize()
for r in res[-3:]:
    print(("delta " if delta else "full ") + " ".join(f"{k}[min/med/p90/max us]={v}" for k, v in r.items()), flush=True)
med = {k: [float(np.median([r[k][i] for r in res])) for i in range(4)] for k in res[0]}
# the last launch by XCD, by age group in the workgroup (wave / 4) and within workgroups
WV = 16
t0 = int(last[:, 0].min())
end = (last[:, 4].astype(np.int64) - t0) / 100.0
xcc = last[:, 5].astype(int)
wave = np.arange(last.shape[0]) % WV
by_xcd = {int(x): round(float(np.median(end[xcc == x])), 2) for x in np.unique(xcc)}
by_age = {int(g): round(float(np.median(end[wave // 4 == g])), 2) for g in range(WV // 4)}
wg = end.reshape(-1, WV)
spread_in_wg = float(np.median(wg.max(1) - wg.min(1)))
wg_end = wg.max(1)
pages = last[:, 6].astype(np.int64)
rate = {int(x): round(float(np.median(((end - (last[:, 3].astype(np.int64) - t0) / 100.0) / np.maximum(pages, 1))[xcc == x])), 3)
        for x in np.unique(xcc)}
print("end median by XCD:", by_xcd, "by age group:", by_age, flush=True)
steals = last[:, 7].astype(np.int64)
print("us per page by XCD (page phase / pages):", rate, "pages per wave min/median/max", int(pages.min()),
      int(np.median(pages)), int(pages.max()), "tails taken:", int(steals.sum()), "by", int((steals > 0).sum()),
      "waves", flush=True)
print(f"workgroup end (last wave): min {wg_end.min():.1f} median {np.median(wg_end):.1f} max {wg_end.max():.1f}; "
      f"median spread inside a workgroup {spread_in_wg:.1f} us", flush=True)
print("median over", len(res), "launches:", json.dumps(med), flush=True)
if out:
    json.dump({"mode": "delta" if delta else "full", "launches": res, "median": med, "end_by_xcd": by_xcd,
               "end_by_age_group": by_age, "wg_end": [round(float(x), 2) for x in wg_end],
               "median_spread_in_wg": spread_in_wg}, open(out, "w"), indent=1)
