#!/usr/bin/env python3
"""Per-wave phase clocks of the write-log page kernel (CC_LOG_TRACE=1 build):
where do a wave's ~135 us go -- LDS fill, the first metadata batch, the page
steps -- and how uneven are the waves?  Bench shape: 65,536 random 512 B-4 KiB
writes over a 16 GiB pool.  usage: trace_log.py LIB.so [--delta]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from curve_amd import crc as C  # noqa: E402

lib_path = sys.argv[1]
delta = "--delta" in sys.argv
fn = "cc_apply_log_delta_dev" if delta else "cc_apply_log_dev"
dev = torch.device("cuda", 0)
pb, U = 4096, 65536
pool = torch.empty(16 << 30, dtype=torch.uint8, device=dev).random_(0, 256)
crcs = C.page_crc(pool, pb)
src = torch.empty(U * pb, dtype=torch.uint8, device=dev).random_(0, 256)
rng = np.random.default_rng(7)
logs = []
for _ in range(4):
    rec = C.log_records(rng.integers(0, pool.numel() - pb, U), rng.integers(0, U * pb - pb, U),
                        rng.integers(512, 4097, U))
    logs.append(torch.from_numpy(rec.view(np.uint8)).to(dev))
L = ctypes.CDLL(os.path.abspath(lib_path))
L.cc_apply_log_work_bytes.restype = ctypes.c_uint64
L.cc_apply_log_work_bytes.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]
getattr(L, fn).argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                           ctypes.c_void_p]
work = torch.empty(L.cc_apply_log_work_bytes(U, pb, pb), dtype=torch.uint8, device=dev)
s = torch.cuda.current_stream()


def call(k):
    rc = getattr(L, fn)(pool.data_ptr(), pool.numel(), pb, src.data_ptr(), logs[k % len(logs)].data_ptr(), U, pb,
                        crcs.data_ptr(), work.data_ptr(), work.numel(), ctypes.c_void_p(s.cuda_stream))
    assert rc == 0, rc


for k in range(200):  # ~30 ms of back-to-back calls: clocks up
    call(k)
torch.cuda.synchronize()
out = []
for rep in range(3):
    call(rep)
    torch.cuda.synchronize()
    tr = np.zeros((6, 4096), dtype=np.uint64)
    assert L.cc_debug_log_trace(tr.ctypes.data_as(ctypes.c_void_p)) == 0
    live = tr[3] > 0
    t0 = tr[0][live].min()
    us = lambda x: (x.astype(np.float64) - float(t0)) / 100.0  # 100 MHz  # noqa: E731
    st, fl, md, en = us(tr[0][live]), us(tr[1][live]), us(tr[2][live]), us(tr[3][live])
    pg, multi, mid = tr[4][live] & 0xFFFF, (tr[4][live] >> 16) & 0xFFFF, us(tr[5][live])
    w = np.nonzero(live)[0]
    xcd = (w // 16) % 8
    steps = en - md
    r = {"waves": int(live.sum()),
         "start_us_p50_max": [round(float(np.median(st)), 2), round(float(st.max()), 2)],
         "lds_fill_us_p50_max": [round(float(np.median(fl - st)), 2), round(float((fl - st).max()), 2)],
         "first_meta_us_p50_max": [round(float(np.median(md - fl)), 2), round(float((md - fl).max()), 2)],
         "steps_us_p50_p99_max": [round(float(np.percentile(steps, q)), 2) for q in (50, 99, 100)],
         "end_us_p1_p50_max": [round(float(np.percentile(en, q)), 2) for q in (1, 50, 100)],
         "pages_per_wave_min_max": [int(pg.min()), int(pg.max())],
         "us_per_page_p50": round(float(np.median(steps / np.maximum(pg, 1))), 3),
         "end_us_median_by_xcd": [round(float(np.median(en[xcd == x])), 2) for x in range(8)],
         "waves_with_multi_frac": round(float((multi > 0).mean()), 3),
         "end_us_median_multi0_vs_multi1plus": [round(float(np.median(en[multi == 0])), 2),
                                                round(float(np.median(en[multi > 0])), 2)],
         "corr_end_vs_multi": round(float(np.corrcoef(en, multi)[0, 1]), 3),
         # is a slow wave slow throughout (systematic) or in bursts? corr of the
         # first-half (12 pages) and second-half durations across waves
         "corr_first_vs_second_half": round(float(np.corrcoef(mid - md, en - mid)[0, 1]), 3),
         "first_half_us_p50_p99": [round(float(np.percentile(mid - md, q)), 2) for q in (50, 99)],
         "slowest_1pct_by_xcd": np.bincount(xcd[en >= np.percentile(en, 99)], minlength=8).tolist()}
    # a workgroup (one per CU) ends with its last wave: the kernel ends with the last workgroup
    blk = w // 16
    bend = np.array([en[blk == b].max() for b in np.unique(blk)])
    bwork = np.array([pg[blk == b].sum() for b in np.unique(blk)])
    r["block_end_us_p1_p50_p90_max"] = [round(float(np.percentile(bend, q)), 2) for q in (1, 50, 90, 100)]
    r["block_end_us_mean"] = round(float(bend.mean()), 2)
    slot = w % 16  # wave index inside its workgroup (launch order)
    r["end_us_median_by_wave_slot"] = [round(float(np.median(en[slot == q])), 1) for q in range(16)]
    r["start_us_median_by_wave_slot"] = [round(float(np.median(md[slot == q])), 2) for q in range(16)]
    r["block_pages_min_max"] = [int(bwork.min()), int(bwork.max())]
    r["block_end_us_median_by_xcd"] = [round(float(np.median(bend[np.unique(blk) % 8 == x])), 2) for x in range(8)]
    out.append(r)
    print(json.dumps(r), flush=True)
json.dump(out, open(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "log_trace.json"), "w"), indent=1)
