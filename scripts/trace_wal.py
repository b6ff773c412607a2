#!/usr/bin/env python3
"""Diagnostic: per-wave start/end wall clock of range_flat_kernel
(CC_WAVE_TRACE=1 build) over repeated WAL-replay batches; where is the tail?"""
import ctypes
import os
import sys

import numpy as np
import torch

lib = ctypes.CDLL(os.path.abspath(sys.argv[1]))
lib.cc_crc_ranges_dev.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint64] + [ctypes.c_void_p] * 2
dev = torch.device("cuda", 0)
pool = torch.empty(16 << 30, dtype=torch.uint8, device=dev).random_(0, 256)
rng = np.random.default_rng(0x3A1)
n = 65536
real = rng.integers(1024, (128 << 10) + 1, n).astype(np.uint64)
page = len(sys.argv) > 2 and sys.argv[2] == "page"
if len(sys.argv) > 2 and not page:
    real[:] = int(sys.argv[2])
lib.cc_page_crc_dev.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
pcrc = torch.empty((16 << 30) // 4096, dtype=torch.int32, device=dev)
slot = (28 + real + 4095) // 4096 * 4096
offs = np.concatenate([[0], np.cumsum(slot)[:-1]]).astype(np.uint64) + 4096 + 28
rec = np.empty((n, 2), dtype=np.uint64)
rec[:, 0], rec[:, 1] = offs, real
d_rec = torch.from_numpy(rec.view(np.uint8).reshape(-1)).to(dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
tr = np.zeros((4, 8192), dtype=np.uint64)
W = 256 * 8
for it in range(40):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    if page:
        assert lib.cc_page_crc_dev(pool.data_ptr(), (16 << 30) // 4096, 4096, pcrc.data_ptr(),
                                   ctypes.c_void_p(s.cuda_stream)) == 0
    else:
        assert lib.cc_crc_ranges_dev(pool.data_ptr(), d_rec.data_ptr(), n, out.data_ptr(),
                                     ctypes.c_void_p(s.cuda_stream)) == 0
    e1.record(s)
    torch.cuda.synchronize()
    if it < 20:
        continue
    ms = e0.elapsed_time(e1)
    assert lib.cc_debug_wave_trace(tr.ctypes.data_as(ctypes.c_void_p)) == 0
    st, en, blk, cu = tr[0, :W].astype(np.int64), tr[1, :W].astype(np.int64), tr[2, :W], tr[3, :W]
    t0 = st.min()
    st_us, en_us = (st - t0) / 100.0, (en - t0) / 100.0  # 100 MHz
    dur = en_us - st_us
    xcd = blk % 8
    slow = np.argsort(en_us)[-20:]
    per_xcd_end = [round(float(np.percentile(en_us[xcd == x], 99)), 1) for x in range(8)]
    print(f"ms {ms:.4f} span {en_us.max():.1f} us start max {st_us.max():.1f} end p50 {np.percentile(en_us, 50):.1f} "
          f"p90 {np.percentile(en_us, 90):.1f} p99 {np.percentile(en_us, 99):.1f} | dur p50 {np.percentile(dur, 50):.1f} "
          f"max {dur.max():.1f} | xcd p99 end {per_xcd_end} | slow xcd {np.bincount(xcd[slow], minlength=8).tolist()} "
          f"slow waves {sorted(slow.tolist())[:8]}", flush=True)
