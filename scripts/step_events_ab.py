#!/usr/bin/env python3
"""The scan step (cc_pool_scan_dev, the bench's shape) with and without the
page-kernel event pair the bench records inside each step, interleaved: what
the two event packets cost the step.  usage: step_events_ab.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from curve_amd import _lib, crc as C  # noqa: E402
from curve_amd.pool import copyset_layout  # noqa: E402
from curve_amd.scan import DevicePool  # noqa: E402

dev = torch.device("cuda", 0)
n, chunk, meta_sz = 1024, C.CHUNK_SIZE, C.META_PAGE_SIZE
data = torch.empty((n, chunk), dtype=torch.uint8, device=dev).random_(0, 256)
meta = torch.zeros((n, meta_sz), dtype=torch.uint8, device=dev)
meta[:, 0] = 2
meta[:, 1:9].random_(0, 256)
pool = DevicePool(data, meta, list(range(n)), page_bytes=4096)
lay = copyset_layout(list(range(n)), [i % 64 for i in range(n)], [chunk + meta_sz] * n)
after_mult = C.xpow8(torch.tensor(lay.after_bytes, dtype=torch.int64, device=dev))
group = torch.tensor(lay.group, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
L = _lib.lib()


def shard(digest, ev):
    sh = _lib.CcPoolShard()
    sh.d_data, sh.d_meta, sh.n_chunks = data.data_ptr(), meta.data_ptr(), n
    sh.chunk_bytes, sh.meta_bytes, sh.page_bytes, sh.slice_bytes = chunk, meta_sz, 4096, pool.scan_size
    sh.d_after_mult, sh.d_group, sh.n_groups = after_mult.data_ptr(), group.data_ptr(), digest.numel()
    sh.d_page_crcs, sh.d_meta_crcs = pool.page_crcs.data_ptr(), pool.meta_crcs.data_ptr()
    sh.d_slice_crcs, sh.d_file_crcs, sh.d_digest = pool.slice_crcs.data_ptr(), pool.file_crcs.data_ptr(), digest.data_ptr()
    if ev is not None:
        sh.ev_pages_begin, sh.ev_pages_end = ev[0].cuda_event, ev[1].cuda_event
    return sh


digest = torch.zeros((lay.n_groups,), dtype=torch.int32, device=dev)
ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
ev[0].record(s)
ev[1].record(s)
modes = {"inner events": shard(digest, ev), "no inner events": shard(digest, None)}


def call(m):
    rc = L.cc_pool_scan_dev(ctypes.byref(modes[m]), None, ctypes.c_void_p(s.cuda_stream))
    assert rc == 0, rc


for _ in range(1200):
    call("inner events")
torch.cuda.synchronize()
step = {m: [] for m in modes}
kern = []
order = list(modes)
for r in range(40):
    for m in (order if r % 2 == 0 else order[::-1]):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(4):
            call(m)
        e1.record(s)
        torch.cuda.synchronize()
        step[m].append(e0.elapsed_time(e1) / 4)
        if m == "inner events":
            kern.append(ev[0].elapsed_time(ev[1]))
kern.sort()
print(f"page kernel by the inner events: median {kern[len(kern) // 2]:.4f} ms", flush=True)
for m, v in step.items():
    v = sorted(v)
    print(f"{m}: step median {v[len(v) // 2]:.4f} ms min {v[0]:.4f}", flush=True)
