#!/usr/bin/env python3
"""Interleaved in-process A/B of the whole scan step (cc_pool_scan_dev: page
CRCs + metapage CRCs + fused epilogue + digest partials) across libcurvecrc
builds, in the bench's shape (1024 x 16 MiB chunks, 64 copysets).  Reports per
build the step time and the page-kernel time from the call's own events, and
checks every build's slice CRCs and digests against the first build's.
usage: pool_ab.py LIB.so [LIB.so ...]"""
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
libs = {}
for path in sys.argv[1:]:
    L = ctypes.CDLL(os.path.abspath(path))
    L.cc_pool_scan_dev.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    libs[path] = L


def shard(digest, ev):
    sh = _lib.CcPoolShard()
    sh.d_data, sh.d_meta, sh.n_chunks = data.data_ptr(), meta.data_ptr(), n
    sh.chunk_bytes, sh.meta_bytes, sh.page_bytes, sh.slice_bytes = chunk, meta_sz, 4096, pool.scan_size
    sh.d_after_mult, sh.d_group, sh.n_groups = after_mult.data_ptr(), group.data_ptr(), digest.numel()
    sh.d_page_crcs, sh.d_meta_crcs = pool.page_crcs.data_ptr(), pool.meta_crcs.data_ptr()
    sh.d_slice_crcs, sh.d_file_crcs, sh.d_digest = pool.slice_crcs.data_ptr(), pool.file_crcs.data_ptr(), digest.data_ptr()
    sh.ev_pages_begin, sh.ev_pages_end = ev[0].cuda_event, ev[1].cuda_event
    return sh


digests = {p: torch.full((lay.n_groups,), 7, dtype=torch.int32, device=dev) for p in libs}
ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
ev[0].record(s)
ev[1].record(s)
shards = {p: shard(digests[p], ev) for p in libs}


def call(p):
    rc = libs[p].cc_pool_scan_dev(ctypes.byref(shards[p]), None, ctypes.c_void_p(s.cuda_stream))
    assert rc == 0, rc


results = {}
for p in libs:
    call(p)
    torch.cuda.synchronize()
    results[p] = (pool.slice_crcs.clone(), pool.file_crcs.clone(), digests[p].clone())
# ~3 s of sustained load first: the clock settles only after ~2.5 s of it (bench.py warm_clock)
for _ in range(1200):
    call(sys.argv[1])
torch.cuda.synchronize()
step, kern = {p: [] for p in libs}, {p: [] for p in libs}
order = list(libs)
for r in range(32):
    for p in (order if r % 2 == 0 else order[::-1]):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(4):
            call(p)  # re-records the page-kernel events (the last call's remain)
        e1.record(s)
        torch.cuda.synchronize()
        step[p].append(e0.elapsed_time(e1) / 4)
        kern[p].append(ev[0].elapsed_time(ev[1]))
ref = results[order[0]]
for p in libs:
    same = all(torch.equal(a, b) for a, b in zip(results[p], ref))
    st, kt = sorted(step[p]), sorted(kern[p])
    med = kt[len(kt) // 2]
    print(f"{os.path.basename(p)}: step median {st[len(st) // 2]:.4f} ms, page kernel median {med:.4f} ms "
          f"(spread {(kt[-1] - kt[0]) / med * 100:.2f} %, mean {sum(kt) / len(kt):.4f}), same_results {same}", flush=True)
