#!/usr/bin/env python3
"""Range (WAL replay shape) and verify-on-read calls while a page kernel runs on
ANOTHER stream: the page kernel holds every CU (one 160 KiB-LDS
workgroup each), so the range / verify kernel's workgroups start only as its
workgroups retire, and the ones that start early wait for tile counts of
workgroups that are not running yet.  Per build: each call alone, then each
enqueued right behind a page kernel over 8 GiB on a second stream; HIP events
on the call's stream, outputs compared with the call alone.
usage: concurrent_ranges.py LIB.so [LIB.so ...]"""
import ctypes
import os
import sys

import numpy as np
import torch

dev = torch.device("cuda", 0)
big = torch.empty(8 << 30, dtype=torch.uint8, device=dev).random_(0, 256)
big_crc = torch.empty(big.numel() // 4096, dtype=torch.int32, device=dev)
buf = big[: 1 << 30]
rng = np.random.default_rng(5)
n = 65536
off = rng.integers(0, buf.numel() - 65536, n).astype(np.uint64)
ln = rng.integers(1, 65536, n).astype(np.uint64)
rec = torch.from_numpy(np.stack([off, ln], axis=1).reshape(-1).view(np.uint8)).to(dev)
reads = torch.from_numpy(np.stack([off // 4096 * 4096, (ln + 4095) // 4096 * 4096], axis=1).reshape(-1)
                         .view(np.uint8)).to(dev)
page_crcs = torch.empty(buf.numel() // 4096, dtype=torch.int32, device=dev)
sA, sB = torch.cuda.Stream(), torch.cuda.Stream()
V = ctypes.c_void_p
# a stream limited to 32 CUs (hipExtStreamCreateWithCUMask): a 256-workgroup
# grid then runs 32 workgroups at a time, the rest not resident while the
# first wait for their tiles
hip = ctypes.CDLL("libamdhip64.so")
hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(V), ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
mask = (ctypes.c_uint32 * 8)(0xFFFFFFFF, 0, 0, 0, 0, 0, 0, 0)
sM_h = V()
assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(sM_h), 8, mask) == 0
sM = torch.cuda.ExternalStream(sM_h.value)
for p in sys.argv[1:]:
    L = ctypes.CDLL(os.path.abspath(p))
    L.cc_crc_ranges_dev.argtypes = [V, V, ctypes.c_uint64, V, V]
    L.cc_page_crc_dev.argtypes = [V, ctypes.c_uint64, ctypes.c_uint32, V, V]
    L.cc_verify_reads_dev.argtypes = [V, ctypes.c_uint64, ctypes.c_uint32, V, ctypes.c_uint64, V, V, V, V,
                                      ctypes.c_uint64, V]
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    bad = torch.zeros(n, dtype=torch.int32, device=dev)
    tot = torch.zeros(1, dtype=torch.int64, device=dev)
    work = torch.empty(256, dtype=torch.uint8, device=dev)
    assert L.cc_page_crc_dev(buf.data_ptr(), page_crcs.numel(), 4096, page_crcs.data_ptr(), V(sB.cuda_stream)) == 0

    def rng_call(st=sB):
        assert L.cc_crc_ranges_dev(buf.data_ptr(), rec.data_ptr(), n, out.data_ptr(), V(st.cuda_stream)) == 0

    def rv_call(st=sB):
        assert L.cc_verify_reads_dev(buf.data_ptr(), buf.numel(), 4096, reads.data_ptr(), n, page_crcs.data_ptr(),
                                     bad.data_ptr(), tot.data_ptr(), work.data_ptr(), 256, V(st.cuda_stream)) == 0

    def page_call():
        assert L.cc_page_crc_dev(big.data_ptr(), big_crc.numel(), 4096, big_crc.data_ptr(), V(sA.cuda_stream)) == 0

    res = {}
    for name, call in (("ranges", rng_call), ("verify_reads", rv_call)):
        for _ in range(20):
            call()
        torch.cuda.synchronize()
        alone, beside = [], []
        for _ in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(sB)
            call()
            e1.record(sB)
            torch.cuda.synchronize()
            alone.append(e0.elapsed_time(e1))
        want = out.clone()
        for _ in range(10):
            page_call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(sB)
            call()
            e1.record(sB)
            torch.cuda.synchronize()
            beside.append(e0.elapsed_time(e1))
        masked = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(sM)
            call(sM)
            e1.record(sM)
            torch.cuda.synchronize()
            masked.append(e0.elapsed_time(e1))
        same = bool(torch.equal(out, want)) if name == "ranges" else int(tot.item()) == 0
        res[name] = (float(np.median(alone)), float(np.median(beside)), max(beside), same, float(np.median(masked)))
    torch.cuda.synchronize()
    for name, (a, b, mx, same, mk) in res.items():
        print(f"{os.path.basename(p)} {name}: alone median {a:.3f} ms; behind a page kernel on another stream "
              f"median {b:.3f} ms max {mx:.3f} ms (page kernel over 8 GiB ~1.2 ms included); on a 32-CU stream "
              f"median {mk:.3f} ms; outputs ok {same}", flush=True)
