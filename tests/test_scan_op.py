"""Row f1 at the reference's call shape: ScanChunkRequest::OnApply hashes one
scan op per raft-applied request -- the 4 KiB metapage or a 4 MiB data slice,
`crc = CRC32(readBuffer, size)` (src/chunkserver/op_request.cpp:776-794, :847) --
from up to wconcurrentapply.size = 10 apply threads at once
(conf/chunkserver.conf:183, op_request.cpp:179-187); a 16 MiB chunk is 5 ops
(test/chunkserver/scan_manager_test.cpp:107-142).

The calls run on native threads (curve_amd/host/scan_op_bench.cpp sob_run, via
bench.run_scan_ops), so callers really are concurrent inside libcurvecrc
(cc_page_crc_host gives each concurrent caller a lane of its own); every op's
ScanMap.crc is checked against the oracle."""
import os
import threading

import numpy as np
import pytest

import bench
from curve_amd import _lib

FILE = 4096 + (16 << 20)
OFFS = [0] + [4096 + k * (4 << 20) for k in range(4)]
LENS = [4096] + [4 << 20] * 4


def _have_gpu():
    return _lib.lib().cc_device_count() > 0


def _files(oracle, n, size=FILE, seed=0x5CA0):
    return [oracle.splitmix64_bytes(seed + t, size) for t in range(n)]


def _want(oracle, bufs, offs, lens):
    return [[oracle.crc32c(b[o:o + n].tobytes()) for o, n in zip(offs, lens)] for b in bufs]


def _check(crcs, want, calls):
    for t, w in enumerate(want):
        assert (crcs[t] == np.resize(np.array(w, dtype=np.uint32), calls)).all(), f"thread {t}"


def test_harness_cpu_mode(oracle):
    """The harness and the CPU primitive, 4 threads, no GPU needed."""
    bufs = _files(oracle, 4, size=1 << 20)
    offs, lens = [0, 4096, 65536 + 3], [4096, 65536, 300000]
    rc, lat, crcs, wall, cpu_s = bench.run_scan_ops(bufs, offs, lens, 9, "cpu")
    assert rc == 0 and wall > 0 and cpu_s >= 0 and (lat >= 0).all()
    _check(crcs, _want(oracle, bufs, offs, lens), 9)


def test_routed_metapage_on_cpu(oracle):
    """cchost::ScanOpCrc keeps the 4 KiB metapage op (below kCpuHashMax) on the
    CPU primitive: it answers without a GPU."""
    bufs = _files(oracle, 3, size=8192)
    rc, _, crcs, _, _ = bench.run_scan_ops(bufs, [0, 4096], [4096, 4096], 4, "routed")
    assert rc == 0
    _check(crcs, _want(oracle, bufs, [0, 4096], [4096, 4096]), 4)


def test_gpu_mode_without_device_fails_loudly(oracle):
    if _have_gpu():
        pytest.skip("a GPU is visible")
    bufs = _files(oracle, 2, size=1 << 20)
    rc, _, _, _, _ = bench.run_scan_ops(bufs, [0], [1 << 20], 2, "gpu")
    assert rc == _lib.CC_ENODEV


def _pinned(arrs):
    import torch
    out = []
    for a in arrs:
        h = torch.empty(a.size, dtype=torch.uint8, pin_memory=True)
        h.numpy()[:] = a
        out.append(h)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["gpu", "routed"])
def test_ten_apply_threads_pinned(oracle, mode):
    """10 threads x 100 ops (20 chunk files' worth each: metapage + 4 slices),
    pinned buffers: every ScanMap.crc == the oracle's."""
    files = _files(oracle, 10)
    hs = _pinned(files)
    bufs = [h.numpy() for h in hs]
    rc, lat, crcs, wall, _ = bench.run_scan_ops(bufs, OFFS, LENS, 100, mode)
    assert rc == 0, rc
    _check(crcs, _want(oracle, files, OFFS, LENS), 100)
    assert wall > 0 and (lat > 0).all()


@pytest.mark.gpu
def test_more_threads_than_lanes_pageable(oracle):
    """24 callers (more than the engine's 16 lanes: some wait for a lane) on
    pageable buffers (the reference's `new char[size]`), ops of every page
    count from 1 to 64 and a whole lane (16 MiB)."""
    n = 24
    files = _files(oracle, n, size=(16 << 20) + 8192, seed=0xA11)
    offs = [0, 4096, 8192, 3 * 4096, 4096]
    lens = [4096, 64 * 4096, 17 * 4096, 4 << 20, 16 << 20]
    rc, _, crcs, _, _ = bench.run_scan_ops(files, offs, lens, 15, "gpu")
    assert rc == 0, rc
    _check(crcs, _want(oracle, files, offs, lens), 15)


@pytest.mark.gpu
def test_lanes_beside_a_large_call(oracle):
    """A large cc_page_crc_host call (the shared two-slot path, held for the
    whole call) runs while 10 threads issue scan ops on lanes: both correct."""
    from curve_amd import crc as C
    big = oracle.splitmix64_bytes(0xB16, 96 << 20)
    want_big = oracle.page_crcs(big.reshape(-1, 4096), 4096)
    got = {}

    def large():
        got["big"] = [C.page_crc_host(big, 4096) for _ in range(3)]

    th = threading.Thread(target=large)
    files = _files(oracle, 10, seed=0xC0C)
    th.start()
    rc, _, crcs, _, _ = bench.run_scan_ops(files, OFFS, LENS, 40, "gpu")
    th.join()
    assert rc == 0, rc
    _check(crcs, _want(oracle, files, OFFS, LENS), 40)
    for r in got["big"]:
        assert (np.asarray(r).view(np.uint32) == want_big).all()


@pytest.mark.gpu
def test_lane_call_errors_leave_lanes_usable(oracle):
    """Bad arguments are refused before a lane is taken; good calls after them work."""
    import ctypes
    L = _lib.lib()
    out = (ctypes.c_uint32 * 4)()
    assert L.cc_page_crc_host(None, 1, 4096, out) == _lib.CC_EINVAL
    assert L.cc_page_crc_host(ctypes.c_void_p(1), 1, 100, out) == _lib.CC_EINVAL
    files = _files(oracle, 2, size=1 << 20)
    rc, _, crcs, _, _ = bench.run_scan_ops(files, [0], [1 << 20], 3, "gpu")
    assert rc == 0
    _check(crcs, _want(oracle, files, [0], [1 << 20]), 3)


@pytest.mark.gpu
@pytest.mark.parametrize("page_bytes", [256, 768, 4096, 8192, 1 << 20])
def test_lane_and_slot_paths_by_page_size(oracle, page_bytes):
    """cc_page_crc_host at every page geometry the ABI accepts, on both sides of
    the lane limit (16 MiB: a lane of its own; above: the two shared staging
    slots), pinned and pageable, the pageable buffer at an odd address (the
    lane's staging copies it a 1 MiB piece at a time, the last piece partial):
    every page CRC equal to the oracle's."""
    import torch
    from curve_amd import crc as C
    rng = np.random.default_rng(page_bytes)
    lane_pages = (16 << 20) // page_bytes
    for n in sorted({1, 3, max(1, lane_pages // 3 + 1), lane_pages, lane_pages + 1}):
        raw = rng.integers(0, 256, n * page_bytes + 3, dtype=np.uint8)
        pages = raw[3:]  # pageable, not 4-byte aligned
        want = oracle.page_crcs(pages, page_bytes, threads=8)
        assert (C.page_crc_host(pages, page_bytes) == want).all(), (page_bytes, n, "pageable")
        pinned = torch.from_numpy(np.ascontiguousarray(pages)).pin_memory()
        assert (C.page_crc_host(pinned.numpy(), page_bytes) == want).all(), (page_bytes, n, "pinned")
