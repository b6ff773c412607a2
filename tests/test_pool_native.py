"""Native sharded pool scan (cc_pool_scan_dev) and the RCCL digest exchange
(cc_comm_* / cc_digest_allreduce_dev), include/curve_crc.h.

GPU cases compare the one-call scan with the oracle (ScanMap slices, file
CRCs, CopysetNode::GetHash chains) and run the RCCL path at world size 1 (RCCL
refuses two ranks on one device, so N>1 RCCL runs only in the driver's 8-GPU
bench, which cross-checks the native digests against torch.distributed's).  The
XOR-partial algebra at N>1 is covered on CPU by tests/test_distributed.py.
"""
import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")


def test_pool_scan_rejects_bad_arguments():
    """Argument checks come before any device work (runs without a GPU)."""
    from curve_amd import _lib
    L = _lib.lib()
    assert L.cc_pool_scan_dev(None, None, None) == _lib.CC_EINVAL
    s = _lib.CcPoolShard()
    s.n_chunks, s.chunk_bytes, s.meta_bytes, s.page_bytes, s.slice_bytes = 1, 1 << 20, 4096, 4096, 3 << 18
    assert L.cc_pool_scan_dev(ctypes.byref(s), None, None) == _lib.CC_EINVAL  # slice does not divide chunk
    s.slice_bytes = 1 << 18
    assert L.cc_pool_scan_dev(ctypes.byref(s), None, None) == _lib.CC_EINVAL  # null buffers
    assert L.cc_digest_allreduce_dev(None, None, 0, None) == _lib.CC_EINVAL
    assert L.cc_comm_init(None, 1, 0, None, 0) == _lib.CC_EINVAL
    h = ctypes.c_void_p()
    assert L.cc_comm_init(ctypes.byref(h), 2, 2, ctypes.create_string_buffer(128), 128) == _lib.CC_EINVAL
    assert L.cc_comm_destroy(None) == _lib.CC_OK
    assert L.cc_comm_size(None) == 0 and L.cc_comm_rank(None) == -1
    assert L.cc_comm_wait(None, None, 0) == _lib.CC_EINVAL
    assert L.cc_strerror(_lib.CC_ECOMM) == b"RCCL communication error"


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from curve_amd import crc as C
    C.engine_init()
    return torch.device("cuda", 0)


def u32(t):
    return t.detach().cpu().numpy().view(np.uint32)


def _small_pool(dev, n=10, chunk=1 << 20, seed=5):
    from curve_amd.scan import DevicePool
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, (n, chunk), dtype=np.uint8)
    meta = rng.integers(0, 256, (n, 4096), dtype=np.uint8)
    meta[:, 0] = 2
    ids = [3, 1, 12, 7, 40, 41, 2, 100, 13, 5][:n]
    pool = DevicePool(torch.from_numpy(data).to(dev), torch.from_numpy(meta).to(dev), ids, scan_size=256 << 10)
    return pool, data, meta, ids


def _layout(ids, groups, file_bytes, dev):
    from curve_amd import crc as C
    from curve_amd.pool import copyset_layout
    lay = copyset_layout(ids, groups, [file_bytes] * len(ids))
    after = torch.tensor(lay.after_bytes, dtype=torch.int64, device=dev)
    return lay, C.xpow8(after), torch.tensor(lay.group, dtype=torch.int32, device=dev)


@pytest.mark.gpu
@pytest.mark.parametrize("use_comm", [False, True])
def test_pool_scan_one_call_matches_oracle(dev, oracle, use_comm):
    from curve_amd.pool import Comm, pool_scan
    from curve_amd.scan import chunk_file_name
    pool, data, meta, ids = _small_pool(dev)
    n = len(ids)
    groups = [i % 3 for i in range(n)]
    lay, mult, grp = _layout(ids, groups, (1 << 20) + 4096, dev)
    digest = torch.full((lay.n_groups,), -1, dtype=torch.int32, device=dev)  # the call must zero it
    comm = Comm(1, 0, Comm.unique_id()) if use_comm else None
    try:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(), e1.record()  # create the events; the call re-records them
        pool_scan(pool, mult, grp, digest, comm=comm, events=(e0, e1))
        torch.cuda.synchronize()
        assert e0.elapsed_time(e1) > 0
    finally:
        if comm is not None:
            comm.close()
    assert (u32(pool.page_crcs) == oracle.page_crcs(data, 4096)).all()
    dig = u32(digest)
    for g in range(lay.n_groups):
        files = {chunk_file_name(ids[i]): meta[i].tobytes() + data[i].tobytes() for i in range(n) if groups[i] == g}
        assert str(int(dig[g])) == oracle.copyset_hash(files)
    sl = u32(pool.slice_crcs).reshape(n, 4)
    fc = u32(pool.file_crcs)
    mc = u32(pool.meta_crcs[:n])
    for c in range(n):
        ref = oracle.scan_slices(meta[c].tobytes(), data[c].tobytes(), 256 << 10)
        assert ref[0][2] == mc[c]
        assert [r[2] for r in ref[1:]] == list(sl[c])
        assert fc[c] == oracle.crc32c(meta[c].tobytes() + data[c].tobytes())


@pytest.mark.gpu
def test_digest_allreduce_world1_is_identity_and_repeatable(dev):
    from curve_amd.pool import Comm
    comm = Comm(1, 0, Comm.unique_id())
    try:
        assert (comm.nranks, comm.rank) == (1, 0)
        for n in (1, 64, 5000, 64):  # scratch grows once, then is reused
            x = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=dev)
            want = x.clone()
            comm.allreduce_digest(x)
            torch.cuda.synchronize()
            assert torch.equal(x, want)
    finally:
        comm.close()


@pytest.mark.gpu
def test_pool_scan_empty_shard_still_exchanges(dev):
    """A rank that owns no chunks still joins the digest exchange (zeros)."""
    from curve_amd import _lib
    from curve_amd.pool import Comm
    comm = Comm(1, 0, Comm.unique_id())
    try:
        digest = torch.full((8,), 7, dtype=torch.int32, device=dev)
        s = _lib.CcPoolShard()
        s.chunk_bytes, s.meta_bytes, s.page_bytes, s.slice_bytes = 1 << 24, 4096, 4096, 1 << 22
        s.n_groups, s.d_digest = 8, digest.data_ptr()
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        _lib.check(_lib.lib().cc_pool_scan_dev(ctypes.byref(s), comm.handle, stream))
        torch.cuda.synchronize()
        assert int(digest.abs().sum()) == 0
        s.d_digest = None  # a comm with nothing to exchange is an error
        assert _lib.lib().cc_pool_scan_dev(ctypes.byref(s), comm.handle, stream) == _lib.CC_EINVAL
    finally:
        comm.close()


@pytest.mark.gpu
def test_comm_wait_bounds_an_exchange_stuck_after_init(dev, monkeypatch):
    """cc_comm_wait: the bounded wait for a step's digest exchange.  A
    collective whose peer stopped participating after init never completes; the
    failpoint CC_INJECT_EXCHANGE_STALL_MS makes the exchange's stream sit that
    long first, as such a collective would.  The wait returns CC_ETIMEDOUT at
    its deadline (not the stall's end), the communicator is aborted -- later
    exchanges answer CC_ECOMM, nothing is enqueued -- and the stream still
    drains.  Without the stall the same wait returns CC_OK.  The failpoint is
    read once, when a communicator is created: one made before the variable
    was set never stalls (the exchange path does not consult the environment)."""
    import time
    from curve_amd import _lib
    from curve_amd.pool import Comm
    comm = Comm(1, 0, Comm.unique_id())
    x = torch.arange(64, dtype=torch.int32, device=dev)
    comm.allreduce_digest(x)
    comm.wait(timeout_ms=5000)
    assert torch.equal(x, torch.arange(64, dtype=torch.int32, device=dev))
    monkeypatch.setenv("CC_INJECT_EXCHANGE_STALL_MS", "4000")
    comm.allreduce_digest(x)  # created before the failpoint was armed: no stall
    comm.wait(timeout_ms=2000)
    comm.close()
    comm = Comm(1, 0, Comm.unique_id())  # armed at its init
    try:
        comm.allreduce_digest(x)
        t0 = time.perf_counter()
        with pytest.raises(_lib.CurveCrcError) as ei:
            comm.wait(timeout_ms=500)
        el = time.perf_counter() - t0
        assert ei.value.code == _lib.CC_ETIMEDOUT and 0.45 < el < 3.0, (ei.value.code, el)
        assert _lib.lib().cc_digest_allreduce_dev(comm.handle, x.data_ptr(), 64, None) == _lib.CC_ECOMM
        assert _lib.lib().cc_comm_wait(comm.handle, None, 100) == _lib.CC_ECOMM
        torch.cuda.synchronize()  # the stall ends; nothing of the aborted comm is left running
    finally:
        monkeypatch.delenv("CC_INJECT_EXCHANGE_STALL_MS")
        comm.abort()
