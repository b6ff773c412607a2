"""A queue of write logs in one call (cc_apply_logs_dev): the page kernel of
batch k also groups batch k+1's pieces.  The result must be the reference's
write path applied batch after batch, write after write -- CSChunkFile::Write
per request in log order (chunkserver_chunkfile.cpp:287-427, applied by
ChunkOpRequest::OnApply, op_request.cpp:429-481) -- so every case is checked
against in-order host application + the oracle's page CRCs, and against one
cc_apply_log_dev call per batch (bit-identical pool and CRCs)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from curve_amd import crc as C
    C.engine_init()
    return torch.device("cuda", 0)


def u32(t):
    return t.detach().cpu().numpy().view(np.uint32)


def to_dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _batches(rng, sizes, pool_bytes, max_len, pb, pile=False, breakers=True):
    """Per batch: (dst, src_off, lens, src_data, bad set)."""
    out = []
    for n in sizes:
        lens = rng.integers(1, max_len + 1, n).astype(np.uint32)
        span = 8 * pb if pile else pool_bytes - max_len - 1
        dst = rng.integers(0, max(1, span), n).astype(np.uint64)
        src_data = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
        src_off = rng.integers(0, (1 << 16) - max_len - 1, n).astype(np.uint64)
        bad = set()
        if breakers and n:
            for i in rng.choice(n, size=min(n, 3), replace=False):
                kind = int(rng.integers(0, 3))
                if kind == 0:
                    lens[i] = 0
                elif kind == 1:
                    lens[i] = max_len + 1
                else:
                    dst[i], lens[i] = pool_bytes - 1, 2
                bad.add(int(i))
        out.append((dst, src_off, lens, src_data, bad))
    return out


def _host_apply(host, batches):
    want = host.copy()
    for dst, src_off, lens, src_data, bad in batches:
        for i in range(len(lens)):
            if i not in bad:
                want[dst[i]:dst[i] + lens[i]] = src_data[src_off[i]:src_off[i] + lens[i]]
    return want


def _run(dev, oracle, sizes, pb, max_len, delta, seed, pool_bytes=4 << 20, pile=False):
    from curve_amd import crc as C
    rng = np.random.default_rng(seed)
    host = rng.integers(0, 256, pool_bytes, dtype=np.uint8)
    bs = _batches(rng, sizes, pool_bytes, max_len, pb, pile=pile)
    dev_b = [(to_dev(sd, dev), torch.from_numpy(C.log_records(d, so, ln).view(np.uint8)).to(dev), len(ln))
             for d, so, ln, sd, _ in bs]
    # the queue in one call
    d_pool = to_dev(host, dev)
    crcs = C.page_crc(d_pool, pb)
    C.apply_logs(d_pool, crcs, dev_b, max_len, pb, delta=delta)
    # one call per batch
    d_pool2 = to_dev(host, dev)
    crcs2 = C.page_crc(d_pool2, pb)
    for src, d_log, n in dev_b:
        if n:
            C.apply_log(d_pool2, crcs2, src, d_log, n, max_len, pb, delta=delta)
    want = _host_apply(host, bs)
    got = d_pool.cpu().numpy()
    assert (got == want).all(), (sizes, pb, max_len, delta)
    assert (u32(crcs) == oracle.page_crcs(want, pb)).all(), (sizes, pb, max_len, delta)
    assert (d_pool2.cpu().numpy() == got).all() and (u32(crcs2) == u32(crcs)).all()


@pytest.mark.parametrize("delta", [False, True])
@pytest.mark.parametrize("sizes", [[3000, 5000], [3000, 50, 5000, 0, 7000, 64, 65, 2000], [65] * 6, [0, 0, 900],
                                   [20000, 1, 20000, 2, 20000]])
def test_log_queue_matches_in_order_application(dev, oracle, sizes, delta):
    """Batches of the hash-table path back to back (each grouped by the page
    kernel before it), <= 64-write batches between them (the one-launch path:
    the batch after one is grouped by the insert kernel again), empty batches,
    contract breakers in every batch, writes of later batches landing on pages
    earlier batches wrote."""
    _run(dev, oracle, sizes, 4096, 4096, delta, seed=sum(sizes) + 7 * len(sizes) + delta)


@pytest.mark.parametrize("pb,max_len", [(512, 1024), (8192, 8192), (256, 700), (1024, 3000)])
def test_log_queue_geometries(dev, oracle, pb, max_len):
    """Other page sizes (8 KiB pages: the 12-wave page kernel groups the next
    batch in 768-piece chunks) and writes of up to several pages."""
    for delta in (False, True):
        _run(dev, oracle, [4000, 100, 6000, 3000], pb, max_len, delta, seed=pb + max_len + delta)


@pytest.mark.parametrize("delta", [False, True])
def test_log_queue_hot_pages(dev, oracle, delta):
    """Every batch piled onto 8 pages (lists longer than 64 pieces: the wave
    replays its batch's log in place), so a batch's grouping and the previous
    batch's hot-page replay share a kernel."""
    _run(dev, oracle, [700, 900, 65, 1200], 4096, 4096, delta, seed=99 + delta, pile=True)


def test_log_queue_large_batches(dev, oracle):
    """Four 65,536-write batches (the bench's shape) over a 256 MiB pool: every
    page kernel grid full, the grouped batch's head segments over all 256
    blocks."""
    _run(dev, oracle, [65536] * 4, 4096, 4096, False, seed=4242, pool_bytes=256 << 20)


@pytest.mark.timeout(300)
def test_log_queue_grid_wider_than_insert_blocks(dev):
    """A device with more CUs than kInsertBlocks (256; e.g. a 304-CU part):
    the page kernel of a batch whose successor it groups runs on kInsertBlocks
    workgroups (one head segment each) instead of skipping the grouping.  The
    large-batch cases run again in a child process whose engine sizes every
    grid for 304 CUs ($CC_TEST_CUS, read when the device context is made)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CC_TEST_CUS="304")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        os.path.join(root, "tests", "test_log_queue.py") + "::test_log_queue_large_batches",
                        os.path.join(root, "tests", "test_log_queue.py") + "::test_log_queue_hot_pages"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "3 passed" in r.stdout, r.stdout[-2000:]


def test_log_queue_arguments(dev):
    """Validation before anything is enqueued: a batch with records but no
    pointers, a misaligned source, too small a work buffer."""
    import ctypes
    from curve_amd import _lib
    from curve_amd import crc as C
    L = _lib.lib()
    pool = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
    crcs = C.page_crc(pool, 4096)
    need = int(L.cc_apply_logs_work_bytes(100, 4096, 4096))
    assert need > 0 and L.cc_apply_logs_work_bytes(100, 0, 4096) == 0
    work = torch.empty(need, dtype=torch.uint8, device=dev)
    log = torch.zeros(100 * 24, dtype=torch.uint8, device=dev)
    src = torch.zeros(4096, dtype=torch.uint8, device=dev)
    arr = (_lib.CcLogBatch * 2)()
    arr[0].d_src, arr[0].d_log, arr[0].n_updates = src.data_ptr(), log.data_ptr(), 100
    arr[1].d_src, arr[1].d_log, arr[1].n_updates = None, None, 5
    s = torch.cuda.current_stream().cuda_stream

    def call(n, wb=need):
        return L.cc_apply_logs_dev(pool.data_ptr(), pool.numel(), 4096, ctypes.cast(arr, ctypes.c_void_p), n, 4096,
                                   crcs.data_ptr(), 0, work.data_ptr(), wb, s)
    assert call(2) == _lib.CC_EINVAL  # batch 1: records without pointers
    arr[1].d_src, arr[1].d_log = src.data_ptr() + 1, log.data_ptr()
    assert call(2) == _lib.CC_EINVAL  # misaligned source
    assert call(1, need - 1) == _lib.CC_EINVAL
    assert call(0) == 0
    arr[1].d_src = src.data_ptr()
    arr[1].n_updates = 0
    assert call(2) == 0  # 100 zero-length records (contract breakers: nothing applied) + an empty batch
    torch.cuda.synchronize()
    assert int(pool.sum()) == 0


def test_log_queue_streams_trim_and_mixed_calls(dev, oracle):
    """The queue's two tables are the halves of its stream's engine table: a
    queue on a second stream, single calls on the same stream between queues
    (they use the whole, larger table), and a queue after cc_engine_trim (the
    table rebuilt) all leave the pool and CRCs of in-order application."""
    from curve_amd import _lib
    from curve_amd import crc as C
    rng = np.random.default_rng(515)
    pb, max_len, pool_bytes = 4096, 4096, 8 << 20
    host = rng.integers(0, 256, pool_bytes, dtype=np.uint8)
    bs = _batches(rng, [2000, 3000, 70, 2500, 1800, 4000], pool_bytes, max_len, pb)
    dev_b = [(to_dev(sd, dev), torch.from_numpy(C.log_records(d, so, ln).view(np.uint8)).to(dev), len(ln))
             for d, so, ln, sd, _ in bs]
    d_pool = to_dev(host, dev)
    crcs = C.page_crc(d_pool, pb)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        C.apply_logs(d_pool, crcs, dev_b[:2], max_len, pb, stream=side)  # a queue on another stream
        src, d_log, n = dev_b[2]
        C.apply_log(d_pool, crcs, src, d_log, n, max_len, pb, stream=side)  # a single call between queues
        C.apply_logs(d_pool, crcs, dev_b[3:4], max_len, pb, stream=side)  # a queue of one
    side.synchronize()
    assert _lib.lib().cc_engine_trim() == 0
    C.apply_logs(d_pool, crcs, dev_b[4:], max_len, pb)  # tables rebuilt after the trim
    torch.cuda.synchronize()
    want = _host_apply(host, bs)
    assert (d_pool.cpu().numpy() == want).all()
    assert (u32(crcs) == oracle.page_crcs(want, pb)).all()
