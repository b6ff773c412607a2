"""BASELINE config 4 at its own geometry: the scan-service stream of 16 MiB chunk
files through cc_scan_host / cc_scan_host_digest (pinned staging ring, two HIP
streams), with the per-copyset digest computed on the device.

Reference: ScanChunkRequest::OnApply (src/chunkserver/op_request.cpp:769-820)
for every op of ScanManager::ScanJobProcess (scan_manager.cpp:250-283), and
CopysetNode::GetHash (copyset_node.cpp:925-975) for the digest.  Every value is
checked against the oracle; the committed 16 MiB chunk fixture rides along.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

CHUNK = 16 << 20
META = 4096
SLICE = 4 << 20


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from curve_amd import crc as C
    C.engine_init()
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def chunk_set(golden):
    """30 distinct chunk files (> 4 staging batches of 7 at the default 256 MiB
    staging), chunk 0 = the committed chunk_c0ffee fixture."""
    from golden.make_golden import synthetic_chunk
    from curve_amd.chunkfile import ChunkFileMetaPage
    n = 30
    rng = np.random.default_rng(0xC3C3)
    data = rng.integers(0, 256, (n, CHUNK), dtype=np.uint8)
    meta = np.zeros((n, META), dtype=np.uint8)
    for i in range(n):
        meta[i] = np.frombuffer(ChunkFileMetaPage(sn=i + 1).encode(), dtype=np.uint8)
    g = golden["chunk_c0ffee"]
    m0, d0 = synthetic_chunk(g["seed"])
    meta[0] = np.frombuffer(m0, dtype=np.uint8)
    data[0] = d0
    ids = [1, 2, 3, 10, 11, 12, 20, 100, 101, 5, 7, 9, 21, 22, 23, 30, 31, 200, 300, 400, 4, 6, 8, 13, 14, 15, 16,
           17, 18, 19]
    groups = [i % 3 for i in range(n)]
    return data, meta, ids, groups


def _layout(ids, groups):
    from curve_amd.pool import copyset_layout
    return copyset_layout(ids, groups, [CHUNK + META] * len(ids))


def _pin(a):
    return torch.from_numpy(a).pin_memory().numpy()


@pytest.mark.parametrize("mode", ["pinned", "pageable", "mixed"])
def test_scan_host_16mib_stream_with_device_digest(dev, oracle, golden, chunk_set, mode):
    from curve_amd import crc as C
    from curve_amd.scan import chunk_file_name
    data, meta, ids, groups = chunk_set
    n = len(ids)
    if mode == "pinned":
        d_src, m_src = _pin(data), _pin(meta)
        chunks = [(m_src[i], d_src[i]) for i in range(n)]
    elif mode == "pageable":
        chunks = [(meta[i], data[i]) for i in range(n)]
    else:  # every combination of pinned / pageable data and metapage
        d_pin, m_pin = _pin(data), _pin(meta)
        chunks = [(m_pin[i] if i % 3 == 0 else meta[i], d_pin[i] if i % 2 == 0 else data[i]) for i in range(n)]
    lay = _layout(ids, groups)
    mc, sc, fc, dig = C.scan_host(chunks, CHUNK, META, 4096, SLICE, after_bytes=lay.after_bytes,
                                  group=lay.group, n_groups=lay.n_groups)
    for i in range(n):
        ref = oracle.scan_slices(meta[i].tobytes(), data[i].tobytes(), SLICE)
        assert int(mc[i]) == ref[0][2], i
        assert [int(x) for x in sc[i]] == [r[2] for r in ref[1:]], i
        assert int(fc[i]) == oracle.crc32c(meta[i].tobytes() + data[i].tobytes()), i
    g = golden["chunk_c0ffee"]
    assert [(0, META, int(mc[0]))] + [(k * SLICE, SLICE, int(sc[0][k])) for k in range(4)] == \
        [(s["offset"], s["len"], s["crc"]) for s in g["scan_slices"]]
    assert int(fc[0]) == g["whole_file_crc"]
    for gi in range(lay.n_groups):
        files = {chunk_file_name(ids[i]): meta[i].tobytes() + data[i].tobytes()
                 for i in range(n) if lay.group[i] == gi}
        assert str(int(dig[gi])) == oracle.copyset_hash(files), gi
    # the digest-free entry point gives the same CRCs
    mc2, sc2, fc2 = C.scan_host(chunks, CHUNK, META, 4096, SLICE)
    assert (mc2 == mc).all() and (sc2 == sc).all() and (fc2 == fc).all()


def test_scan_host_digest_partials_compose(dev, oracle, chunk_set):
    """Two calls over disjoint halves of the pool (two ranks' shards) give XOR
    partials whose XOR is the whole copyset's GetHash value."""
    from curve_amd import crc as C
    from curve_amd.scan import chunk_file_name
    data, meta, ids, groups = chunk_set
    n = 16
    ids, groups = ids[:n], groups[:n]
    lay = _layout(ids, groups)
    parts = []
    for lo, hi in ((0, 9), (9, n)):
        chunks = [(meta[i], data[i]) for i in range(lo, hi)]
        *_, dig = C.scan_host(chunks, CHUNK, META, 4096, SLICE, after_bytes=lay.after_bytes[lo:hi],
                              group=lay.group[lo:hi], n_groups=lay.n_groups)
        parts.append(dig)
    full = parts[0] ^ parts[1]
    for gi in range(lay.n_groups):
        files = {chunk_file_name(ids[i]): meta[i].tobytes() + data[i].tobytes()
                 for i in range(n) if lay.group[i] == gi}
        assert str(int(full[gi])) == oracle.copyset_hash(files)


def test_scan_host_error_leaves_nothing_in_flight(dev, oracle, chunk_set):
    """A call that fails (a null chunk at index 10 of 20, a copyset index past
    the digest) returns CC_EINVAL before moving a byte, and a normal call made
    right after it gives exact CRCs (no batch of the failed call still owns the
    staging)."""
    from curve_amd import _lib
    from curve_amd import crc as C
    data, meta, ids, _ = chunk_set
    L = _lib.lib()
    n = 20
    arr = (_lib.CcChunkSrc * n)()
    for i in range(n):
        arr[i].meta, arr[i].data = meta[i].ctypes.data, data[i].ctypes.data
    arr[10].data = None
    out = np.zeros(n * 8, dtype=np.uint32)
    p = ctypes.c_void_p(out.ctypes.data)
    assert L.cc_scan_host(arr, n, CHUNK, META, 4096, SLICE, p, None, None) == _lib.CC_EINVAL
    arr[10].data = data[10].ctypes.data
    grp = np.zeros(n, dtype=np.uint32)
    grp[7] = 5
    after = np.zeros(n, dtype=np.uint64)
    dig = np.zeros(4, dtype=np.uint32)
    d = _lib.CcScanDigest(after.ctypes.data, grp.ctypes.data, 4, dig.ctypes.data)
    assert L.cc_scan_host_digest(arr, n, CHUNK, META, 4096, SLICE, p, None, None, ctypes.byref(d)) == _lib.CC_EINVAL
    mc, sc, fc = C.scan_host([(meta[i], data[i]) for i in range(n)], CHUNK, META, 4096, SLICE)
    for i in range(n):
        ref = oracle.scan_slices(meta[i].tobytes(), data[i].tobytes(), SLICE)
        assert int(mc[i]) == ref[0][2] and [int(x) for x in sc[i]] == [r[2] for r in ref[1:]]


def test_crc_bufs_host(dev, oracle):
    """cc_crc_bufs_host: many host buffers of every size (empty, 1 byte,
    unaligned, one larger than a staging slot) in one call == the oracle."""
    from curve_amd import crc as C
    rng = np.random.default_rng(17)
    bufs = [b"", b"x", bytes(range(7))]
    bufs += [rng.integers(0, 256, int(n), dtype=np.uint8)[int(o):] for n, o in
             zip(rng.integers(1, 140000, 600), rng.integers(0, 8, 600))]
    bufs.insert(300, rng.integers(0, 256, (200 << 20) + 13, dtype=np.uint8))  # > one 128 MiB slot
    got = C.crc_bufs_host(bufs)
    want = [oracle.crc32c(b if isinstance(b, bytes) else b.tobytes()) for b in bufs]
    assert got.tolist() == want
