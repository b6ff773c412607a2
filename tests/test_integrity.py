"""Per-page CRC sidecar format + IntegrityService state machine (CPU parts)."""
import numpy as np
import pytest

from curve_amd import integrity as I


def test_table_roundtrip_and_corruption():
    """cc_pcrc_encode / cc_pcrc_decode: round trip; any flipped header or
    table byte, a truncated table, or a wrong magic is corrupt."""
    pc = np.random.default_rng(0).integers(0, 2**32, 4096, dtype=np.uint64).astype(np.uint32)
    buf = I.encode_table(pc, 4096, chunk_sn=9, data_mtime_ns=123456789, data_size=4096 + (16 << 20))
    h, got = I.decode_table(buf)
    assert (h.page_bytes, h.n_pages, h.chunk_sn, h.data_mtime_ns, h.data_size) == (4096, 4096, 9, 123456789,
                                                                                    4096 + (16 << 20))
    assert (got == pc).all()
    for pos in (3, 9, 20, 33, 45, 57, 62, 64 + 7, len(buf) - 1):
        b = bytearray(buf)
        b[pos] ^= 0x01
        with pytest.raises(I.TableCorrupt):
            I.decode_table(bytes(b))
    with pytest.raises(I.TableCorrupt):
        I.decode_table(buf[:-4])
    with pytest.raises(I.TableCorrupt):
        I.decode_table(b"")


def test_metapage_sn_and_store_load(tmp_path):
    """cc_chunk_meta_sn follows ChunkFileMetaPage::decode (header CRC, version);
    cc_pcrc_store records the chunk's sn / mtime / size and cc_pcrc_load reads
    them back (no GPU needed: the store only stats the chunk file)."""
    import ctypes
    import os
    from curve_amd import _lib
    from curve_amd.chunkfile import ChunkFileMetaPage, write_chunk_file
    L = _lib.lib()
    meta = ChunkFileMetaPage(sn=77).encode()
    sn = ctypes.c_uint64(0)
    assert L.cc_chunk_meta_sn(meta, 4096, ctypes.byref(sn)) == 0 and sn.value == 77
    clone = ChunkFileMetaPage(sn=5, location=b"s3://bucket/obj@1", bitmap_bits=4096, bitmap=b"\xff" * 64).encode()
    assert L.cc_chunk_meta_sn(clone, 4096, ctypes.byref(sn)) == 0 and sn.value == 5
    bad = bytearray(meta)
    bad[3] ^= 1
    assert L.cc_chunk_meta_sn(bytes(bad), 4096, ctypes.byref(sn)) == _lib.CC_ECORRUPT
    huge = bytearray(meta)
    huge[17:25] = (1 << 40).to_bytes(8, "little")  # location length past the page
    assert L.cc_chunk_meta_sn(bytes(huge), 4096, ctypes.byref(sn)) == _lib.CC_ECORRUPT
    chunk = 1 << 16
    d = tmp_path / "data"
    d.mkdir()
    path = str(d / "chunk_3")
    write_chunk_file(path, meta, bytes(chunk))
    pc = np.arange(chunk // 4096, dtype=np.uint32) * 7
    tp = I.store_table(path, pc, 4096)
    assert tp == I.sidecar_path(path) and os.path.dirname(tp) == str(tmp_path / "pcrc")
    h, got = I.load_table(tp)
    st = os.stat(path)
    assert (h.chunk_sn, h.data_size, h.data_mtime_ns) == (77, st.st_size, st.st_mtime_ns)
    assert (got == pc).all()
    with pytest.raises(I.C.CurveCrcError):  # wrong page count for the file's size
        I.store_table(path, pc[:-1], 4096)


def test_service_state_machine(tmp_path):
    svc = I.IntegrityService()
    try:
        S = I.IntegrityJobState
        assert svc.PauseJob(1) == I.IntegrityOpStatus.FAILURE_UNKNOWN   # unknown job
        assert svc.ScheduleJob(1, 7, str(tmp_path)) == I.IntegrityOpStatus.SUCCESS
        assert svc.ScheduleJob(1, 7, str(tmp_path)) == I.IntegrityOpStatus.FAILURE_UNKNOWN  # duplicate id
        j = svc.wait(1, 20)
        assert j.state == S.FINISHED and j.progress == 100 and j.copyset == 7   # empty dir
        assert svc.CancelJob(1) == I.IntegrityOpStatus.FAILURE_UNKNOWN  # already finished
        assert [x.id for x in svc.ListJobs()] == [1]
        # a job can be paused before it starts, then resumed; or canceled
        svc.PauseJob(1)
        assert svc.ScheduleJob(2, 8, str(tmp_path)) == I.IntegrityOpStatus.SUCCESS
        svc.wait(2, 20)
        assert svc.ResumeJob(2) == I.IntegrityOpStatus.FAILURE_UNKNOWN  # not paused
    finally:
        svc.close()


def _chunk(tmp_path, sn=77, chunk=1 << 16):
    from curve_amd.chunkfile import ChunkFileMetaPage, write_chunk_file
    d = tmp_path / "data"
    d.mkdir(exist_ok=True)
    path = str(d / f"chunk_{sn}")
    write_chunk_file(path, ChunkFileMetaPage(sn=sn).encode(), bytes(chunk))
    return path, np.arange(chunk // 4096, dtype=np.uint32) * 3


def test_racy_table_rule(tmp_path):
    """git's racily-clean rule for tables (cc_pcrc_is_racy): a table stamped
    within one coarse-clock tick of the chunk's mtime cannot prove a later
    write did not keep that mtime, so it never condemns data; one stamped a
    tick or more after it can."""
    import ctypes
    import os
    import time
    from curve_amd import _lib
    L = _lib.lib()
    h = _lib.CcPcrcHeader(4096, 16, 1, 1_000_000_000_123, 4096 * 17, 1_000_000_000_123)
    assert L.cc_pcrc_is_racy(ctypes.byref(h)) == 1          # same instant
    h.stamp_ns = h.data_mtime_ns + 2_000_000_000
    assert L.cc_pcrc_is_racy(ctypes.byref(h)) == 0          # 2 s later
    h.stamp_ns = 0
    assert L.cc_pcrc_is_racy(ctypes.byref(h)) == 1          # a table of the old format (no stamp)
    # a store right after a write whose mtime is "now" is racy; the stamp is the store's clock
    path, pc = _chunk(tmp_path)
    os.utime(path, ns=(time.time_ns(), time.time_ns() + 200_000_000))  # the write's mtime is this tick (or later)
    t0 = time.time_ns()
    hdr, _ = I.load_table(I.store_table(path, pc, 4096))
    assert t0 <= hdr.stamp_ns <= time.time_ns()
    assert L.cc_pcrc_is_racy(ctypes.byref(hdr)) == 1
    # an old write: not racy
    os.utime(path, ns=(time.time_ns(), time.time_ns() - 5_000_000_000))
    hdr, _ = I.load_table(I.store_table(path, pc, 4096))
    assert L.cc_pcrc_is_racy(ctypes.byref(hdr)) == 0


def test_store_expect_refuses_a_later_write(tmp_path):
    """cc_pcrc_store_expect: the CRCs are stored only under the identity the
    caller saw right after its own pwrite; a later write (new mtime) in between
    gets CC_ESTALE and no table."""
    import ctypes
    import os
    from curve_amd import _lib
    L = _lib.lib()
    path, pc = _chunk(tmp_path, sn=5)
    st = os.stat(path)
    expect = _lib.CcPcrcHeader(4096, pc.size, 5, st.st_mtime_ns, st.st_size, 0)
    tp = I.sidecar_path(path)
    os.makedirs(os.path.dirname(tp), exist_ok=True)
    args = (os.fsencode(path), 4096, os.fsencode(tp), pc.ctypes.data, pc.size, 4096)
    assert L.cc_pcrc_store_expect(*args, ctypes.byref(expect)) == 0
    h, got = I.load_table(tp)
    assert (h.chunk_sn, h.data_mtime_ns) == (5, st.st_mtime_ns) and (got == pc).all()
    os.unlink(tp)
    os.utime(path, ns=(st.st_atime_ns, st.st_mtime_ns + 1_000_000))  # a later write landed
    assert L.cc_pcrc_store_expect(*args, ctypes.byref(expect)) == _lib.CC_ESTALE
    assert not os.path.exists(tp)
    expect.chunk_sn = 6  # a snapshot bumped the sn
    os.utime(path, ns=(st.st_atime_ns, st.st_mtime_ns))
    assert L.cc_pcrc_store_expect(*args, ctypes.byref(expect)) == _lib.CC_ESTALE


def test_load_bounds_a_hostile_sidecar(tmp_path):
    """cc_pcrc_load never allocates more than a table of max_pages needs: a
    huge (sparse) sidecar is CC_ECORRUPT at once; header-only loads read 64 B."""
    import ctypes
    import os
    from curve_amd import _lib
    L = _lib.lib()
    path, pc = _chunk(tmp_path, sn=9)
    tp = I.store_table(path, pc, 4096)
    h = _lib.CcPcrcHeader()
    out = np.zeros(pc.size, dtype=np.uint32)
    assert L.cc_pcrc_load(os.fsencode(tp), ctypes.byref(h), None, 0) == 0 and h.n_pages == pc.size
    assert L.cc_pcrc_load(os.fsencode(tp), ctypes.byref(h), out.ctypes.data, pc.size) == 0 and (out == pc).all()
    assert L.cc_pcrc_load(os.fsencode(tp), ctypes.byref(h), out.ctypes.data, pc.size - 1) == _lib.CC_ECORRUPT
    big = str(tmp_path / "hostile.pcrc")
    with open(big, "wb") as f:
        f.write(open(tp, "rb").read()[:64])
        f.truncate(8 << 30)  # 8 GiB, sparse
    assert L.cc_pcrc_load(os.fsencode(big), ctypes.byref(h), out.ctypes.data, pc.size) == _lib.CC_ECORRUPT
    assert L.cc_pcrc_load(os.fsencode(big), ctypes.byref(h), None, 0) == _lib.CC_ECORRUPT  # length != header's


def test_service_is_the_cpp_one():
    """The Python IntegrityService is a facade over the C++ service
    (libcurvehost.so, include/curve_integrity.h): no second state machine."""
    import inspect
    src = inspect.getsource(I.IntegrityService)
    assert "cc_isvc_" in src and "threading" not in src
    svc = I.IntegrityService()
    try:
        assert svc._s
    finally:
        svc.close()


def test_wrong_size_chunk_files_are_format_errors(tmp_path):
    """IntegrityService lists every file NAMED as a chunk or snapshot
    (FileNameOperator, datastore/filename_operator.h:55-62): one whose size is
    not metapage + chunk is that file's CC_EFORMAT result (CSChunkFile::Open's
    FileFormatError, chunkserver_chunkfile.cpp:233-238) instead of vanishing
    from the job, and the job's progress counts it.  Such files never reach the
    device, so a copyset holding only those runs without a GPU."""
    from curve_amd import _lib
    d = tmp_path / "data"
    d.mkdir()
    chunk = 1 << 16
    (d / "chunk_1").write_bytes(bytes(4096 + chunk - 4096))   # truncated: lost its last page
    (d / "chunk_2_snap_3").write_bytes(bytes(4096 + chunk + 1))  # extended snapshot file
    (d / "chunk_x").write_bytes(b"?")                          # not a chunk name: ignored
    (d / "notes").write_bytes(b"hello")                        # ignored
    svc = I.IntegrityService(chunk_size=chunk)
    try:
        svc.ScheduleJob(1, 1, str(d))
        j = svc.wait(1, 30)
        assert j.state == I.IntegrityJobState.FINISHED and j.progress == 100, j.error
        assert [(r.name, r.status, r.bad_pages) for r in j.results] == [
            ("chunk_1", _lib.CC_EFORMAT, 0), ("chunk_2_snap_3", _lib.CC_EFORMAT, 0)]
        assert not (tmp_path / "pcrc" / "chunk_1.pcrc").exists()  # no table for a misfit
    finally:
        svc.close()


def test_store_expect_stamps_with_the_callers_clock(tmp_path):
    """a second same-size write within the mtime's tick keeps the
    chunk's identity.  cc_pcrc_store_expect therefore stamps the table with the
    caller's clock taken before its pwrite (expect->stamp_ns) -- or, given 0,
    with the mtime itself -- never with the store's own later clock, so such a
    table stays racy and a check cannot condemn the newer bytes."""
    import ctypes
    import os
    import time
    from curve_amd import _lib
    L = _lib.lib()
    path, pc = _chunk(tmp_path, sn=4)
    t0 = time.time_ns()                      # the caller's clock before its pwrite
    m = t0 + 1_234_567                       # the pwrite's mtime, in the same tick
    os.utime(path, ns=(m, m))
    st = os.stat(path)
    tp = I.sidecar_path(path)
    os.makedirs(os.path.dirname(tp), exist_ok=True)
    args = (os.fsencode(path), 4096, os.fsencode(tp), pc.ctypes.data, pc.size, 4096)
    time.sleep(0.05)                         # the store runs ticks later
    for stamp, want in ((t0, t0), (0, st.st_mtime_ns)):
        expect = _lib.CcPcrcHeader(4096, pc.size, 4, st.st_mtime_ns, st.st_size, stamp)
        assert L.cc_pcrc_store_expect(*args, ctypes.byref(expect)) == 0
        h, _ = I.load_table(tp)
        assert h.stamp_ns == want and h.data_mtime_ns == st.st_mtime_ns
        assert L.cc_pcrc_is_racy(ctypes.byref(h)) == 1   # a same-tick write cannot be ruled out


def test_racy_rule_boundary_and_whole_second_mtimes():
    """the racy boundary is closed (git's >=: the coarse clock can lag
    a write by a full tick), and an mtime with no sub-second part -- a
    filesystem keeping whole seconds, or FAT's 2 s -- keeps a table racy for 1 s
    (2 s on an even second) instead of one coarse-clock tick."""
    import ctypes
    from curve_amd import _lib
    L = _lib.lib()
    m = 1_000_000_000_123                        # sub-second part: one coarse tick (<= 1 s)
    h = _lib.CcPcrcHeader(4096, 16, 1, m, 4096 * 17, m + 1_000_000_000)
    assert L.cc_pcrc_is_racy(ctypes.byref(h)) == 0
    h.stamp_ns = m + 1_000_000                   # at most one tick after: racy (closed boundary)
    assert L.cc_pcrc_is_racy(ctypes.byref(h)) == 1
    odd = 1_001_000_000_000                      # whole, odd second: 1 s granule
    h = _lib.CcPcrcHeader(4096, 16, 1, odd, 4096 * 17, odd + 600_000_000)
    assert L.cc_pcrc_is_racy(ctypes.byref(h)) == 1
    h.stamp_ns = odd + 1_000_000_000             # exactly one granule: still racy (>=)
    assert L.cc_pcrc_is_racy(ctypes.byref(h)) == 1
    h.stamp_ns = odd + 1_000_000_001
    assert L.cc_pcrc_is_racy(ctypes.byref(h)) == 0
    even = 1_002_000_000_000                     # whole, even second: FAT's 2 s granule
    h = _lib.CcPcrcHeader(4096, 16, 1, even, 4096 * 17, even + 1_500_000_000)
    assert L.cc_pcrc_is_racy(ctypes.byref(h)) == 1
    h.stamp_ns = even + 2_000_000_001
    assert L.cc_pcrc_is_racy(ctypes.byref(h)) == 0
