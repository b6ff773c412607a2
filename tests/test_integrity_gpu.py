"""Per-page CRC persistence end to end on the device (SURVEY §8f row 4,
VERDICT r1 "what's missing" 1): the write path keeps the sidecar tables
current, so an integrity job after client writes finds NO bad pages; a write
that bypasses its table is stale (refreshed, never condemned); bit rot is
reported page-exact.  Device path: cc_apply_log_delta_dev keeps the CRC table
current, cc_pcrc_store persists it, cc_integrity_check rehashes every page
(cc_scan_files) against the tables."""
import os

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


def test_write_path_tables_then_job_then_bit_rot(dev, oracle, tmp_path):
    from curve_amd import crc as C
    from curve_amd import integrity as I
    from curve_amd.chunkfile import ChunkFileMetaPage, chunk_file_name, write_chunk_file
    chunk, pb, n = 1 << 20, 4096, 8
    ppc = chunk // pb
    d = tmp_path / "data"
    d.mkdir()
    rng = np.random.default_rng(8)
    host = rng.integers(0, 256, n * chunk, dtype=np.uint8)
    paths = []
    for c in range(n):
        paths.append(str(d / chunk_file_name(c + 1)))
        write_chunk_file(paths[-1], ChunkFileMetaPage(sn=c + 1).encode(), host[c * chunk:(c + 1) * chunk].tobytes())
    pool = torch.from_numpy(host).to(dev)
    crcs = C.page_crc(pool, pb)
    for c in range(n):  # tables of the freshly written chunks
        I.store_table(paths[c], crcs[c * ppc:(c + 1) * ppc], pb)
    # an ordered write log over chunks 0..n-2, applied on the device in delta
    # mode (the stored CRCs kept current by linearity) and written to the files
    U = 500
    lens = rng.integers(1, 4097, U)
    cidx = rng.integers(0, n - 1, U)
    dst = cidx * chunk + rng.integers(0, chunk - 4096, U)
    src = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    soff = rng.integers(0, (1 << 20) - 4096, U)
    C.apply_updates(pool, crcs, torch.from_numpy(src).to(dev), dst, soff, lens, pb, delta=True)
    for i in range(U):  # the datastore's pwrite of the same log, in order
        with open(paths[cidx[i]], "r+b") as f:
            f.seek(4096 + int(dst[i] % chunk))
            f.write(src[soff[i]:soff[i] + lens[i]].tobytes())
    for c in sorted(set(cidx.tolist())):  # persist the touched chunks' tables
        I.store_table(paths[c], crcs[c * ppc:(c + 1) * ppc], pb)
    svc = I.IntegrityService(chunk_size=chunk, batch=3)
    try:
        svc.ScheduleJob(1, 1, str(d))
        j = svc.wait(1, 120)
        assert j.state == I.IntegrityJobState.FINISHED, j.error
        assert len(j.results) == n and all(r.table == "ok" and r.bad_pages == 0 for r in j.results), j.results
        # the tables hold exactly the oracle's CRCs of the final bytes
        for c in range(n):
            _, tab = I.load_table(I.sidecar_path(paths[c]))
            with open(paths[c], "rb") as f:
                data = np.frombuffer(f.read()[4096:], dtype=np.uint8)
            assert (tab == oracle.page_crcs(data, pb)).all()
        # a write that skips its table: stale -> refreshed, no bad pages
        with open(paths[2], "r+b") as f:
            f.seek(4096 + 5000)
            f.write(b"no table update")
        st = os.stat(paths[2])
        os.utime(paths[2], ns=(st.st_atime_ns, st.st_mtime_ns + 1_000_000))  # a later write's mtime
        svc.ScheduleJob(2, 1, str(d))
        j = svc.wait(2, 120)
        res = {r.name: r for r in j.results}
        assert res[chunk_file_name(3)].table == "refreshed" and res[chunk_file_name(3)].bad_pages == 0
        assert all(r.table == "ok" and r.bad_pages == 0 for k, r in res.items() if k != chunk_file_name(3))
        # bit rot: a flipped byte with the mtime left as it was
        p = paths[n - 1]
        st = os.stat(p)
        with open(p, "r+b") as f:
            f.seek(4096 + 200 * pb + 1)
            b = f.read(1)
            f.seek(4096 + 200 * pb + 1)
            f.write(bytes([b[0] ^ 0x04]))
        os.utime(p, ns=(st.st_atime_ns, st.st_mtime_ns))
        svc.ScheduleJob(3, 1, str(d))
        j = svc.wait(3, 120)
        res = {r.name: r for r in j.results}
        r = res[chunk_file_name(n)]
        assert (r.table, r.bad_pages, r.first_bad, r.bad_list) == ("ok", 1, 200, [200])
        assert all(x.bad_pages == 0 for k, x in res.items() if k != chunk_file_name(n))
    finally:
        svc.close()


def _flip(path, off, restore_mtime=True):
    st = os.stat(path)
    with open(path, "r+b") as f:
        f.seek(off)
        b = f.read(1)
        f.seek(off)
        f.write(bytes([b[0] ^ 0x10]))
    if restore_mtime:  # bit rot: the bytes change, the file's identity does not
        os.utime(path, ns=(st.st_atime_ns, st.st_mtime_ns))


def test_service_at_product_geometry(dev, oracle, tmp_path):
    """The C++ IntegrityService (through its C ABI, curve_amd/host/libcurvehost.so)
    over 12 chunk files of 16 MiB + 4 KiB -- one cc_integrity_check call whose
    cc_scan_files spans two staging batches (7 files a slot) -- with, in one
    job: bit rot in the LAST page (4095) of a chunk in the second batch, a
    stale table (a write that skipped it), a corrupt table, a chunk whose
    metapage header fails its CRC and an unreadable chunk; then a truncated
    and an extended chunk file (CC_EFORMAT, FileFormatError in the reference).
    The per-file failures are those files' results; the job still checks
    every chunk."""
    import time
    from curve_amd import _lib
    from curve_amd import integrity as I
    from curve_amd.chunkfile import ChunkFileMetaPage, chunk_file_name, write_chunk_file
    chunk, meta, pb, n = 16 << 20, 4096, 4096, 12
    d = tmp_path / "data"
    d.mkdir()
    rng = np.random.default_rng(12)
    paths, old = [], time.time_ns() - 30 * 10**9
    for c in range(n):
        p = str(d / chunk_file_name(c + 1))
        write_chunk_file(p, ChunkFileMetaPage(sn=c + 1).encode(), rng.integers(0, 256, chunk, dtype=np.uint8).tobytes())
        os.utime(p, ns=(old, old))  # written long before the jobs: tables are not racy
        paths.append(p)
    names = sorted(chunk_file_name(c + 1) for c in range(n))  # std::sort order: chunk_1, chunk_10, chunk_11, chunk_12, chunk_2 ...
    svc = I.IntegrityService(chunk_size=chunk, batch=16)
    try:
        svc.ScheduleJob(1, 1, str(d))
        j = svc.wait(1, 180)
        assert j.state == I.IntegrityJobState.FINISHED, j.error
        assert [r.name for r in j.results] == names
        assert all(r.table == "created" and r.status == 0 and r.bad_pages == 0 for r in j.results), j.results
        for c in (0, n - 1):  # a file of each staging batch: the table is the oracle's CRCs of its data
            _, tab = I.load_table(I.sidecar_path(paths[c]))
            with open(paths[c], "rb") as f:
                assert (tab == oracle.page_crcs(np.frombuffer(f.read()[meta:], dtype=np.uint8), pb)).all()
        rot = names.index(chunk_file_name(9))      # position 11 of 12: the second staging batch
        assert rot >= 7
        _flip(paths[8], meta + 4095 * pb + 77)      # last page of chunk_9
        with open(paths[1], "r+b") as f:            # chunk_2: a write that skipped its table
            f.seek(meta + 123_456)
            f.write(b"unrecorded write")
        tp = I.sidecar_path(paths[6])               # chunk_7: its table rots
        with open(tp, "r+b") as f:
            f.seek(64 + 4 * 1000)
            f.write(b"\xde\xad\xbe\xef")
        _flip(paths[4], 3)                          # chunk_5: metapage header (sn) no longer matches its CRC
        unreadable = os.geteuid() != 0
        if unreadable:
            os.chmod(paths[10], 0)                  # chunk_11: cannot be opened
        svc.ScheduleJob(2, 1, str(d))
        j = svc.wait(2, 180)
        assert j.state == I.IntegrityJobState.FINISHED, j.error
        res = {r.name: r for r in j.results}
        assert len(res) == n
        r = res[chunk_file_name(9)]
        assert (r.table, r.bad_pages, r.first_bad, r.bad_list, r.status) == ("ok", 1, 4095, [4095], 0)
        assert (res[chunk_file_name(2)].table, res[chunk_file_name(2)].bad_pages) == ("refreshed", 0)
        assert (res[chunk_file_name(7)].table, res[chunk_file_name(7)].bad_pages) == ("rebuilt", 0)
        assert res[chunk_file_name(5)].status == _lib.CC_ECORRUPT
        if unreadable:
            assert res[chunk_file_name(11)].status == -13  # -EACCES
        special = {chunk_file_name(c) for c in (9, 2, 7, 5, 11)}
        assert all(x.status == 0 and x.table == "ok" and x.bad_pages == 0 for k, x in res.items() if k not in special)
        # the refreshed / rebuilt tables describe the current bytes
        for c in (1, 6):
            _, tab = I.load_table(I.sidecar_path(paths[c]))
            with open(paths[c], "rb") as f:
                assert (tab == oracle.page_crcs(np.frombuffer(f.read()[meta:], dtype=np.uint8), pb)).all()
        if unreadable:
            os.chmod(paths[10], 0o644)
        # a truncated and an extended chunk file (CSChunkFile::Open: FileFormatError,
        # chunkserver_chunkfile.cpp:233-238): each is its own CC_EFORMAT result, the
        # job still checks the rest, and progress counts them among the listed files
        with open(paths[2], "r+b") as f:
            f.truncate(meta + chunk - 4096)         # chunk_3: lost its last page
        with open(paths[3], "ab") as f:
            f.write(b"x" * 100)                     # chunk_4: 100 bytes too long
        (d / "LOG").write_bytes(b"not a chunk")     # not chunk-named, wrong size: not listed
        svc.ScheduleJob(3, 1, str(d))
        j = svc.wait(3, 180)
        assert j.state == I.IntegrityJobState.FINISHED and j.progress == 100, j.error
        res = {r.name: r for r in j.results}
        assert sorted(res) == names
        for c in (3, 4):
            assert (res[chunk_file_name(c)].status, res[chunk_file_name(c)].bad_pages) == (_lib.CC_EFORMAT, 0)
        assert all(x.status == 0 and x.bad_pages == 0 for k, x in res.items()
                   if k not in {chunk_file_name(c) for c in (3, 4, 5, 9)})
        assert (res[chunk_file_name(9)].bad_pages, res[chunk_file_name(9)].bad_list) == (1, [4095])
        # a file that vanishes between a job's listing and its check: that file's -ENOENT
        got = I.check_files([paths[0], str(d / "chunk_999")],
                            [I.sidecar_path(paths[0]), I.sidecar_path(str(d / "chunk_999"))], chunk, meta, pb)
        assert got[0].status == 0 and got[0].bad_pages == 0 and got[1].status == -2
    finally:
        svc.close()


def test_racy_table_never_condemns_a_same_tick_write(dev, oracle, tmp_path):
    """mtime comes from a coarse clock, so a second write in the same
    tick as the one a table was stored after leaves the identity unchanged.
    Such a table is racy (stamp within a tick of the mtime): a mismatch makes it
    STALE and refreshed, never bad pages; once re-stamped a tick later, real
    bit rot with the mtime restored is reported page-exact again."""
    import time
    from curve_amd import integrity as I
    from curve_amd.chunkfile import ChunkFileMetaPage, chunk_file_name, write_chunk_file
    chunk, pb = 1 << 20, 4096
    d = tmp_path / "data"
    d.mkdir()
    p = str(d / chunk_file_name(1))
    data = np.random.default_rng(1).integers(0, 256, chunk, dtype=np.uint8)
    write_chunk_file(p, ChunkFileMetaPage(sn=1).encode(), data.tobytes())
    # the write path's pwrite and its table in the same tick -- made certain
    # whatever the kernel's tick by an mtime 200 ms ahead of the clock
    m = time.time_ns() + 200_000_000
    os.utime(p, ns=(m, m))
    I.store_table(p, oracle.page_crcs(data, pb), pb)  # racy: stamped before mtime + one tick
    _flip(p, 4096 + 10 * pb)                          # a second write in that tick: same mtime
    svc = I.IntegrityService(chunk_size=chunk)
    try:
        svc.ScheduleJob(1, 1, str(d))
        r = svc.wait(1, 60).results[0]
        assert (r.table, r.bad_pages) == ("refreshed", 0)
        time.sleep(0.5)                               # the clock passes mtime + one tick
        svc.ScheduleJob(2, 1, str(d))                 # racy but matching: re-stamped after the mtime
        r = svc.wait(2, 60).results[0]
        assert (r.table, r.bad_pages) == ("ok", 0)
        _flip(p, 4096 + 200 * pb + 9)                 # bit rot now: reported
        svc.ScheduleJob(3, 1, str(d))
        r = svc.wait(3, 60).results[0]
        assert (r.table, r.bad_pages, r.bad_list) == ("ok", 1, [200])
    finally:
        svc.close()
