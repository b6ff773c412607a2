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
