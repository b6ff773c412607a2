"""The reference's parametrised chunk geometries on the device.

CSDataStore is instantiated over four (chunk size, block size, metapage size)
tuples (test/chunkserver/datastore/datastore_mock_unittest.cpp:4270-4279):
(16 MiB, 4096, 4096), (16 MiB, 4096, 8192), (16 MiB, 512, 8192) and
(16 MiB, 512, 16384); conf/chunkserver.conf:13-22 says a 512-B block size needs
an 8 KiB metapage (the clone bitmap of 32,768 bits is 4 KiB).  What changes on
the scan path:
  * the readMetaPage op hashes the whole metapage (len = chunkMetaPageSize,
    scan_manager.cpp:250-254, :269-271; op_request.cpp:781-794);
  * every chunk file is metapage || 16 MiB, so CopysetNode::GetHash chains
    files of 16 MiB + 8 KiB (copyset_node.cpp:925-975);
  * GetHash(0, chunkSize) covers the metapage and data[0, 16 MiB - meta)
    (chunkserver_chunkfile.cpp:785-811: raw FILE offsets).
The engine's page is the block size here (512 B pages: 32,768 per chunk, 8,192
per 4 MiB slice through the fused epilogue).  Every result is checked against
the oracle on the same bytes, through each entry point that takes a geometry:
cc_pool_scan_dev (+ digest), cc_scan_host_digest, cc_scan_files (and the
directory walkers above it) and DevicePool.chunk_hash."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

CHUNK = 16 << 20
SCAN = 4 << 20
# (block size = engine page, metapage size): datastore_mock_unittest.cpp:4270-4279
GEOMETRIES = [(4096, 4096), (4096, 8192), (512, 8192), (512, 16384)]
IDS = [7, 10, 2, 31]          # chunk_10 < chunk_2 < chunk_31 < chunk_7 in std::sort order
GROUPS = [0, 1, 0, 0]         # two copysets


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _files(meta_bytes, seed):
    """Chunk files of the geometry: V2 metapages (clone chunks with a full
    block bitmap where the metapage has room for it, as 512-B blocks need) and
    random data."""
    from curve_amd.chunkfile import ChunkFileMetaPage
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, (len(IDS), CHUNK), dtype=np.uint8)
    metas = []
    for k, cid in enumerate(IDS):
        if meta_bytes >= 8192:
            bits = CHUNK // 512
            mp = ChunkFileMetaPage(sn=cid, correctedSn=k, location=f"s3://pool/{cid}@{k}".encode(),
                                   bitmap_bits=bits, bitmap=rng.integers(0, 256, bits // 8, dtype=np.uint8).tobytes())
        else:
            mp = ChunkFileMetaPage(sn=cid + 1)
        metas.append(np.frombuffer(mp.encode(meta_bytes), dtype=np.uint8).copy())
    return np.stack(metas), data


def _expected(oracle, meta, data, meta_bytes):
    from curve_amd.scan import chunk_file_name
    mc = [oracle.crc32c(meta[k].tobytes()) for k in range(len(IDS))]
    sc = [[oracle.crc32c(data[k, j * SCAN:(j + 1) * SCAN].tobytes()) for j in range(CHUNK // SCAN)]
          for k in range(len(IDS))]
    fc = [oracle.crc32c(data[k].tobytes(), mc[k]) for k in range(len(IDS))]  # Extend(V(meta), data)
    dig = []
    for g in sorted(set(GROUPS)):
        files = {chunk_file_name(IDS[k]): meta[k].tobytes() + data[k].tobytes()
                 for k in range(len(IDS)) if GROUPS[k] == g}
        dig.append(oracle.copyset_hash(files))
    return mc, sc, fc, dig


@pytest.mark.parametrize("page_bytes,meta_bytes", GEOMETRIES)
def test_pool_scan_geometry(oracle, page_bytes, meta_bytes):
    """cc_pool_scan_dev: page CRCs at the block size, the metapage op over the
    whole metapage, slices, file CRCs and copyset digests over files of
    16 MiB + metapage; plus GetHash ranges of the raw file."""
    _need_gpu()
    from curve_amd import crc as C
    from curve_amd.pool import copyset_layout, pool_scan
    from curve_amd.scan import DevicePool
    dev = torch.device("cuda", 0)
    meta, data = _files(meta_bytes, seed=page_bytes + meta_bytes)
    pool = DevicePool(torch.from_numpy(data).to(dev), torch.from_numpy(meta).to(dev), IDS, page_bytes=page_bytes)
    assert pool.epilogue_ok()
    lay = copyset_layout(IDS, GROUPS, [CHUNK + meta_bytes] * len(IDS))
    after = torch.tensor(lay.after_bytes, dtype=torch.int64, device=dev)
    grp = torch.tensor(lay.group, dtype=torch.int32, device=dev)
    digest = torch.full((lay.n_groups,), -1, dtype=torch.int32, device=dev)
    pool_scan(pool, C.xpow8(after), grp, digest)
    torch.cuda.synchronize()
    mc, sc, fc, dig = _expected(oracle, meta, data, meta_bytes)
    assert C.as_u32(pool.page_crcs) == oracle.page_crcs(data, page_bytes).tolist()
    assert C.as_u32(pool.meta_crcs[:len(IDS)]) == mc
    assert C.as_u32(pool.slice_crcs) == [x for row in sc for x in row]
    assert C.as_u32(pool.file_crcs) == fc
    assert [str(x) for x in C.as_u32(digest)] == dig
    # ScanMaps: the metapage op's len is the metapage size
    maps = pool.scan_maps(1, 100)
    assert len(maps) == len(IDS) * 5
    assert maps[0].len == meta_bytes and maps[0].crc == mc[0] and maps[1].len == SCAN and maps[1].crc == sc[0][0]
    # CSChunkFile::GetHash over the raw FILE: the tools' (0, chunkSize) range
    # (src/tools/chunkserver_client.cpp:142-143) now covers meta_bytes of metapage
    for k in (0, 3):
        raw = meta[k].tobytes() + data[k].tobytes()
        for off, ln in ((0, CHUNK), (meta_bytes, CHUNK), (0, meta_bytes), (meta_bytes - 512, 4096 + 512),
                        (CHUNK + meta_bytes - 8192, 8192)):
            assert pool.chunk_hash(k, off, ln) == oracle.chunk_hash(raw, off, ln), (k, off, ln)


@pytest.mark.parametrize("page_bytes,meta_bytes", GEOMETRIES)
def test_scan_host_digest_geometry(oracle, page_bytes, meta_bytes):
    """cc_scan_host_digest: host-resident chunk files of the geometry through
    the pinned staging pipeline, digests folded on the device."""
    _need_gpu()
    from curve_amd import crc as C
    from curve_amd.pool import copyset_layout
    meta, data = _files(meta_bytes, seed=3 * page_bytes + meta_bytes)
    lay = copyset_layout(IDS, GROUPS, [CHUNK + meta_bytes] * len(IDS))
    chunks = [(meta[k], data[k]) for k in range(len(IDS))]
    got_mc, got_sc, got_fc, got_dig = C.scan_host(chunks, CHUNK, meta_bytes, page_bytes, SCAN,
                                                  after_bytes=lay.after_bytes, group=lay.group,
                                                  n_groups=lay.n_groups)
    mc, sc, fc, dig = _expected(oracle, meta, data, meta_bytes)
    assert got_mc.tolist() == mc
    assert got_sc.tolist() == sc
    assert got_fc.tolist() == fc
    assert [str(int(x)) for x in got_dig] == dig


@pytest.mark.parametrize("page_bytes,meta_bytes", GEOMETRIES)
def test_scan_files_geometry(oracle, tmp_path, page_bytes, meta_bytes):
    """cc_scan_files over chunk files of 16 MiB + metapage on disk (native
    pread into pinned staging), and the two directory walkers built on it:
    ScanJobProcess over a copyset directory and CopysetNode::GetHash."""
    _need_gpu()
    from curve_amd import crc as C
    from curve_amd.chunkfile import copyset_hash_dir, write_chunk_file
    from curve_amd.scan import chunk_file_name, scan_copyset_dir
    meta, data = _files(meta_bytes, seed=5 * page_bytes + meta_bytes)
    d = tmp_path / "data"
    d.mkdir()
    paths = []
    for k, cid in enumerate(IDS):  # one copyset directory holding all four chunks
        p = str(d / chunk_file_name(cid))
        write_chunk_file(p, meta[k].tobytes(), data[k].tobytes())
        paths.append(p)
    assert os.path.getsize(paths[0]) == CHUNK + meta_bytes
    st, got_mc, got_sc, got_fc = C.scan_files(paths + [str(d / "missing")], CHUNK, meta_bytes, page_bytes, SCAN)
    mc, sc, fc, _ = _expected(oracle, meta, data, meta_bytes)
    assert st.tolist()[:4] == [0, 0, 0, 0] and st[4] != 0
    assert got_mc.tolist()[:4] == mc and got_sc.tolist()[:4] == sc and got_fc.tolist()[:4] == fc
    # the whole copyset: std::sort names, chain whole files
    want = oracle.copyset_hash({chunk_file_name(IDS[k]): meta[k].tobytes() + data[k].tobytes()
                                for k in range(len(IDS))})
    assert copyset_hash_dir(str(d), CHUNK, meta_bytes, page_bytes=page_bytes) == want
    # ScanJobProcess over the directory: chunks by id, metapage op then slices
    maps = scan_copyset_dir(str(d), 1, 100, chunk_size=CHUNK, meta_size=meta_bytes, scan_size=SCAN,
                            page_bytes=page_bytes)
    order = sorted(range(len(IDS)), key=lambda k: IDS[k])
    want_maps = []
    for k in order:
        want_maps.append((IDS[k], 0, meta_bytes, mc[k]))
        want_maps += [(IDS[k], j * SCAN, SCAN, sc[k][j]) for j in range(CHUNK // SCAN)]
    assert [(m.chunkId, m.offset, m.len, m.crc) for m in maps] == want_maps
    assert [m.index for m in maps] == list(range(len(want_maps)))
