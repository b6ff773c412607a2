"""GPU parity tests: libcurvecrc's HIP path vs the oracle, bit-exact.

Small/medium cases compare every CRC with the oracle; full-size cases use
size-independent properties (fold of page CRCs == CRC of the whole buffer,
verify of a clean pool == 0 mismatches, corruptions found exactly).
All calls go through the C ABI (ctypes) -- never through the oracle.
"""
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


def u32(t):
    return t.detach().cpu().numpy().view(np.uint32)


def to_dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.parametrize("page_bytes", [4096, 512, 256, 768, 1024, 2048, 8192, 16384, 65536])
@pytest.mark.parametrize("n_pages", [1, 15, 16, 17, 4097])
def test_page_crc_random(dev, oracle, page_bytes, n_pages):
    from curve_amd import crc as C
    rng = np.random.default_rng(page_bytes * 131 + n_pages)
    pages = rng.integers(0, 256, page_bytes * n_pages, dtype=np.uint8)
    got = u32(C.page_crc(to_dev(pages, dev), page_bytes))
    assert (got == oracle.page_crcs(pages, page_bytes)).all()


def test_golden_seeded_pages(dev, oracle, golden):
    from curve_amd import crc as C
    for key in ("seeded_pages", "seeded_pages_512"):
        s = golden[key]
        pages = oracle.splitmix64_bytes(s["seed"], s["n_pages"] * s["page_bytes"])
        assert [int(x) for x in u32(C.page_crc(to_dev(pages, dev), s["page_bytes"]))] == s["crcs"]


def test_golden_chunk(dev, oracle, golden):
    """The committed 16 MiB chunk fixture: all 4096 page CRCs, the 4 ScanMap
    slice CRCs, metapage CRC and chunk hash, derived on the device."""
    from golden.make_golden import synthetic_chunk
    from curve_amd.scan import DevicePool
    g = golden["chunk_c0ffee"]
    meta, data = synthetic_chunk(g["seed"])
    pool = DevicePool(to_dev(data.reshape(1, -1), dev),
                      to_dev(np.frombuffer(meta, dtype=np.uint8).reshape(1, -1), dev), [1])
    pool.scan()
    pc = np.fromfile(os.path.join(os.path.dirname(__file__), "golden", g["page_crcs_file"]), dtype="<u4")
    assert (u32(pool.page_crcs) == pc).all()
    maps = pool.scan_maps(logical_pool_id=1, copyset_id=2)
    assert [(m.offset, m.len, m.crc) for m in maps] == \
        [(s["offset"], s["len"], s["crc"]) for s in g["scan_slices"]]
    assert pool.chunk_hash(0, 0, 16 << 20) == g["chunk_hash_0_chunksize"]
    assert pool.chunk_hash(0, 4096, 8192) == g["chunk_hash_4096_8192"]
    raw = meta + data.tobytes()
    for off, ln in ((0, 1), (100, 5000), (4095, 2), (4097, 123457), ((16 << 20) - 7, 4096 + 7), (0, (16 << 20) + 4096)):
        assert pool.chunk_hash(0, off, ln) == oracle.chunk_hash(raw, off, ln), (off, ln)
    assert (int(u32(pool.file_crcs)[0])) == g["whole_file_crc"]


def test_zero_pages(dev):
    from curve_amd import crc as C
    z = torch.zeros(4096 * 1000, dtype=torch.uint8, device=dev)
    assert (u32(C.page_crc(z, 4096)) == 0x98F94189).all()


def test_unaligned_view_rejected_or_exact(dev, oracle):
    """A 4-byte-aligned offset view works; a non-4-byte-aligned one is refused."""
    from curve_amd import crc as C
    rng = np.random.default_rng(5)
    buf = rng.integers(0, 256, 4096 * 9 + 8, dtype=np.uint8)
    d = to_dev(buf, dev)
    got = u32(C.page_crc(d[4:4 + 4096 * 9], 4096))
    assert (got == oracle.page_crcs(buf[4:4 + 4096 * 9], 4096)).all()
    with pytest.raises(C.CurveCrcError):
        C.page_crc(d[1:1 + 4096 * 9], 4096)


def test_verify_clean_and_corrupt(dev, oracle):
    from curve_amd import crc as C
    rng = np.random.default_rng(11)
    n = 3000
    pages = rng.integers(0, 256, 4096 * n, dtype=np.uint8)
    want = oracle.page_crcs(pages, 4096)
    d = to_dev(pages, dev)
    exp = to_dev(want.view(np.int32), dev)
    cnt = C.page_verify(d, exp, 4096)
    torch.cuda.synchronize()
    assert int(cnt[0]) == 0 and int(cnt[1]) == -1
    bad = [7, 1234, 2999]
    for p in bad:
        d[p * 4096 + 100] ^= 0x40
    cnt = C.page_verify(d, exp, 4096)
    torch.cuda.synchronize()
    assert int(cnt[0]) == len(bad) and int(cnt[1]) == min(bad)


def test_verify_flags_exactly_the_corrupted_pages(dev, oracle):
    """SURVEY §8d C1 sub-case: one corrupted byte in a known page per chunk (plus
    a cluster inside one 64-page tile); the listed bad pages are exactly those."""
    from curve_amd import crc as C
    from curve_amd.scan import DevicePool
    rng = np.random.default_rng(99)
    n, chunk = 64, 1 << 20
    data = torch.empty((n, chunk), dtype=torch.uint8, device=dev)
    data.random_(0, 256)
    meta = torch.zeros((n, 4096), dtype=torch.uint8, device=dev)
    pool = DevicePool(data, meta, list(range(n)), scan_size=chunk)
    good = pool.hash_pages().clone()
    want = set()
    for c in range(n):
        p = int(rng.integers(0, 256))
        data[c, p * 4096 + int(rng.integers(0, 4096))] ^= 0x01
        want.add((c, p))
    for p in (3, 4, 5, 9, 63):  # several bad pages in one tile of chunk 7
        data[7, p * 4096] ^= 0x80
        want.add((7, p))
    assert pool.bad_pages(good) == sorted(want)
    cnt, lst = C.page_verify_list(data, good, 4096, max_bad=10)  # truncated list, full count
    assert int(cnt[0]) == len(want)
    got = [int(x) for x in lst.cpu()]
    assert len(set(got)) == 10 and all((g // 256, g % 256) in want for g in got)
    # the dynamic-M kernel (768-byte pages) through the same sink
    buf = rng.integers(0, 256, 768 * 1000, dtype=np.uint8)
    exp = to_dev(oracle.page_crcs(buf, 768).view(np.int32), dev)
    buf[768 * 17 + 5] ^= 1
    buf[768 * 999] ^= 1
    cnt, lst = C.page_verify_list(to_dev(buf, dev), exp, 768, max_bad=8)
    assert int(cnt[0]) == 2 and int(cnt[1]) == 17
    assert sorted(int(x) for x in lst[:2].cpu()) == [17, 999]


@pytest.mark.parametrize("per_group,unit", [(1024, 4096), (64, 4096), (128, 512), (4, 4 << 20), (3, 4096), (100, 4096), (1, 4096)])
def test_fold(dev, oracle, per_group, unit):
    from curve_amd import crc as C
    rng = np.random.default_rng(per_group + unit)
    groups = 9
    crcs = rng.integers(0, 2**32, per_group * groups, dtype=np.uint64).astype(np.uint32)
    got = u32(C.fold(to_dev(crcs.view(np.int32), dev), per_group, unit))
    from curve_amd.crc import fold_host
    want = [fold_host(crcs[g * per_group:(g + 1) * per_group], unit) for g in range(groups)]
    assert [int(x) for x in got] == want
    # and the fold is the CRC of the concatenation (cross-check with the oracle on real data)
    if unit == 4096 and per_group <= 128:
        data = rng.integers(0, 256, unit * per_group, dtype=np.uint8)
        pc = C.page_crc(to_dev(data, dev), unit)
        assert int(u32(C.fold(pc, per_group, unit))[0]) == oracle.crc32c(data.tobytes())


def test_shift_combine_digest(dev, oracle):
    from curve_amd import crc as C
    rng = np.random.default_rng(2)
    n = 500
    crcs = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    sh = rng.integers(0, 1 << 40, n, dtype=np.int64)
    sh[:5] = [0, 1, 4096, 16 << 20, (16 << 20) + 4096]
    got = u32(C.shift_dev(to_dev(crcs.view(np.int32), dev), to_dev(sh, dev)))
    assert [int(x) for x in got] == [oracle.raw_shift(int(c), int(s)) for c, s in zip(crcs, sh)]
    b = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    got = u32(C.combine_dev(to_dev(crcs.view(np.int32), dev), to_dev(b.view(np.int32), dev), 16 << 20))
    assert [int(x) for x in got] == [oracle.combine(int(x), int(y), 16 << 20) for x, y in zip(crcs, b)]


def test_copyset_digest_matches_reference_chain(dev, oracle, golden):
    """The 5-file fixture of copyset_node_test.cpp:811-835 through the device
    path: page CRCs (files zero-padded into 256-B pages is NOT allowed, so the
    file CRCs come from the CPU primitive) -> digest partials split over two
    'ranks' -> XOR == 1355371765."""
    from conftest import copyset_files
    from curve_amd import crc as C
    from curve_amd.scan import copyset_after_bytes
    files = copyset_files(golden)
    names = list(files)
    sizes = [len(files[k]) for k in names]
    after = copyset_after_bytes(names, sizes)
    fcrc = np.array([C.CRC32(files[k]) for k in names], dtype=np.uint32)
    parts = []
    for sel in ([0, 2, 4], [1, 3]):
        out = C.digest_dev(to_dev(fcrc[sel].view(np.int32), dev), to_dev(np.array(after, dtype=np.int64)[sel], dev),
                           to_dev(np.zeros(len(sel), dtype=np.int32), dev), 1)
        parts.append(int(u32(out)[0]))
    assert str(parts[0] ^ parts[1]) == "1355371765"


def test_copyset_hash_one_chunk_golden(dev, golden, tmp_path):
    """chunkserver_snapshot_test.cpp:339-388 -> "3049021227", on the device
    path twice: the resident pool's fused epilogue digest, and GetHash over a
    real data directory (cc_scan_files preads chunk_1 itself)."""
    from curve_amd import chunkfile as CF
    from curve_amd import crc as C
    from curve_amd.pool import digests_as_hash_strings
    from curve_amd.scan import DevicePool
    g = golden["copyset_hash_one_chunk"]
    data = torch.zeros((1, g["chunk_bytes"]), dtype=torch.uint8, device=dev)
    data[0, : g["blocks"] * g["block_bytes"]] = ord(g["fill"])
    meta_np = np.frombuffer(CF.ChunkFileMetaPage(sn=1).encode(), dtype=np.uint8).reshape(1, -1).copy()
    pool = DevicePool(data, to_dev(meta_np, dev), [1])
    digest = torch.zeros(1, dtype=torch.int32, device=dev)
    pool.scan(after_bytes=torch.zeros(1, dtype=torch.int64, device=dev),
              group=torch.zeros(1, dtype=torch.int32, device=dev), digest=digest)
    assert digests_as_hash_strings(digest) == [g["hash"]]
    d = tmp_path / "data"
    d.mkdir()
    CF.write_chunk_file(str(d / g["file"]), meta_np.tobytes(), data[0].cpu().numpy().tobytes())
    assert CF.copyset_hash_dir(str(d)) == g["hash"]


def test_pool_digest_equals_chained_copyset_hash(dev, oracle):
    """A small pool of real chunk files (metapage + data): the device digest
    equals CopysetNode::GetHash's sorted-name chain computed by the oracle."""
    from curve_amd import crc as C
    from curve_amd.scan import DevicePool, chunk_file_name, copyset_after_bytes
    chunk = 1 << 20  # 1 MiB chunks keep the oracle chain fast
    n = 12
    rng = np.random.default_rng(9)
    data = rng.integers(0, 256, (n, chunk), dtype=np.uint8)
    meta = rng.integers(0, 256, (n, 4096), dtype=np.uint8)
    meta[:, 0] = 2  # FORMAT_VERSION_V2 ...
    meta[4, 0] = 1  # ... except one V1 chunk, which ScanJobProcess skips
    ids = [1, 2, 3, 10, 11, 20, 100, 5, 7, 9, 12, 21]
    pool = DevicePool(to_dev(data, dev), to_dev(meta, dev), ids, scan_size=256 << 10)
    pool.scan()
    names = [chunk_file_name(i) for i in ids]
    groups = [i % 2 for i in range(n)]
    after = [0] * n
    for g in (0, 1):
        mem = [i for i in range(n) if groups[i] == g]
        for i, a in zip(mem, copyset_after_bytes([names[i] for i in mem], [chunk + 4096] * len(mem))):
            after[i] = a
    dig = u32(pool.copyset_digest_partial(names, after, groups, 2))
    for g in (0, 1):
        files = {names[i]: meta[i].tobytes() + data[i].tobytes() for i in range(n) if groups[i] == g}
        assert str(int(dig[g])) == oracle.copyset_hash(files)
    # ScanMaps of every chunk vs the oracle's slice schedule
    maps = pool.scan_maps(1, 1)
    k = 0
    assert len(maps) == 5 * (n - 1)
    for c in range(n):
        if c == 4:
            continue
        ref = oracle.scan_slices(meta[c].tobytes(), data[c].tobytes(), 256 << 10)
        for off, ln, crc in ref:
            m = maps[k]
            assert (m.chunkId, m.offset, m.len, m.crc) == (ids[c], off, ln, crc)
            k += 1


def test_host_path_pageable_and_pinned(dev, oracle):
    from curve_amd import crc as C
    rng = np.random.default_rng(4)
    n = 70000  # > one staging slot (128 MiB / 4 KiB = 32768 pages) -> exercises the 2-slot ring
    pages = rng.integers(0, 256, 4096 * n, dtype=np.uint8)
    want = oracle.page_crcs(pages, 4096, threads=8)
    assert (C.page_crc_host(pages, 4096) == want).all()
    pinned = torch.from_numpy(pages).pin_memory()
    assert (C.page_crc_host(pinned.numpy(), 4096) == want).all()


def test_host_call_blocks_without_spinning(dev):
    """SURVEY §8b threading rule: a blocking *_host call parks the caller (event
    waits use hipEventBlockingSync) instead of burning a bthread worker.  With
    pinned input there is no host copy, so the caller's own CPU time stays a
    small fraction of the wall time of a PCIe-bound 2 GiB call."""
    import time
    from curve_amd import crc as C
    h = torch.empty(2 << 30, dtype=torch.uint8, pin_memory=True)
    h[:] = 7
    a = h.numpy()
    C.page_crc_host(a[: 1 << 20], 4096)  # warm: staging allocated
    w0, c0 = time.perf_counter(), time.thread_time()
    out = C.page_crc_host(a, 4096)
    wall, cpu = time.perf_counter() - w0, time.thread_time() - c0
    assert out.size == (2 << 30) // 4096 and (out == out[0]).all()
    assert cpu < 0.5 * wall, (cpu, wall)


def test_large_pool_properties(dev, oracle):
    """Full-size-ish (2 GiB = 128 chunks): every page CRC equals the oracle's
    (multithreaded) and the fold of all page CRCs equals the CRC of the whole buffer."""
    from curve_amd import crc as C
    n_chunks = 128
    d = torch.empty((n_chunks, 16 << 20), dtype=torch.uint8, device=dev)
    d.random_(0, 256)
    pc = C.page_crc(d, 4096)
    host = d.cpu().numpy()
    assert (u32(pc) == oracle.page_crcs(host, 4096, threads=16)).all()
    whole = C.fold(pc, pc.numel(), 4096)
    assert int(u32(whole)[0]) == oracle.crc32c(host)
    cnt = C.page_verify(d, pc, 4096)
    torch.cuda.synchronize()
    assert int(cnt[0]) == 0


@pytest.mark.parametrize("page_bytes", [256, 1024])
def test_page_kernel_dynamic_tail(dev, oracle, page_bytes):
    """Launches large enough for the page kernel's dynamic tail (>= 8 tiles per
    wave: the last 1/16 of the tiles go out in 64-page chunks through an atomic
    counter): every CRC equals the oracle's, and verify-with-list finds exactly
    the corrupted pages, in the static shares, at the static/dynamic boundary,
    inside the tail and at the very last page (1M + 77 pages: a partial chunk)."""
    from curve_amd import crc as C
    n_pages = (1 << 20) + 77
    d = torch.empty(n_pages * page_bytes, dtype=torch.uint8, device=dev).random_(0, 256)
    pc = C.page_crc(d, page_bytes)
    host = d.cpu().numpy()
    assert (u32(pc) == oracle.page_crcs(host, page_bytes, threads=16)).all()
    tiles = (n_pages + 63) // 64
    bad = {0, 12345, n_pages - 64, n_pages - 1}
    for div in (8, 16):  # the static/dynamic boundary for a 1/8 and a 1/16 tail (engine.hip CC_PAGE_DYN_DIV)
        first_dyn = (tiles - tiles // div) * 64
        bad |= {first_dyn - 1, first_dyn, first_dyn + 64 * 37 + 5}
    bad = sorted(bad)
    for p in bad:
        d[p * page_bytes + 3] ^= 0x80
    cnt, lst = C.page_verify_list(d, pc, page_bytes, max_bad=64)
    torch.cuda.synchronize()
    assert int(cnt[0]) == len(bad) and int(cnt[1]) == bad[0]
    assert sorted(int(x) for x in lst[:len(bad)].cpu()) == bad
    # repeated launches on one stream: the per-call tail counter starts from 0 each time
    for _ in range(3):
        again = C.page_crc(d, page_bytes)
    torch.cuda.synchronize()
    for p in bad:
        d[p * page_bytes + 3] ^= 0x80
    assert torch.equal(C.page_crc(d, page_bytes), pc)
    assert not torch.equal(again, pc)


def test_page_load_probe_diagnostic(dev):
    """cc_page_load_probe_dev (the bench's load-only ceiling): runs the page
    kernel's schedule, static shares and dynamic tail, over 1M + 77 pages and
    writes one word per page, the same words every run; no CRC arithmetic."""
    from curve_amd import crc as C
    n = (1 << 20) + 77
    d = torch.empty(n * 4096, dtype=torch.uint8, device=dev).random_(0, 256)
    a = torch.zeros(n, dtype=torch.int32, device=dev)
    b = torch.ones(n, dtype=torch.int32, device=dev)
    C.page_load_probe(d, a)
    C.page_load_probe(d, b)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    # every page was visited: the word of a page changes when the page does
    d[(n - 1) * 4096] ^= 1
    d[12345 * 4096 + 7] ^= 1
    C.page_load_probe(d, b)
    torch.cuda.synchronize()
    assert sorted(torch.nonzero(a != b).flatten().tolist()) == [12345, n - 1]


def test_full_size_config1_scan_step(dev, oracle):
    """BASELINE config 1 at full size through the bench's own step
    (cc_pool_scan_dev over 1024 x 16 MiB chunk files, 64 copysets), checked by
    size-independent properties against the oracle on the host copy: the
    ordered fold of all 4M page CRCs equals CRC32 of the whole 16 GiB; every
    copyset digest equals CopysetNode::GetHash's sorted-name chain over its 16
    files (metapage || data, chained from 0); 32 sampled chunks' four 4 MiB
    slice CRCs equal the oracle's; 64 sampled pages' CRCs equal the oracle's."""
    from curve_amd import crc as C
    from curve_amd.pool import copyset_layout, pool_scan
    from curve_amd.scan import DevicePool, chunk_file_name
    n, chunk, meta_sz, G = 1024, C.CHUNK_SIZE, C.META_PAGE_SIZE, 64
    data = torch.empty((n, chunk), dtype=torch.uint8, device=dev).random_(0, 256)
    meta = torch.zeros((n, meta_sz), dtype=torch.uint8, device=dev)
    meta[:, 0] = 2
    meta[:, 1:9].random_(0, 256)
    pool = DevicePool(data, meta, list(range(n)), page_bytes=4096)
    lay = copyset_layout(list(range(n)), [i % G for i in range(n)], [chunk + meta_sz] * n)
    after_mult = C.xpow8(torch.tensor(lay.after_bytes, dtype=torch.int64, device=dev))
    group = torch.tensor(lay.group, dtype=torch.int32, device=dev)
    digest = torch.full((lay.n_groups,), 7, dtype=torch.int32, device=dev)
    pool_scan(pool, after_mult, group, digest)
    whole = C.fold(pool.page_crcs, pool.page_crcs.numel(), 4096)
    torch.cuda.synchronize()
    hd, hm = data.cpu().numpy(), meta.cpu().numpy()
    assert int(u32(whole)[0]) == oracle.crc32c(hd.reshape(-1))
    dig = u32(digest)
    for g in range(G):
        mem = sorted((chunk_file_name(i), i) for i in range(n) if i % G == g)
        crc = 0
        for _, i in mem:  # CopysetNode::GetHash: whole files in name order, one chained CRC
            crc = oracle.crc32c(hd[i], oracle.crc32c(hm[i], crc))
        assert int(dig[lay.group[mem[0][1]]]) == crc, g
    rng = np.random.default_rng(0xC1)
    sl = u32(pool.slice_crcs).reshape(n, 4)
    for i in rng.choice(n, 32, replace=False):
        ref = oracle.scan_slices(hm[i].tobytes(), hd[i].tobytes(), C.SCAN_SIZE)
        assert [int(x) for x in sl[i]] == [c for (_, _, c) in ref[1:]]
    pc = u32(pool.page_crcs)
    for p in rng.choice(pc.size, 64, replace=False):
        assert int(pc[p]) == oracle.crc32c(hd.reshape(-1)[p * 4096:(p + 1) * 4096])


@pytest.mark.parametrize("meta_sz", [4096, 8192])
def test_pool_scan_fused_metapages_and_tail_reuse(dev, oracle, meta_sz):
    """cc_pool_scan_dev large enough for the page kernel's dynamic tail (300
    chunks = 1,228,800 pages).  A 4 KiB metapage (the page size) rides the data
    launch's tail as chunks of its own -- 300 metapages = 4 full 64-page chunks
    and a partial one; an 8 KiB metapage gets a launch of its own.  Every page,
    metapage and slice CRC and every digest equals the oracle's, and stays so
    over back-to-back scans on one stream and on two streams in turn: each
    launch zeroes the tail-counter slot set its stream's next launch pulls from
    (kernels.hip tail_clear_next), so no call clears them."""
    from curve_amd import crc as C
    from curve_amd.pool import copyset_layout, pool_scan
    from curve_amd.scan import DevicePool, chunk_file_name
    n, chunk, G = 300, C.CHUNK_SIZE, 7
    data = torch.empty((n, chunk), dtype=torch.uint8, device=dev).random_(0, 256)
    meta = torch.empty((n, meta_sz), dtype=torch.uint8, device=dev).random_(0, 256)
    meta[:, 0] = 2
    pool = DevicePool(data, meta, list(range(n)), page_bytes=4096)
    lay = copyset_layout(list(range(n)), [i % G for i in range(n)], [chunk + meta_sz] * n)
    after_mult = C.xpow8(torch.tensor(lay.after_bytes, dtype=torch.int64, device=dev))
    group = torch.tensor(lay.group, dtype=torch.int32, device=dev)
    hd, hm = data.cpu().numpy(), meta.cpu().numpy()
    want_pc = oracle.page_crcs(hd.reshape(-1), 4096, threads=16)
    want_mc = [oracle.crc32c(hm[i].tobytes()) for i in range(n)]
    want_dig = {}
    for g in range(G):
        mem = sorted((chunk_file_name(i), i) for i in range(n) if i % G == g)
        crc = 0
        for _, i in mem:
            crc = oracle.crc32c(hd[i], oracle.crc32c(hm[i], crc))
        want_dig[lay.group[mem[0][1]]] = crc
    rng = np.random.default_rng(0xF5)
    sample = rng.choice(n, 8, replace=False)
    want_sl = {int(i): [c for (_, _, c) in oracle.scan_slices(hm[i].tobytes(), hd[i].tobytes(), C.SCAN_SIZE)[1:]]
               for i in sample}
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    for rep, st in enumerate([0, 0, 1, 0, 1, 1]):
        s = streams[st]
        pool.page_crcs.fill_(0)
        pool.meta_crcs.fill_(0)
        digest = torch.full((lay.n_groups,), rep, dtype=torch.int32, device=dev)
        s.wait_stream(torch.cuda.current_stream())  # after the fills: the scan must not race them
        with torch.cuda.stream(s):
            pool_scan(pool, after_mult, group, digest, stream=s)
        s.synchronize()
        assert (u32(pool.page_crcs) == want_pc).all(), rep
        assert u32(pool.meta_crcs[:n]).tolist() == want_mc, rep
        dig = u32(digest)
        assert all(int(dig[k]) == v for k, v in want_dig.items()), rep
        sl = u32(pool.slice_crcs).reshape(n, 4)
        assert all([int(x) for x in sl[i]] == want_sl[i] for i in want_sl), rep


def test_write_log_full_size_config3(dev, oracle):
    """BASELINE config 3 at full size: a 16 GiB pool (1024 chunks), 65,536 random
    512 B-4 KiB writes in one log (unaligned, straddling, some overlapping).
    Size-independent properties: every page CRC still verifies against the
    final bytes (all 4M pages), and 300 sampled touched pages equal their host
    rebuild -- the original page with every log entry touching it applied in
    log order -- byte for byte, with the oracle's CRC."""
    from curve_amd import crc as C
    n_chunks, pb, U = 1024, 4096, 65536
    pool = torch.empty(n_chunks << 24, dtype=torch.uint8, device=dev).random_(0, 256)
    pcs = C.page_crc(pool, pb)
    src = torch.empty(U * 4096, dtype=torch.uint8, device=dev).random_(0, 256)
    rng = np.random.default_rng(0xC3)
    lens = rng.integers(512, 4097, U).astype(np.uint64)
    dst = rng.integers(0, pool.numel() - 4096, U).astype(np.uint64)
    dst[:64] = np.minimum(dst[64:128] + rng.integers(0, 2048, 64).astype(np.uint64),
                          pool.numel() - 4097)  # guaranteed overlaps
    src_off = rng.integers(0, U * 4096 - 4096, U).astype(np.uint64)
    p0, p1 = dst // pb, (dst + lens - 1) // pb
    touched = np.unique(np.concatenate([p0, p1]))
    sample = rng.choice(touched, 300, replace=False)
    sample = np.unique(np.concatenate([sample, p0[:64]]))  # include overlapped pages
    before = {int(p): pool[int(p) * pb:(int(p) + 1) * pb].cpu().numpy().copy() for p in sample}
    C.apply_updates(pool, pcs, src, dst, src_off, lens, pb)
    cnt = C.page_verify(pool, pcs, pb)
    torch.cuda.synchronize()
    assert int(cnt[0]) == 0  # every page's CRC matches its final bytes
    src_h = src.cpu().numpy()
    pcs_h = u32(pcs)
    for p in sample:
        p = int(p)
        page = before[p]
        lo, hi = p * pb, (p + 1) * pb
        for i in np.flatnonzero((dst < hi) & (dst + lens > lo)):  # log order
            a, b = max(int(dst[i]), lo), min(int(dst[i] + lens[i]), hi)
            s = int(src_off[i]) + (a - int(dst[i]))
            page[a - lo:b - lo] = src_h[s:s + (b - a)]
        assert (pool[lo:hi].cpu().numpy() == page).all(), p
        assert pcs_h[p] == oracle.crc32c(page.tobytes()), p
    del pool, src, pcs
    torch.cuda.empty_cache()


@pytest.mark.parametrize("page_bytes", [4096, 512])
def test_verify_reads_batch(dev, oracle, page_bytes):
    """cc_verify_reads_dev: a batch of reads of every shape (page-aligned as
    CheckRequestOffsetAndLength demands, 512 B blocks, unaligned, empty, one
    spanning the whole pool, one past the end) against a pool with corrupted
    pages: each read reports exactly the corrupted pages it touches."""
    from curve_amd import crc as C
    rng = np.random.default_rng(page_bytes)
    n_pages = 3000
    host = rng.integers(0, 256, n_pages * page_bytes, dtype=np.uint8)
    stored = to_dev(oracle.page_crcs(host, page_bytes).view(np.int32), dev)
    pool = to_dev(host, dev)
    bad_pages = {0, 7, 64, 65, 1999, n_pages - 1}
    for p in bad_pages:
        pool[p * page_bytes + int(rng.integers(0, page_bytes))] ^= 0x10
    total_bytes = n_pages * page_bytes
    reads = [(0, page_bytes), (7 * page_bytes, 3 * page_bytes), (512, 4096), (100, 1), (5 * page_bytes, 0),
             (63 * page_bytes + 17, 2 * page_bytes), (0, total_bytes), (total_bytes - 10, 10),
             (total_bytes - 10, 11), (1500 * page_bytes, 400 * page_bytes)]
    for _ in range(300):
        o = int(rng.integers(0, total_bytes - 1))
        reads.append((o, int(rng.integers(0, min(64 * page_bytes, total_bytes - o) + 1))))
    off, ln = zip(*reads)
    bad, total = C.verify_reads(pool, stored, off, ln, page_bytes)
    got = bad.cpu().numpy()
    want_total = 0
    for i, (o, n) in enumerate(reads):
        if o + n > total_bytes:
            assert got[i] == -1, i
            continue
        touched = set(range(o // page_bytes, (o + n - 1) // page_bytes + 1)) if n else set()
        want = len(touched & bad_pages)
        want_total += want
        assert got[i] == want, (i, o, n)
    assert int(total.item()) == want_total
    # the device-resident entry point (records already in HBM) agrees
    d_reads = to_dev(np.stack([np.array(off, dtype=np.uint64), np.array(ln, dtype=np.uint64)], axis=1)
                     .reshape(-1).view(np.int64), dev)
    bad2 = torch.zeros(len(reads), dtype=torch.int32, device=dev)
    total2 = torch.zeros(1, dtype=torch.int64, device=dev)
    C.verify_read_records(pool, stored, d_reads, len(reads), bad2, total2, page_bytes)
    assert (bad2.cpu().numpy() == got).all() and int(total2.item()) == want_total


def test_verify_reads_full_batch_with_corruption(dev):
    """The bench's read-verify shape at full size (65,536 reads of 1-32 pages
    over the 16 GiB pool): with 300 corrupted pages every read reports exactly
    the corrupted pages it touches -- reads split over waves at page granularity
    and the dynamic tail included -- and the total matches."""
    from curve_amd import crc as C
    pb, n = 4096, 65536
    n_pages = (16 << 30) // pb
    pool = torch.empty(n_pages * pb, dtype=torch.uint8, device=dev).random_(0, 256)
    stored = C.page_crc(pool, pb)
    rng = np.random.default_rng(0xBAD)
    bad_pages = np.unique(rng.integers(0, n_pages, 300))
    for p in bad_pages:
        pool[int(p) * pb + int(rng.integers(0, pb))] ^= 0x01
    first = rng.integers(0, n_pages - 32, n)
    npg = rng.integers(1, 33, n)
    d_reads = torch.from_numpy(np.stack([first * pb, npg * pb], axis=1).reshape(-1).astype(np.int64)).to(dev)
    bad = torch.zeros(n, dtype=torch.int32, device=dev)
    total = torch.zeros(1, dtype=torch.int64, device=dev)
    C.verify_read_records(pool, stored, d_reads, n, bad, total, pb)
    ind = np.zeros(n_pages + 1, dtype=np.int64)
    ind[bad_pages + 1] = 1
    csum = np.cumsum(ind)
    want = csum[first + npg] - csum[first]
    assert (bad.cpu().numpy() == want).all()
    assert int(total.item()) == int(want.sum())


@pytest.mark.parametrize("page_bytes", [4096, 512])
@pytest.mark.parametrize("n_reads", [1, 2, 17, 64, 65])
def test_verify_reads_small_batches(dev, oracle, page_bytes, n_reads):
    """cc_verify_reads_dev for small batches (<= 64 reads take the one-launch
    path: counts and a wave prefix sum in registers, pages split over waves;
    65 takes count + scan + verify): every read shape -- page-aligned, 512 B,
    unaligned, empty, past the end, the whole pool -- reports exactly the
    corrupted pages it touches, and the totals agree."""
    from curve_amd import crc as C
    rng = np.random.default_rng(page_bytes * 1000 + n_reads)
    n_pages = 3000
    host = rng.integers(0, 256, n_pages * page_bytes, dtype=np.uint8)
    stored = to_dev(oracle.page_crcs(host, page_bytes).view(np.int32), dev)
    pool = to_dev(host, dev)
    bad_pages = {0, 7, 64, 65, 1999, n_pages - 1}
    for p in bad_pages:
        pool[p * page_bytes + int(rng.integers(0, page_bytes))] ^= 0x10
    total_bytes = n_pages * page_bytes
    shapes = [(0, total_bytes), (7 * page_bytes, 3 * page_bytes), (total_bytes - 10, 11), (5 * page_bytes, 0),
              (63 * page_bytes + 17, 2 * page_bytes), (total_bytes - 10, 10), (100, 1), (512, 4096)]
    reads = shapes[:n_reads]
    while len(reads) < n_reads:
        o = int(rng.integers(0, total_bytes - 1))
        reads.append((o, int(rng.integers(0, min(40 * page_bytes, total_bytes - o) + 1))))
    off, ln = zip(*reads)
    bad, total = C.verify_reads(pool, stored, off, ln, page_bytes)
    got = bad.cpu().numpy()
    want_total = 0
    for i, (o, n) in enumerate(reads):
        if o + n > total_bytes:
            assert got[i] == -1, i
            continue
        touched = set(range(o // page_bytes, (o + n - 1) // page_bytes + 1)) if n else set()
        want = len(touched & bad_pages)
        want_total += want
        assert got[i] == want, (i, o, n)
    assert int(total.item()) == want_total


def test_beyond_4gib_offsets(dev, oracle):
    """Maximum-size addressing: a 4.25 GiB buffer (byte offsets past 2^32):
    every page CRC, verify finding a page past 4 GiB, and ranges at offsets
    > 2^32 -- no 32-bit index truncation anywhere on the path."""
    from curve_amd import crc as C
    nbytes = (4 << 30) + (256 << 20)
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    d.random_(0, 256)
    pc = C.page_crc(d, 4096)
    host = d.cpu().numpy()
    assert (u32(pc) == oracle.page_crcs(host, 4096, threads=16)).all()
    bad_page = (nbytes >> 12) - 7  # lives above 4 GiB
    d[bad_page * 4096 + 11] ^= 0x40
    cnt = C.page_verify(d, pc, 4096)
    torch.cuda.synchronize()
    assert int(cnt[0]) == 1 and int(cnt[1]) == bad_page
    d[bad_page * 4096 + 11] ^= 0x40
    offs = [(4 << 30) + 1, (4 << 30) - 100, nbytes - 5000, 123]
    lens = [70001, 4096, 5000, (1 << 20)]
    got = u32(C.crc_ranges(d, offs, lens))
    assert [int(x) for x in got] == [oracle.crc32c(host[o:o + l].tobytes()) for o, l in zip(offs, lens)]
    # write log with destinations and sources past 2^31 / 2^32 (64-bit offsets in
    # every lane-to-scalar move of the log kernel), overlapping in log order
    rng = np.random.default_rng(31)
    n = 4000
    lens_u = rng.integers(1, 4097, n).astype(np.uint32)
    dst = rng.integers(0, nbytes - 4096, n).astype(np.uint64)
    dst[:1000] = rng.integers((4 << 30) - 8192, (4 << 30) + 8192, 1000)  # pile-up across the 4 GiB line
    dst[1000:2000] = rng.integers((2 << 30) - 8192, (2 << 30) + 8192, 1000)  # and across 2 GiB
    src_off = rng.integers(0, nbytes - 4096, n).astype(np.uint64)
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev).random_(0, 256)
    C.apply_updates(d, pc, src, dst, src_off, lens_u, 4096)
    src_h = src.cpu().numpy()
    want = host  # in-order host application (host is d's pre-log copy)
    for i in range(n):
        want[dst[i]:dst[i] + lens_u[i]] = src_h[src_off[i]:src_off[i] + lens_u[i]]
    got_h = d.cpu().numpy()
    touched = np.unique(np.concatenate([dst // 4096, (dst + lens_u - 1) // 4096])).astype(np.int64)
    for p in touched:
        assert (got_h[p * 4096:(p + 1) * 4096] == want[p * 4096:(p + 1) * 4096]).all(), p
    pcs = u32(pc)
    for p in touched:
        assert pcs[p] == oracle.crc32c(want[p * 4096:(p + 1) * 4096].tobytes()), p
    del d, pc, src
    torch.cuda.empty_cache()


def test_streams_and_multithread_callers(dev, oracle):
    """Device calls on side streams from several Python threads (apply-thread shape)."""
    import threading
    from curve_amd import crc as C
    rng = np.random.default_rng(8)
    bufs = [rng.integers(0, 256, 4096 * 513, dtype=np.uint8) for _ in range(4)]
    results = [None] * 4

    def work(i):
        s = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(s):
            d = to_dev(bufs[i], dev)
            out = C.page_crc(d, 4096, stream=s)
            s.synchronize()
            results[i] = u32(out)

    ts = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    for i in range(4):
        assert (results[i] == oracle.page_crcs(bufs[i], 4096)).all()


def test_dynamic_tail_concurrent_streams(dev, oracle):
    """Four Python threads, each on a stream of its own, run tail-sized page
    launches (1M + 77 pages of 256 B) back to back at the same time: each stream
    has its own self-resetting tail counters, so every run of every thread
    equals the oracle."""
    import threading
    from curve_amd import crc as C
    n_pages, pb = (1 << 20) + 77, 256
    bufs = [torch.empty(n_pages * pb, dtype=torch.uint8, device=dev).random_(0, 256) for _ in range(4)]
    torch.cuda.synchronize()
    want = [oracle.page_crcs(b.cpu().numpy(), pb, threads=16) for b in bufs]
    bad = []

    def work(i):
        s = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(s):
            outs = [C.page_crc(bufs[i], pb, stream=s) for _ in range(4)]
            s.synchronize()
        for k, o in enumerate(outs):
            if not (u32(o) == want[i]).all():
                bad.append((i, k))

    ts = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert bad == []


@pytest.mark.parametrize("n_pages", [8192 + 5, 20000, 65536 + 3, 262144 + 77])
def test_tiled_geometries(dev, oracle, n_pages):
    """Batches large enough for 2..64-page wave tiles (coalesced CRC stores and
    ballot verify), with a partial last tile; corruptions found exactly."""
    from curve_amd import crc as C
    rng = np.random.default_rng(n_pages)
    pages = rng.integers(0, 256, 256 * n_pages, dtype=np.uint8)
    d = to_dev(pages, dev)
    want = oracle.page_crcs(pages, 256)
    got = C.page_crc(d, 256)
    assert (u32(got) == want).all()
    bad = sorted({3, n_pages // 2, n_pages - 1, int(rng.integers(0, n_pages))})
    for p in bad:
        d[p * 256 + 17] ^= 1
    cnt = C.page_verify(d, got, 256)
    torch.cuda.synchronize()
    assert int(cnt[0]) == len(bad) and int(cnt[1]) == bad[0]


@pytest.mark.parametrize("pinned", [False, True])
def test_scan_host_stream(dev, oracle, pinned):
    """cc_scan_host: host-resident chunk files streamed through the 2-slot pinned
    pipeline -> metapage / slice / file CRCs == the oracle's ScanJobProcess geometry."""
    from curve_amd import crc as C
    chunk, meta, slice_ = 1 << 20, 4096, 256 << 10
    n = 300  # > 2 staging slots' worth of 1 MiB chunks (128 MiB slots)
    rng = np.random.default_rng(77 + pinned)
    pool_d = rng.integers(0, 256, (8, chunk), dtype=np.uint8)
    pool_m = rng.integers(0, 256, (8, meta), dtype=np.uint8)
    if pinned:
        pool_d = torch.from_numpy(pool_d).pin_memory().numpy()
        pool_m = torch.from_numpy(pool_m).pin_memory().numpy()
    chunks = [(pool_m[(i * 3) % 8], pool_d[i % 8]) for i in range(n)]
    mc, sc, fc = C.scan_host(chunks, chunk, meta, 4096, slice_)
    for i in range(n):
        m, d = chunks[i]
        ref = oracle.scan_slices(m.tobytes(), d.tobytes(), slice_)
        assert mc[i] == ref[0][2]
        assert [int(x) for x in sc[i]] == [c for (_, _, c) in ref[1:]]
        assert fc[i] == oracle.crc32c(m.tobytes() + d.tobytes())


@pytest.mark.parametrize("mode", ["log", "delta"])
@pytest.mark.parametrize("page_bytes,n_upd,overlap", [(4096, 3000, False), (4096, 2000, True), (512, 2500, True),
                                                      (256, 1500, True), (8192, 1000, True)])
def test_partial_writes(dev, oracle, page_bytes, n_upd, overlap, mode):
    """cc_apply_log_dev / cc_apply_log_delta_dev:
    unaligned sub-page writes (1 B .. >1 page, straddling pages, overlapping in
    order) -> pool bytes == in-order host application and every page CRC ==
    oracle on the final bytes (touched pages recomputed or delta-updated,
    untouched ones kept)."""
    from curve_amd import crc as C
    rng = np.random.default_rng(n_upd + overlap + page_bytes)
    pool_bytes = 8 << 20
    host = rng.integers(0, 256, pool_bytes, dtype=np.uint8)
    d_pool = to_dev(host, dev)
    crcs = C.page_crc(d_pool, page_bytes)
    lens = rng.integers(512, 4097, n_upd)
    lens[:50] = rng.integers(1, 16, 50)          # tiny writes
    lens[50:60] = page_bytes + 700                 # longer than a page
    span = 64 << 10 if overlap else pool_bytes - 9000
    dst = rng.integers(0, span, n_upd)
    src_data = rng.integers(0, 256, int(lens.sum()) + 8, dtype=np.uint8)
    src_off = np.concatenate([[0], np.cumsum(lens)[:-1]]) + rng.integers(0, 4, n_upd) * 0
    nb = C.apply_updates(d_pool, crcs, to_dev(src_data, dev), dst, src_off, lens, page_bytes, delta=mode == "delta")
    assert nb == 1
    want = host.copy()
    for i in range(n_upd):
        want[dst[i]:dst[i] + lens[i]] = src_data[src_off[i]:src_off[i] + lens[i]]
    got = d_pool.cpu().numpy()
    assert (got == want).all()
    assert (u32(crcs) == oracle.page_crcs(want, page_bytes, threads=8)).all()


@pytest.mark.parametrize("spread", [0, 4000])
@pytest.mark.parametrize("delta", [False, True])
def test_write_log_hot_pages_and_contract(dev, oracle, delta, spread):
    """cc_apply_log_dev with 700 writes piled on a few pages (piece lists longer
    than 64: the owning wave replays the log, strictly in log order), plus
    entries that break the contract (len 0, len > max_len, beyond the pool):
    those are skipped whole, everything else lands as in-order application.
    spread > 0 interleaves that many writes scattered over the pool, so the
    hot pages sit among thousands of touched pages (static shares and the
    dynamic tail of the page kernel)."""
    from curve_amd import crc as C
    rng = np.random.default_rng(77 + spread)
    pool_bytes, pb = 16 << 20 if spread else 1 << 20, 4096
    host = rng.integers(0, 256, pool_bytes, dtype=np.uint8)
    d_pool = to_dev(host, dev)
    crcs = C.page_crc(d_pool, pb)
    n = 700 + spread
    lens = rng.integers(1, 3000, n).astype(np.uint32)
    dst = (rng.integers(0, 3 * pb, n) + 5 * pb).astype(np.uint64)  # pages 5..8
    if spread:
        far = rng.permutation(n)[:spread]
        far = far[~np.isin(far, [3, 100, 101, 650])]
        dst[far] = rng.integers(16 * pb, pool_bytes - 4096, far.size).astype(np.uint64)
    src_off = rng.integers(0, 1 << 16, n).astype(np.uint64)
    src_data = rng.integers(0, 256, (1 << 16) + 4096, dtype=np.uint8)
    bad = [3, 100, 101, 650]
    lens[3] = 0                       # empty
    lens[100] = 3500                  # > max_len below
    dst[101] = pool_bytes - 10        # runs past the pool
    lens[101] = 20
    dst[650] = 1 << 40                # far beyond the pool
    max_len = 3000
    rec = C.log_records(dst, src_off, lens)
    d_log = torch.from_numpy(rec.view(np.uint8)).to(dev)
    C.apply_log(d_pool, crcs, to_dev(src_data, dev), d_log, n, max_len, pb, delta=delta)
    want = host.copy()
    for i in range(n):
        if i in bad:
            continue
        want[dst[i]:dst[i] + lens[i]] = src_data[src_off[i]:src_off[i] + lens[i]]
    got = d_pool.cpu().numpy()
    assert (got == want).all()
    assert (u32(crcs) == oracle.page_crcs(want, pb)).all()


@pytest.mark.parametrize("delta", [False, True])
@pytest.mark.parametrize("page_bytes", [4096, 512])
@pytest.mark.parametrize("n", [1, 7, 64, 65])
def test_write_log_small_logs(dev, oracle, n, page_bytes, delta):
    """Small logs (<= 64 writes of at most one page's length take the one-launch
    path: every wave finds the distinct touched pages from the log in its lanes,
    then replays the writes touching its page in log order): overlapping writes
    on a few pages, straddling writes, scattered writes and contract breakers
    (len 0, len > max_len, past the pool) land exactly as in-order application,
    and every page CRC equals the oracle's (full rehash or delta update)."""
    from curve_amd import crc as C
    rng = np.random.default_rng(n * 31 + page_bytes + delta)
    pool_bytes = 4 << 20
    host = rng.integers(0, 256, pool_bytes, dtype=np.uint8)
    d_pool = to_dev(host, dev)
    crcs = C.page_crc(d_pool, page_bytes)
    max_len = page_bytes
    lens = rng.integers(1, max_len + 1, n).astype(np.uint32)
    dst = rng.integers(0, pool_bytes - max_len, n).astype(np.uint64)
    dst[: n // 2] = rng.integers(3 * page_bytes - 200, 5 * page_bytes, n // 2)  # overlapping, straddling
    src_off = rng.integers(0, (1 << 16) - max_len, n).astype(np.uint64)
    src_data = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
    bad = set()
    if n >= 7:
        lens[1] = 0                          # empty
        lens[3] = max_len + 1                # longer than max_len
        dst[5], lens[5] = pool_bytes - 3, 7  # runs past the pool
        bad = {1, 3, 5}
    rec = C.log_records(dst, src_off, lens)
    d_log = torch.from_numpy(rec.view(np.uint8)).to(dev)
    C.apply_log(d_pool, crcs, to_dev(src_data, dev), d_log, n, max_len, page_bytes, delta=delta)
    want = host.copy()
    for i in range(n):
        if i not in bad:
            want[dst[i]:dst[i] + lens[i]] = src_data[src_off[i]:src_off[i] + lens[i]]
    assert (d_pool.cpu().numpy() == want).all()
    assert (u32(crcs) == oracle.page_crcs(want, page_bytes)).all()


def test_write_log_pseudo_streams_per_thread_and_trim(dev, oracle):
    """The engine keys its per-stream state (the write log's hash table, the
    page kernel's tail counters) by stream.  The null stream is ONE real stream
    (the legacy default stream: one key, enqueues ordered by the engine's
    mutex); hipStreamPerThread is one handle standing for a different real
    stream in each thread, so it is keyed per calling thread.  Four threads
    apply their own logs at the same time through those two handles (two
    threads each); every page lands as in-order application with the oracle's
    CRC.  Then cc_engine_trim frees the cached tables and the next call
    rebuilds."""
    import ctypes
    import threading
    from curve_amd import crc as C
    from curve_amd import _lib
    L = _lib.lib()
    pb, per, n_thr, U = 4096, 4 << 20, 4, 3000
    rng = np.random.default_rng(404)
    host = rng.integers(0, 256, per * n_thr, dtype=np.uint8)
    d_pool = to_dev(host, dev)
    crcs = C.page_crc(d_pool, pb)
    torch.cuda.synchronize()
    src = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    d_src = to_dev(src, dev)
    jobs = []
    for t in range(n_thr):  # thread t writes only into its own 4 MiB
        lens = rng.integers(1, 3 * pb, U).astype(np.uint32)
        dst = (t * per + rng.integers(0, per - 3 * pb, U)).astype(np.uint64)
        so = rng.integers(0, (1 << 20) - 3 * pb, U).astype(np.uint64)
        rec = C.log_records(dst, so, lens)
        need = int(L.cc_apply_log_work_bytes(U, 3 * pb, pb))
        jobs.append((dst, so, lens, torch.from_numpy(rec.view(np.uint8)).to(dev),
                     torch.empty(need, dtype=torch.uint8, device=dev)))
    torch.cuda.synchronize()
    errs = []

    def run(t, handle):
        _, _, _, d_log, work = jobs[t]
        for _ in range(3):  # re-applying a log is idempotent
            rc = L.cc_apply_log_dev(d_pool.data_ptr(), d_pool.numel(), pb, d_src.data_ptr(), d_log.data_ptr(), U,
                                    3 * pb, crcs.data_ptr(), work.data_ptr(), work.numel(), ctypes.c_void_p(handle))
            if rc:
                errs.append((t, rc))

    ths = [threading.Thread(target=run, args=(t, 2 if t % 2 else 0)) for t in range(n_thr)]
    [x.start() for x in ths]
    [x.join() for x in ths]
    torch.cuda.synchronize()
    assert not errs, errs
    want = host.copy()
    for dst, so, lens, _, _ in jobs:
        for i in range(U):
            want[dst[i]:dst[i] + lens[i]] = src[so[i]:so[i] + lens[i]]
    assert (d_pool.cpu().numpy() == want).all()
    assert (u32(crcs) == oracle.page_crcs(want, pb)).all()
    assert L.cc_engine_trim() == 0
    run(0, 0)  # tables rebuilt after the trim
    torch.cuda.synchronize()
    assert not errs and (u32(crcs) == oracle.page_crcs(want, pb)).all()


@pytest.mark.parametrize("seed", range(40))
def test_write_log_random_configs(dev, oracle, seed):
    """Randomised write logs across the geometry space -- page size 256 B..8 KiB,
    1..20000 writes (the one-launch path, and the hash-table path from a handful of
    touched pages to thousands in every workgroup, each workgroup's share cut
    among its waves by SIMD age), max_len up to two pages, overlap density,
    contract breakers, full or delta CRC mode -- against in-order host
    application and the oracle's page CRCs."""
    from curve_amd import crc as C
    rng = np.random.default_rng(1000 + seed)
    pb = int(rng.choice([256, 512, 1024, 4096, 8192]))
    n = int(rng.choice([1, 2, 5, 33, 64, 65, 300, 3000, 20000]))
    max_len = int(rng.integers(1, 2 * pb + 1))
    delta = bool(rng.integers(0, 2))
    pool_bytes = (int(rng.choice([1, 2, 4])) << 20) if n < 20000 else (64 << 20)
    host = rng.integers(0, 256, pool_bytes, dtype=np.uint8)
    d_pool = to_dev(host, dev)
    crcs = C.page_crc(d_pool, pb)
    lens = rng.integers(1, max_len + 1, n).astype(np.uint32)
    span = int(rng.choice([pool_bytes - max_len - 1, 8 * pb]))  # scattered or piled up
    dst = rng.integers(0, max(1, span), n).astype(np.uint64)
    src_off = rng.integers(0, (1 << 16) - max_len - 1, n).astype(np.uint64)
    src_data = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
    bad = set()
    for i in rng.choice(n, size=min(n, int(rng.integers(0, 4))), replace=False):
        kind = int(rng.integers(0, 3))
        if kind == 0:
            lens[i] = 0
        elif kind == 1:
            lens[i] = max_len + 1
        else:
            dst[i], lens[i] = pool_bytes - 1, 2
        bad.add(int(i))
    rec = C.log_records(dst, src_off, lens)
    d_log = torch.from_numpy(rec.view(np.uint8)).to(dev)
    C.apply_log(d_pool, crcs, to_dev(src_data, dev), d_log, n, max_len, pb, delta=delta)
    want = host.copy()
    for i in range(n):
        if i not in bad:
            want[dst[i]:dst[i] + lens[i]] = src_data[src_off[i]:src_off[i] + lens[i]]
    assert (d_pool.cpu().numpy() == want).all(), (pb, n, max_len, delta)
    assert (u32(crcs) == oracle.page_crcs(want, pb)).all(), (pb, n, max_len, delta)


@pytest.mark.parametrize("delta", [False, True])
def test_write_log_many_segments_and_batches(dev, oracle, delta):
    """A log big enough for every layer of the write log's bookkeeping:
    200,000 writes of 1 B .. 3 pages (4 pieces a write: 800,000 pieces, 1,563
    insert chunks, so each of the 256 insert blocks fills its head segment from
    6-7 chunks) over a 1 GiB pool (~260,000 touched pages: waves with more than
    64 heads run several batches, each batch finding its heads across segment
    ends).  Bytes == in-order host application, every page CRC == the oracle."""
    from curve_amd import crc as C
    rng = np.random.default_rng(4242 + delta)
    pb, n = 4096, 200000
    pool_bytes = 1 << 30
    host = rng.integers(0, 256, pool_bytes, dtype=np.uint8)
    d_pool = to_dev(host, dev)
    crcs = C.page_crc(d_pool, pb)
    max_len = 3 * pb
    lens = rng.integers(1, 2 * pb, n).astype(np.uint32)
    long = rng.random(n) < 0.3  # 3-page writes: 4 pieces
    lens[long] = rng.integers(2 * pb, max_len + 1, int(long.sum()))
    dst = rng.integers(0, pool_bytes - max_len, n).astype(np.uint64)
    src_data = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    src_off = rng.integers(0, (1 << 20) - max_len, n).astype(np.uint64)
    rec = C.log_records(dst, src_off, lens)
    d_log = torch.from_numpy(rec.view(np.uint8)).to(dev)
    C.apply_log(d_pool, crcs, to_dev(src_data, dev), d_log, n, max_len, pb, delta=delta)
    want = host
    for i in range(n):
        want[dst[i]:dst[i] + lens[i]] = src_data[src_off[i]:src_off[i] + lens[i]]
    assert (d_pool.cpu().numpy() == want).all()
    assert (u32(crcs) == oracle.page_crcs(want, pb, threads=8)).all()
    del d_pool, crcs
    torch.cuda.empty_cache()


@pytest.mark.parametrize("seed", range(16))
def test_verify_reads_random_configs(dev, oracle, seed):
    """Randomised read batches (1..2000 reads: the one-launch and the count +
    scan paths; page sizes 256 B..8 KiB; aligned, unaligned, empty, past-the-end
    and whole-pool reads) over a pool with random corrupted pages: exact
    per-read bad-page counts."""
    from curve_amd import crc as C
    rng = np.random.default_rng(2000 + seed)
    pb = int(rng.choice([256, 512, 1024, 4096, 8192]))
    n_pages = int(rng.integers(64, 3000))
    host = rng.integers(0, 256, n_pages * pb, dtype=np.uint8)
    stored = to_dev(oracle.page_crcs(host, pb).view(np.int32), dev)
    pool = to_dev(host, dev)
    bad_pages = set(int(p) for p in rng.choice(n_pages, size=int(rng.integers(0, 12)), replace=False))
    for p in bad_pages:
        pool[p * pb + int(rng.integers(0, pb))] ^= 0x04
    total_bytes = n_pages * pb
    n = int(rng.choice([1, 3, 64, 65, 500, 2000]))
    reads = []
    for _ in range(n):
        k = int(rng.integers(0, 10))
        if k == 0:
            reads.append((int(rng.integers(0, total_bytes)), 0))
        elif k == 1:
            o = int(rng.integers(total_bytes - pb, total_bytes))
            reads.append((o, total_bytes - o + int(rng.integers(1, 100))))  # past the end
        elif k == 2:
            reads.append((0, total_bytes))
        else:
            o = int(rng.integers(0, total_bytes - 1))
            reads.append((o, int(rng.integers(1, min(48 * pb, total_bytes - o) + 1))))
    off, ln = zip(*reads)
    bad, total = C.verify_reads(pool, stored, off, ln, pb)
    got = bad.cpu().numpy()
    want_total = 0
    for i, (o, m) in enumerate(reads):
        if o + m > total_bytes:
            assert got[i] == -1, (i, o, m)
            continue
        want = len(set(range(o // pb, (o + m - 1) // pb + 1)) & bad_pages) if m else 0
        want_total += want
        assert got[i] == want, (i, o, m, pb, n)
    assert int(total.item()) == want_total


@pytest.mark.parametrize("page_bytes", [4096, 512])
def test_write_log_delta_keeps_latent_corruption(dev, oracle, page_bytes):
    """cc_apply_log_delta_dev on a pool where some pages were corrupted after
    their CRC was stored: the full rehash (cc_apply_log_dev) would hand those
    pages a fresh CRC over the corrupt bytes; the delta update keeps the
    mismatch, stored' = stored ^ V(old bytes) ^ V(new bytes), so verify still
    flags exactly the corrupted pages after the write, clean pages match the
    oracle, and the pool bytes equal in-order application either way."""
    from curve_amd import crc as C
    rng = np.random.default_rng(page_bytes + 5)
    n_pages = 2048
    pool_bytes = n_pages * page_bytes
    host = rng.integers(0, 256, pool_bytes, dtype=np.uint8)
    stored = oracle.page_crcs(host, page_bytes).copy()
    rotten = sorted({1, 2, 500, 1023, n_pages - 1} | set(rng.integers(0, n_pages, 20).tolist()))
    for p in rotten:  # bit rot after the CRC was written
        host[p * page_bytes + int(rng.integers(0, page_bytes))] ^= 0x08
    d_pool = to_dev(host, dev)
    crcs = to_dev(stored.view(np.int32), dev)
    n = 3000
    lens = rng.integers(1, page_bytes + 300, n).astype(np.uint32)
    dst = rng.integers(0, pool_bytes - page_bytes - 300, n).astype(np.uint64)
    dst[:len(rotten)] = np.array(rotten, dtype=np.uint64) * page_bytes + 3  # write into every rotten page
    dst[:len(rotten)] = np.minimum(dst[:len(rotten)], pool_bytes - page_bytes - 300)
    src_data = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    src_off = rng.integers(0, (1 << 20) - page_bytes - 300, n).astype(np.uint64)
    C.apply_updates(d_pool, crcs, to_dev(src_data, dev), dst, src_off, lens, page_bytes, delta=True)
    want = host.copy()
    for i in range(n):
        want[dst[i]:dst[i] + lens[i]] = src_data[src_off[i]:src_off[i] + lens[i]]
    assert (d_pool.cpu().numpy() == want).all()
    got = u32(crcs)
    old_c = oracle.page_crcs(host, page_bytes)
    new_c = oracle.page_crcs(want, page_bytes)
    assert (got == (stored ^ old_c ^ new_c)).all()
    assert np.flatnonzero(got != new_c).tolist() == rotten  # exactly the rotten pages still fail


def test_crc_ranges_large_batch(dev, oracle):
    """cc_crc_ranges_dev over a batch larger than the grid: 10,000 ranges of
    every shape (empty, 1-3 bytes, unaligned, multi-block, one 3 MiB giant cut
    over several waves' block shares) == the oracle."""
    from curve_amd import crc as C
    rng = np.random.default_rng(4096)
    buf = rng.integers(0, 256, 8 << 20, dtype=np.uint8)
    d = to_dev(buf, dev)
    n = 10000
    lens = rng.integers(0, 70000, n)
    lens[:40] = [0, 1, 2, 3, 4, 5, 255, 256, 257, 4095, 4096, 4097] + list(range(28))
    lens[5000] = 3 << 20
    offs = rng.integers(0, (8 << 20) - lens - 1)
    got = u32(C.crc_ranges(d, offs, lens))
    want = np.array([oracle.crc32c(buf[o:o + l].tobytes()) for o, l in zip(offs, lens)], dtype=np.uint32)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (bad[:10], offs[bad[:3]], lens[bad[:3]])


def test_wal_replay_full_batch(dev, oracle):
    """The bench's WAL-replay batch at full size: 65,536 entries laid out as
    CurveSegment::append writes them (28-byte header, 1-128 KiB of data, each
    entry padded to 4 KiB) over ~4.3 GB, one cc_crc_ranges_dev call -- every
    entry's data CRC equals the oracle's (static shares, segments cut at share
    boundaries and the dynamic tail all exercised)."""
    from curve_amd import crc as C
    rng = np.random.default_rng(0x3A1)
    n = 65536
    real = rng.integers(1, (128 << 10) + 1, n).astype(np.uint64)
    slot = (28 + real + 4095) // 4096 * 4096
    offs = np.concatenate([[0], np.cumsum(slot)[:-1]]).astype(np.uint64) + 4096 + 28
    size = int(offs[-1] + real[-1] + 4096)
    d = torch.empty(size, dtype=torch.uint8, device=dev).random_(0, 256)
    got = u32(C.crc_ranges(d, offs, real))
    host = d.cpu().numpy()
    want = np.array([oracle.crc32c(host[o:o + l]) for o, l in zip(offs.tolist(), real.tolist())], dtype=np.uint32)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (bad[:10], offs[bad[:3]], real[bad[:3]])


@pytest.mark.parametrize("shape", ["tiny_many", "giants"])
def test_crc_ranges_flat_schedule(dev, oracle, shape):
    """Large batches through cc_crc_ranges_dev's flat block schedule (every
    wave an equal share of the batch's 4 KiB blocks, in 2 pieces).
    tiny_many: 300,000 ranges of 0-300 bytes, so a wave's piece spans more than
    one 64-descriptor window, plus empty ranges at tile edges.  giants: ranges of
    up to 24 MiB cut into segments by many wave pieces (segments that start and
    end inside one range: shift-and-XOR combine) next to 0-3 byte ranges."""
    from curve_amd import crc as C
    rng = np.random.default_rng(len(shape) * 7)
    size = 32 << 20
    buf = rng.integers(0, 256, size, dtype=np.uint8)
    d = to_dev(buf, dev)
    if shape == "tiny_many":
        n = 300000
        lens = rng.integers(0, 301, n)
        lens[::97] = 0
        lens[:3] = [0, 0, 0]
        lens[-3:] = [0, 1, 0]
    else:
        n = 9000
        lens = rng.integers(0, 4, n)
        lens[::500] = rng.integers(1 << 20, 24 << 20, lens[::500].size)
        lens[-1] = 24 << 20
    offs = rng.integers(0, size - lens)
    got = u32(C.crc_ranges(d, offs, lens))
    want = np.array([oracle.crc32c(buf[o:o + l].tobytes()) for o, l in zip(offs, lens)], dtype=np.uint32)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (bad[:10], offs[bad[:3]], lens[bad[:3]])


def test_crc_ranges_arbitrary(dev, oracle):
    """cc_crc_ranges_dev: any offset / alignment / length (0 .. > 1 row)."""
    from curve_amd import crc as C
    rng = np.random.default_rng(31)
    buf = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    d = to_dev(buf, dev)
    offs = [0, 0, 1, 3, 5, 0, 2, 0, 1, 3, 7, 1000, 4, 13, (1 << 20) - 1, (1 << 20) - 300]
    lens = [0, 1, 1, 2, 3, 4, 7, 256, 256, 255, 600, 1999, 28, 1, 1, 300]
    offs += rng.integers(0, 900000, 500).tolist()
    lens += rng.integers(0, 70000, 500).tolist()
    got = u32(C.crc_ranges(d, offs, lens))
    want = [oracle.crc32c(buf[o:o + l].tobytes()) for o, l in zip(offs, lens)]
    assert [int(x) for x in got] == want


def _range_batch(rng, size, shape):
    """Offsets / lengths of a range batch: "giants" (ranges of MiBs cut into
    segments by many wave shares, next to 0-3 byte ranges), "wal" (1-128 KiB),
    "tiny" (0-40 bytes, many empties)."""
    if shape == "giants":
        n = 3000
        lens = rng.integers(0, 4, n)
        lens[::300] = rng.integers(1 << 20, 6 << 20, lens[::300].size)
    elif shape == "wal":
        n = 20000
        lens = rng.integers(1, (128 << 10) + 1, n)
    else:
        n = 50000
        lens = rng.integers(0, 41, n)
        lens[::7] = 0
    offs = rng.integers(0, size - lens)
    return offs, lens


def test_crc_ranges_scratch_left_clean_between_calls(dev, oracle):
    """cc_crc_ranges_dev is ONE launch: the tile counts are epoch-tagged words
    the launch computes itself, split ranges meet in per-range accumulator
    pairs, and the tail counters self-reset -- all in the stream's engine-owned
    scratch, never cleared between calls.  Batches of different shapes (split-
    heavy giants, WAL-sized, tiny with empties) run back to back on one stream,
    twice over, each == the oracle: no call sees a previous call's tile words,
    partial XORs or counters.  Then a batch past the cached scratch's size
    (4 Mi + 7 ranges: scratch of its own, allocated and cleared for the call)
    and the cached path again after it; then cc_engine_trim and one more batch."""
    from curve_amd import crc as C
    from curve_amd import _lib
    rng = np.random.default_rng(0xF01D)
    size = 24 << 20
    buf = rng.integers(0, 256, size, dtype=np.uint8)
    d = to_dev(buf, dev)

    def check(offs, lens, sample=None):
        got = u32(C.crc_ranges(d, offs, lens))
        idx = np.arange(len(offs)) if sample is None else sample
        want = np.array([oracle.crc32c(buf[offs[i]:offs[i] + lens[i]].tobytes()) for i in idx], dtype=np.uint32)
        bad = idx[got[idx] != want]
        assert bad.size == 0, (bad[:10], offs[bad[:3]], lens[bad[:3]])

    batches = [_range_batch(rng, size, sh) for sh in ("giants", "wal", "tiny")]
    for _ in range(2):
        for offs, lens in batches:
            check(offs, lens)
    n = (4 << 20) + 7  # past kRangeCacheRanges
    lens = rng.integers(0, 17, n)
    lens[-1] = 5 << 20  # one range cut by many shares
    offs = rng.integers(0, size - lens)
    sample = np.unique(np.concatenate([np.arange(0, n, 211), np.arange(n - 3000, n)]))
    check(offs, lens, sample)
    check(*batches[0])
    # verify on read shares the stream's scratch and epochs: interleaved with
    # range batches it still flags exactly the reads over a rotten page
    crcs = C.page_crc(d, 4096)
    crcs[333] ^= 4
    roff = rng.integers(0, size - (130 << 10), 20000)
    rlen = rng.integers(1, 128 << 10, 20000)
    want_per = (((roff // 4096) <= 333) & (333 <= (roff + rlen - 1) // 4096)).astype(np.int64)
    for k in range(3):
        per, tot = C.verify_reads(d, crcs, roff, rlen)
        assert (per.cpu().numpy() == want_per).all() and int(tot.item()) == int(want_per.sum())
        check(*batches[k])
    assert _lib.lib().cc_engine_trim() == 0
    check(*batches[2])


def test_crc_ranges_streams_and_threads(dev, oracle):
    """Per-stream range scratch: four threads, two on streams of their own and
    two on the null stream (one handle, keyed per calling thread), run batches
    at the same time; every CRC == the oracle."""
    import threading
    from curve_amd import crc as C
    rng = np.random.default_rng(77)
    size = 16 << 20
    buf = rng.integers(0, 256, size, dtype=np.uint8)
    d = to_dev(buf, dev)
    jobs = [_range_batch(rng, size, ("giants", "wal", "tiny", "giants")[t]) for t in range(4)]
    want = [np.array([oracle.crc32c(buf[o:o + l].tobytes()) for o, l in zip(*j)], dtype=np.uint32) for j in jobs]
    torch.cuda.synchronize()
    res, errs = [None] * 4, []

    def run(t):
        try:
            s = torch.cuda.Stream(dev) if t < 2 else None  # None: the null stream, keyed per thread
            for _ in range(3):
                out = C.crc_ranges(d, *jobs[t], stream=s)
            torch.cuda.synchronize()
            res[t] = u32(out)
        except Exception as e:  # surfaced below
            errs.append((t, repr(e)))

    ths = [threading.Thread(target=run, args=(t,)) for t in range(4)]
    [x.start() for x in ths]
    [x.join() for x in ths]
    assert not errs, errs
    for t in range(4):
        assert (res[t] == want[t]).all(), t


def test_crc_ranges_without_every_workgroup_resident(dev, oracle):
    """cc_crc_ranges_dev and cc_verify_reads_dev count their own schedule:
    tile counts come from every workgroup, and a wave never waits for one
    without a bound.  With the process's queues limited to 8 CUs (HSA_CU_MASK)
    the grid of one workgroup per CU cannot be resident at once: the running
    waves give up on the missing tile words after their wait and count those
    tiles themselves.  Range CRCs still == the oracle, verify on read flags
    exactly the reads over the two rotten pages, and the write log (whose
    kernels never wait on another workgroup) still lands as in-order
    application (run in a child process so the mask applies to its queues
    only)."""
    import subprocess
    import sys
    code = r"""
import sys, numpy as np, torch
sys.path.insert(0, %r)
from curve_amd import crc as C
from oracle import oracle as O
rng = np.random.default_rng(5)
size = 8 << 20
buf = rng.integers(0, 256, size, dtype=np.uint8)
d = torch.from_numpy(buf).to("cuda:0")
lens = rng.integers(0, 70000, 4000); lens[::400] = 3 << 20
offs = rng.integers(0, size - lens)
for _ in range(2):
    got = C.crc_ranges(d, offs, lens).cpu().numpy().view(np.uint32)
want = np.array([O.crc32c(buf[o:o + l].tobytes()) for o, l in zip(offs, lens)], dtype=np.uint32)
bad = np.flatnonzero(got != want)
# verify on read, the same schedule: 3,000 reads, pages 17 and 901 rotten
crcs = C.page_crc(d, 4096)
crcs[17] ^= 1
crcs[901] ^= 2
roff = rng.integers(0, size - (130 << 10), 3000)
rlen = rng.integers(1, 128 << 10, 3000)
per, tot = C.verify_reads(d, crcs, roff, rlen)
per = per.cpu().numpy()
hit = [int(((o // 4096) <= p) & (p <= (o + l - 1) // 4096)) for o, l in zip(roff, rlen) for p in (17, 901)]
want_per = np.array(hit, dtype=np.int64).reshape(-1, 2).sum(1)
# the write log on the 8 CUs: 30,000 writes, both modes, twice each (the
# stream's table reused)
ok_log = True
for delta in (False, True):
    for rnd in range(2):
        host = d.cpu().numpy()
        crcs = C.page_crc(d, 4096)
        n = 30000
        lens = rng.integers(1, 4097, n)
        dst = rng.integers(0, size - 4096, n)
        src = rng.integers(0, 256, int(lens.sum()) + 8, dtype=np.uint8)
        soff = np.concatenate([[0], np.cumsum(lens)[:-1]])
        C.apply_updates(d, crcs, torch.from_numpy(src).to("cuda:0"), dst, soff, lens, 4096, delta=delta)
        want_b = host.copy()
        for i in range(n):
            want_b[dst[i]:dst[i] + lens[i]] = src[soff[i]:soff[i] + lens[i]]
        ok_log &= bool((d.cpu().numpy() == want_b).all())
        ok_log &= bool((crcs.cpu().numpy().view(np.uint32) == O.page_crcs(want_b, 4096)).all())
print("bad", bad.size, "verify", int((per != want_per).sum()), int(tot.item()), int(want_per.sum()), "log", ok_log)
sys.exit(1 if bad.size or (per != want_per).any() or int(tot.item()) != int(want_per.sum()) or not ok_log else 0)
""" % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, HSA_CU_MASK="0:0-7")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])


def test_wal_segment_replay_verify(dev, oracle):
    """Synthetic CurveSegment file: header walk on the host, every entry's data
    checksum verified in one device call; a flipped data byte is caught."""
    from curve_amd import wal
    rng = np.random.default_rng(5)
    ents = []
    for i in range(300):
        ln = int(rng.integers(1, 66000))
        ents.append((3, wal.ENTRY_TYPE_DATA, rng.integers(0, 256, ln, dtype=np.uint8).tobytes()))
    seg = bytearray(wal.build_segment(ents))
    hs = wal.parse_segment(bytes(seg))
    assert len(hs) == 300
    d = to_dev(np.frombuffer(bytes(seg), dtype=np.uint8), dev)
    r = wal.verify_segment_dev(d, hs)
    assert r.bad == [] and r.unverified == [] and r.corrupt_header == [] and r.checked == list(range(300))
    assert [int(x) for x in u32(r.crcs)] == [oracle.crc32c(e[2]) for e in ents]
    seg[hs[123].offset + wal.ENTRY_HEADER_SIZE + 5] ^= 0x10
    d = to_dev(np.frombuffer(bytes(seg), dtype=np.uint8), dev)
    assert wal.verify_segment_dev(d, hs).bad == [123]


def test_wal_mixed_checksum_types_and_corrupt_header(dev, oracle):
    """a MURMURHASH32 entry must not shift the indices of later bad
    entries, is reported unverified (never silently skipped), and a corrupt
    last header is reported without hashing its untrusted length."""
    import struct
    from curve_amd import wal
    rng = np.random.default_rng(6)
    ents = [(2, wal.ENTRY_TYPE_DATA, rng.integers(0, 256, int(rng.integers(1, 9000)), dtype=np.uint8).tobytes())
            for _ in range(20)]
    seg = bytearray(wal.build_segment(ents))
    hs = wal.parse_segment(bytes(seg))
    # entry 4 declares the murmur checksum type (header re-sealed with a valid header CRC)
    o = hs[4].offset
    term, mf, dl, real, dck = struct.unpack_from(">qIIII", seg, o)
    struct.pack_into(">qIIII", seg, o, term, (mf & ~0xFF0000) | (wal.CHECKSUM_MURMURHASH32 << 16), dl, real, 0x1234)
    struct.pack_into(">I", seg, o + 24, oracle.crc32c(bytes(seg[o:o + 24])))
    seg[hs[9].offset + wal.ENTRY_HEADER_SIZE] ^= 1       # bad data in entry 9
    seg[hs[15].offset + 3] ^= 1                           # corrupt header of entry 15: the walk stops there
    hs = wal.parse_segment(bytes(seg))
    assert len(hs) == 16 and not hs[15].header_ok and hs[4].checksum_type == wal.CHECKSUM_MURMURHASH32
    r = wal.verify_segment_dev(to_dev(np.frombuffer(bytes(seg), dtype=np.uint8), dev), hs)
    assert r.bad == [9] and r.unverified == [4] and r.corrupt_header == [15]
    assert r.checked == [k for k in range(15) if k != 4]


def test_copyset_dir_real_chunk_files(dev, oracle, tmp_path):
    """CopysetNode::GetHash over a directory of real chunk files (+ a stray file):
    native pread into pinned staging (cc_scan_files) -> combine in std::sort order ==
    the oracle's chained CRC over the same files."""
    from curve_amd import chunkfile as CF
    rng = np.random.default_rng(12)
    chunk = 1 << 20
    files = {}
    for cid in (1, 2, 10, 11, 100, 3):
        meta = CF.ChunkFileMetaPage(sn=cid).encode()
        data = rng.integers(0, 256, chunk, dtype=np.uint8).tobytes()
        CF.write_chunk_file(str(tmp_path / CF.chunk_file_name(cid)), meta, data)
        files[CF.chunk_file_name(cid)] = meta + data
    (tmp_path / "chunk_5_snap_1").write_bytes(b"x" * 5000)  # other geometry -> CPU
    files["chunk_5_snap_1"] = b"x" * 5000
    assert CF.copyset_hash_dir(str(tmp_path), chunk_size=chunk) == oracle.copyset_hash(files)


def test_chunk_service_hash_on_device(dev, golden):
    """GetChunkHash vectors on the device path: the 'a'-filled block of
    chunk_service_test.cpp:563-578 at raw offset 4096 -> "650595490"; raw
    [0, 4096) is the metapage -> the residue constant; ScanMap of the metapage
    op carries the same constant."""
    from curve_amd import chunkfile as CF
    from curve_amd.scan import DevicePool
    data = torch.zeros((2, 1 << 20), dtype=torch.uint8, device=dev)
    data[:, :4096] = ord("a")
    meta = torch.from_numpy(np.frombuffer(CF.ChunkFileMetaPage(sn=1).encode() * 2, dtype=np.uint8).reshape(2, -1).copy()).to(dev)
    pool = DevicePool(data, meta, [1, 2], scan_size=256 << 10)
    pool.scan()
    assert pool.chunk_hash(0, 4096, 4096) == golden["chunk_service_hash"]["hash"]
    assert pool.chunk_hash(1, 0, 4096) == str(golden["metapage_residue"]["crc"])
    maps = pool.scan_maps(1, 1)
    assert maps[0].crc == golden["metapage_residue"]["crc"] and maps[0].len == 4096


def test_scan_copyset_dir(dev, oracle, tmp_path):
    """ScanJobProcess over real chunk files: V2 chunks give metapage + slice
    ScanMaps equal to the oracle's scan_slices; a V1 chunk and a snapshot file
    are not scanned; a follower copy with one flipped byte fails CompareMap on
    exactly the slice holding it."""
    from curve_amd import chunkfile as CF
    from curve_amd.scan import compare_maps, scan_copyset_dir
    chunk, sl = 1 << 20, 256 << 10
    rng = np.random.default_rng(41)
    lead, foll = tmp_path / "lead", tmp_path / "foll"
    lead.mkdir()
    foll.mkdir()
    raws = {}
    for cid, ver in ((3, 2), (12, 2), (7, 1), (40, 2)):
        raw = CF.ChunkFileMetaPage(version=ver, sn=cid).encode() + rng.integers(0, 256, chunk, dtype=np.uint8).tobytes()
        (lead / CF.chunk_file_name(cid)).write_bytes(raw)
        bad = bytearray(raw)
        if cid == 12:
            bad[4096 + 2 * sl + 77] ^= 4  # slice 2 of chunk 12
        (foll / CF.chunk_file_name(cid)).write_bytes(bytes(bad))
        raws[cid] = raw
    (lead / CF.chunk_file_name(3, 5)).write_bytes(b"s" * 1000)  # snapshot: not in the ChunkMap
    ml = scan_copyset_dir(str(lead), 1, 9, chunk_size=chunk, scan_size=sl)
    mf = scan_copyset_dir(str(foll), 1, 9, chunk_size=chunk, scan_size=sl)
    assert [m.chunkId for m in ml] == [3] * 5 + [12] * 5 + [40] * 5
    for cid in (3, 12, 40):
        want = oracle.scan_slices(raws[cid][:4096], raws[cid][4096:], sl)
        got = [(m.offset, m.len, m.crc) for m in ml if m.chunkId == cid]
        assert got == want
    fails = [(a.chunkId, a.offset) for a, b in zip(ml, mf) if not compare_maps(a, [b, b])[0]]
    assert fails == [(12, 2 * sl)]


def test_scan_files(dev, oracle, tmp_path):
    """cc_scan_files: the engine opens/preads real chunk files itself (3 staging
    batches of 1 MiB chunks), metapage / slice / file CRCs == oracle; a missing
    file and short, truncated and extended files get a status and leave the
    others intact."""
    from curve_amd import _lib
    from curve_amd import crc as C
    chunk, meta_b, sl = 1 << 20, 4096, 256 << 10
    rng = np.random.default_rng(77)
    paths, raws = [], []
    for i in range(260):
        raw = rng.integers(0, 256, meta_b + chunk, dtype=np.uint8).tobytes()
        p = tmp_path / f"chunk_{i}"
        p.write_bytes(raw)
        paths.append(str(p))
        raws.append(raw)
    (tmp_path / "short").write_bytes(b"y" * 1000)
    (tmp_path / "truncated").write_bytes(raws[0][:meta_b + chunk - 4096])
    (tmp_path / "extended").write_bytes(raws[1] + b"x" * 4096)
    for at, name in ((5, "missing"), (140, "short"), (141, "truncated"), (200, "extended")):
        paths.insert(at, str(tmp_path / name))
        raws.insert(at, None)
    st, mc, sc, fc = C.scan_files(paths, chunk, meta_b, 4096, sl, io_threads=4)
    # -ENOENT; a size != metapage + chunk is CSChunkFile::Open's FileFormatError
    # (chunkserver_chunkfile.cpp:233-238): CC_EFORMAT, whether short, truncated or extended
    assert st[5] == -2 and [int(st[i]) for i in (140, 141, 200)] == [_lib.CC_EFORMAT] * 3
    for i, raw in enumerate(raws):
        if raw is None:
            continue
        assert st[i] == 0
        m, d = raw[:meta_b], raw[meta_b:]
        want = oracle.scan_slices(m, d, sl)
        assert int(mc[i]) == want[0][2]
        assert [int(x) for x in sc[i]] == [w[2] for w in want[1:]]
        assert int(fc[i]) == oracle.crc32c(raw)
    # slice == page: the per-slice CRCs are the page CRCs of the data part
    st, _, pc, _ = C.scan_files(paths[:3], chunk, meta_b, 4096, 4096)
    assert (st == 0).all()
    for i in range(3):
        d = np.frombuffer(raws[i][meta_b:], dtype=np.uint8)
        assert (pc[i] == oracle.page_crcs(d, 4096)).all()


def test_integrity_job_sidecars(dev, oracle, tmp_path):
    """IntegrityService over real chunk files: first job creates the per-page CRC
    sidecars (== oracle page CRCs); after flipping one data byte and one sidecar
    byte a second job reports exactly that page and the corrupt table."""
    import os
    from curve_amd import chunkfile as CF
    from curve_amd import integrity as I
    rng = np.random.default_rng(21)
    chunk = 1 << 20
    datas = {}
    tmp_path = tmp_path / "data"  # <copyset>/data; sidecars go to <copyset>/pcrc
    tmp_path.mkdir()
    import time
    old = time.time_ns() - 30 * 10**9  # written long before the job: its tables are not racy (cc_pcrc_is_racy)
    for cid in range(1, 8):
        data = rng.integers(0, 256, chunk, dtype=np.uint8)
        CF.write_chunk_file(str(tmp_path / CF.chunk_file_name(cid)), CF.ChunkFileMetaPage(sn=cid).encode(), data.tobytes())
        os.utime(str(tmp_path / CF.chunk_file_name(cid)), ns=(old, old))
        datas[cid] = data
    svc = I.IntegrityService(chunk_size=chunk, batch=3)
    try:
        svc.ScheduleJob(1, 1, str(tmp_path))
        j = svc.wait(1, 120)
        assert j.state == I.IntegrityJobState.FINISHED, j.error
        assert all(r.table == "created" for r in j.results) and len(j.results) == 7
        assert sorted(os.listdir(tmp_path)) == sorted(CF.chunk_file_name(c) for c in datas)  # data dir untouched
        for cid, data in datas.items():
            h, tab = I.load_table(I.sidecar_path(str(tmp_path / CF.chunk_file_name(cid))))
            assert h.chunk_sn == cid and (tab == oracle.page_crcs(data, 4096)).all()
        p3 = str(tmp_path / CF.chunk_file_name(3))
        with open(p3, "r+b") as f:  # data page 77 of chunk 3
            f.seek(4096 + 77 * 4096 + 5)
            b = f.read(1)
            f.seek(4096 + 77 * 4096 + 5)
            f.write(bytes([b[0] ^ 0xFF]))
        s5 = I.sidecar_path(str(tmp_path / CF.chunk_file_name(5)))
        raw = bytearray(open(s5, "rb").read())
        raw[100] ^= 1
        open(s5, "wb").write(bytes(raw))
        # bit rot does not move mtime: restore it, as a flipped bit on the medium would
        st3 = os.stat(p3)
        os.utime(p3, ns=(st3.st_atime_ns, int(I.load_table(I.sidecar_path(p3))[0].data_mtime_ns)))
        svc.ScheduleJob(2, 1, str(tmp_path))
        j = svc.wait(2, 120)
        res = {r.name: r for r in j.results}
        assert res["chunk_3"].bad_pages == 1 and res["chunk_3"].first_bad == 77 and res["chunk_3"].bad_list == [77]
        assert res["chunk_5"].table in ("corrupt", "rebuilt")
        assert all(r.bad_pages == 0 for n, r in res.items() if n != "chunk_3")
    finally:
        svc.close()


def test_host_calls_from_many_threads(dev, oracle):
    """Blocking *_host calls from 6 threads at once (apply-thread shape): the
    per-device submission lock serialises them, every result is exact."""
    import threading
    from curve_amd import crc as C
    rng = np.random.default_rng(44)
    bufs = [rng.integers(0, 256, 4096 * int(rng.integers(1, 3000)), dtype=np.uint8) for _ in range(6)]
    out = [None] * 6
    errs = []

    def work(i):
        try:
            for _ in range(3):
                out[i] = C.page_crc_host(bufs[i], 4096)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=work, args=(i,)) for i in range(6)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errs
    for i in range(6):
        assert (out[i] == oracle.page_crcs(bufs[i], 4096)).all()


@pytest.mark.parametrize("ppc,pps", [(4096, 1024), (256, 64), (256, 256), (512, 2), (1024, 512), (1024, 4), (768, 96)])
def test_scan_epilogue_geometries(dev, oracle, ppc, pps):
    """cc_scan_epilogue_dev (one launch) == fold_host per slice / file, and the
    digest partials == shifted file CRCs XORed per group."""
    from curve_amd import crc as C
    rng = np.random.default_rng(ppc * 7 + pps)
    n, pb = 9, 4096
    pages = rng.integers(0, 2**32, n * ppc, dtype=np.uint64).astype(np.uint32)
    metas = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    S = ppc // pps
    sl = torch.zeros(n * S, dtype=torch.int32, device=dev)
    fc = torch.zeros(n, dtype=torch.int32, device=dev)
    after = rng.integers(0, 1 << 36, n, dtype=np.int64)
    grp = rng.integers(0, 3, n).astype(np.int32)
    dig = torch.zeros(3, dtype=torch.int32, device=dev)
    mult = C.xpow8(to_dev(after, dev))
    assert [int(x) for x in u32(mult)] == [C.shift(0x80000000, int(a)) for a in after]  # x^(8a) * 1
    C.scan_epilogue(to_dev(pages.view(np.int32), dev), to_dev(metas.view(np.int32), dev), n, ppc, pb, pps,
                    sl, fc, mult, to_dev(grp, dev), dig)
    want_sl, want_fc, want_dig = [], [], [0, 0, 0]
    for c in range(n):
        pc = pages[c * ppc:(c + 1) * ppc]
        want_sl += [C.fold_host(pc[k * pps:(k + 1) * pps], pb) for k in range(S)]
        f = C.combine(int(metas[c]), C.fold_host(pc, pb), ppc * pb)
        want_fc.append(f)
        want_dig[grp[c]] ^= C.shift(f, int(after[c]))
    assert [int(x) for x in u32(sl)] == want_sl
    assert [int(x) for x in u32(fc)] == want_fc
    assert [int(x) for x in u32(dig)] == want_dig


def test_per_thread_stream_entries_dropped_at_thread_exit(dev, oracle):
    """hipStreamPerThread scratch is keyed by (handle, thread) and a
    thread's entries are dropped when the thread exits (after its per-thread
    stream drained).  300 short-lived threads in turn -- glibc reuses their
    thread ids -- each run a range batch (cc_crc_ranges_dev: the stream's range
    scratch) on hipStreamPerThread and check it against the oracle; the engine
    holds no more entries afterwards than before (round 4 kept every exited
    thread's scratch, up to 256 entries, then fell back to per-call
    allocations for good, and a new thread could inherit an exited one's)."""
    import ctypes
    import threading
    from curve_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(77)
    buf = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    d_buf = to_dev(buf, dev)
    n = 64
    off = rng.integers(0, (1 << 20) - 8192, n)
    ln = rng.integers(0, 8192, n)
    want = [oracle.crc32c(buf[o:o + k].tobytes()) for o, k in zip(off, ln)]
    rec = np.stack([off, ln], axis=1).astype(np.uint64)
    d_rec = to_dev(rec.view(np.uint8).reshape(-1), dev)
    torch.cuda.synchronize()
    base = int(L.cc_engine_stream_entries())
    errs = []

    def run():
        torch.cuda.set_device(dev)
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        rc = L.cc_crc_ranges_dev(d_buf.data_ptr(), d_rec.data_ptr(), n, out.data_ptr(), ctypes.c_void_p(2))
        if rc:
            errs.append(rc)
            return
        L.cc_engine_stream_entries()  # (no sync here: the exit path waits for the stream)
        torch.cuda.synchronize()
        if [int(x) & 0xFFFFFFFF for x in out.cpu().tolist()] != want:
            errs.append("mismatch")

    for _ in range(300):
        t = threading.Thread(target=run)
        t.start()
        t.join()
    assert not errs, errs[:5]
    assert int(L.cc_engine_stream_entries()) <= base


def test_ranges_and_verify_on_a_cu_masked_stream(dev, oracle):
    """on a stream limited to 32 CUs the range and verify kernels'
    256-workgroup grids run 32 workgroups at a time, so the first waves wait
    for tile counts of workgroups that are not resident; after the bound they
    claim those tiles (one CAS each), count and publish them (kernels.hip
    wait_tiles).  Results must equal the oracle's (ranges: CRC32C of every range,
    butil Value; verify: exactly the corrupted page flagged)."""
    import ctypes
    from curve_amd import crc as C
    from curve_amd import _lib
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                 ctypes.POINTER(ctypes.c_uint32)]
    h = ctypes.c_void_p()
    mask = (ctypes.c_uint32 * 8)(0xFFFFFFFF, 0, 0, 0, 0, 0, 0, 0)
    assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), 8, mask) == 0
    st = torch.cuda.ExternalStream(h.value)
    rng = np.random.default_rng(31)
    host = rng.integers(0, 256, 64 << 20, dtype=np.uint8)
    d = to_dev(host, dev)
    n = 5000
    off = rng.integers(0, host.size - 20000, n).astype(np.uint64)
    ln = rng.integers(0, 20000, n).astype(np.uint64)
    rec = to_dev(np.stack([off, ln], axis=1).reshape(-1).view(np.uint8), dev)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    L = _lib.lib()
    torch.cuda.synchronize()
    for _ in range(3):  # the scratch's epochs alternate: several calls
        assert L.cc_crc_ranges_dev(d.data_ptr(), rec.data_ptr(), n, out.data_ptr(), ctypes.c_void_p(h.value)) == 0
    st.synchronize()
    want = [oracle.crc32c(host[o:o + k].tobytes()) for o, k in zip(off.tolist(), ln.tolist())]
    assert u32(out).tolist() == want
    crcs = C.page_crc(d, 4096)
    torch.cuda.synchronize()
    d[4096 * 777 + 5] ^= 1  # corrupt page 777
    torch.cuda.synchronize()
    roff = rng.integers(0, host.size // 4096 - 40, n) * 4096
    rlen = rng.integers(1, 40, n) * 4096
    roff[17], rlen[17] = 4096 * 770, 4096 * 10
    bad, total = C.verify_reads(d, crcs, roff, rlen, 4096, stream=st)
    st.synchronize()
    hits = [i for i in range(n) if roff[i] <= 4096 * 777 < roff[i] + rlen[i]]
    assert int(total.item()) == len(hits)
    assert sorted(np.nonzero(bad.cpu().numpy())[0].tolist()) == hits


def test_scan_files_reader_pool_threads_and_counts(dev, oracle, tmp_path):
    """cc_scan_files' persistent reader pool (curve_amd/csrc/reader_pool.h):
    three threads at once (the per-device submission lock serialises them),
    each with a different io_threads -- 1, 64 (more readers than a batch has
    pieces: the pool grows, the run is capped) and 0 (the default) -- and calls
    over 1, 2 and 9 files (one batch short of a slot, two batches); every file
    CRC and slice CRC == the oracle's.  1 MiB chunks keep it small."""
    import threading
    from curve_amd import crc as C
    chunk, meta_b, sl = 1 << 20, 4096, 256 << 10
    rng = np.random.default_rng(81)
    raws, paths = [], []
    for i in range(40):
        raw = rng.integers(0, 256, meta_b + chunk, dtype=np.uint8).tobytes()
        p = tmp_path / f"chunk_{i}"
        p.write_bytes(raw)
        raws.append(raw)
        paths.append(str(p))
    jobs = [(1, paths[:1]), (64, paths[1:3]), (0, paths[3:12]), (64, paths[12:40]), (1, paths[:40]), (0, paths[5:6])]
    out = [None] * len(jobs)
    errs = []

    def work(k):
        try:
            io, ps = jobs[k]
            for _ in range(2):
                out[k] = C.scan_files(ps, chunk, meta_b, 4096, sl, io_threads=io)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=work, args=(k,)) for k in range(len(jobs))]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errs, errs
    index = {p: i for i, p in enumerate(paths)}
    for k, (_, ps) in enumerate(jobs):
        st, mc, sc, fc = out[k]
        assert (st == 0).all()
        for j, p in enumerate(ps):
            raw = raws[index[p]]
            want = oracle.scan_slices(raw[:meta_b], raw[meta_b:], sl)
            assert int(mc[j]) == want[0][2] and [int(x) for x in sc[j]] == [w[2] for w in want[1:]]
            assert int(fc[j]) == oracle.crc32c(raw)
