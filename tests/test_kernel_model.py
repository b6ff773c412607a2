"""Host-logic tests of the page kernel: replay its arithmetic on the CPU with
the library's own LDS image and check it bit-exact against the oracle, and
check the LDS layout is bank-conflict-free for every lookup the kernel makes."""
import numpy as np
import pytest

import kernel_model as km


@pytest.fixture(scope="module")
def img():
    return km.lds_image()


@pytest.mark.parametrize("page_bytes", [256, 512, 1024, 4096, 8192, 3 * 256, 16384])
def test_model_matches_oracle(oracle, img, page_bytes):
    rng = np.random.default_rng(page_bytes)
    pages = rng.integers(0, 256, page_bytes * 19, dtype=np.uint8)
    assert (km.page_crcs_model(pages, page_bytes, img) == oracle.page_crcs(pages, page_bytes)).all()


def test_model_golden_pages(oracle, golden, img):
    s = golden["seeded_pages"]
    pages = oracle.splitmix64_bytes(s["seed"], s["n_pages"] * s["page_bytes"])
    assert [int(c) for c in km.page_crcs_model(pages, 4096, img)] == s["crcs"]


def test_zero_and_ones_pages(img):
    z = np.zeros(4096 * 3, dtype=np.uint8)
    assert (km.page_crcs_model(z, 4096, img) == 0x98F94189).all()


def test_lookups_bank_conflict_free():
    lane = np.arange(64, dtype=np.uint32)
    c0 = (lane << 2) & np.uint32(0x7C)
    c1 = c0 | np.uint32(0x10000)
    rng = np.random.default_rng(0)
    for _ in range(50):
        s = rng.integers(0, 2**32, 64, dtype=np.uint64).astype(np.uint32)
        for c, sel, off in ((c0, 0x0C060004, 0), (c0, 0x0C060104, 128), (c1, 0x0C060204, 0), (c1, 0x0C060304, 128)):
            assert km.bank_conflicts(km.v_perm_b32(c, s, sel) + off) == 0
        cf = np.uint32(km.K_FIN_BASE) + (lane << 2)
        for n in range(8):
            v = (s >> np.uint32(4 * n)) & np.uint32(15)
            assert km.bank_conflicts(((v << np.uint32(8)) | cf) + 4096 * n) == 0


@pytest.mark.parametrize("n_pages", [1, 2, 63, 64, 65, 4095, 4096, 4097, 8192, 8197, 20000, 262143, 262144,
                                     262144 + 77, 4194304 + 13])
@pytest.mark.parametrize("cus", [256, 255, 80])
def test_tile_walk_covers_every_page_once(n_pages, cus):
    blocks, ts = km.geometry(n_pages, cus)
    assert 0 <= ts <= 6 and 1 <= blocks <= cus
    if n_pages > 300000:  # the full walk is slow in Python: check the geometry only
        assert (n_pages >> ts) >= cus * 16 or ts == 0
        return
    hashed, flushes = km.tile_walk(n_pages, blocks, ts)
    assert sorted(hashed) == list(range(n_pages))
    covered = []
    for first, cnt in flushes:
        assert 1 <= cnt <= (1 << ts) and first % (1 << ts) == 0
        covered += range(first, first + cnt)
    assert sorted(covered) == list(range(n_pages))


def test_range_model_matches_oracle(oracle, img):
    rng = np.random.default_rng(42)
    buf = rng.integers(0, 256, 3000, dtype=np.uint8)
    cases = [(0, 0), (0, 1), (1, 1), (3, 2), (5, 3), (0, 4), (2, 7), (0, 256), (1, 256), (3, 255),
             (0, 257), (7, 600), (1000, 1999), (4, 28), (13, 1)]
    cases += [(int(rng.integers(0, 1500)), int(rng.integers(0, 1400))) for _ in range(25)]
    for off, ln in cases:
        assert km.range_crc_model(buf, off, ln, img) == oracle.crc32c(buf[off:off + ln].tobytes()), (off, ln)


def test_div_x_inverts_mul_x():
    rng = np.random.default_rng(1)
    for b in rng.integers(0, 2**32, 200, dtype=np.uint64).tolist():
        assert km.div_x(km.mulmod(0x40000000, b)) == b  # (b * x) / x
    assert km.mulmod(km.xinv_bytes(3), km.mulmod(0x80000000 >> 24, 0xDEADBEEF)) == 0xDEADBEEF  # x^-24 * x^24


@pytest.mark.parametrize("shape", ["wal", "giants", "tiny", "few"])
@pytest.mark.parametrize("waves", [2048, 256, 7])
def test_range_flat_schedule_and_split_meeting(shape, waves):
    """range_flat_kernel's schedule (static block shares + dynamic chunks) cuts
    every range into segments covering each of its blocks once; the split
    ranges' accumulator pairs (XOR, then block count) end with exactly one
    store per non-empty range, of the XOR of its segments, and leave every pair
    zero for the next call -- in any arrival order."""
    rng = np.random.default_rng(len(shape) * 1000 + waves)
    n = {"wal": 20000, "giants": 300, "tiny": 30000, "few": 3}[shape]
    if shape == "wal":
        nbs = (rng.integers(1, 131073, n) + 28 + 4095) // 4096
    elif shape == "giants":
        nbs = rng.integers(0, 2, n)
        nbs[::30] = rng.integers(256, 6000, nbs[::30].size)
    elif shape == "tiny":
        nbs = rng.integers(0, 3, n)
    else:
        nbs = np.array([4097, 0, 1])
    for rounds in (1, 2):  # the shipped schedule (one static piece a wave) and round 3's
        segs = km.range_flat_segments(nbs, waves, rounds=rounds)
        cover = {}
        for r, kb, cnt in segs:
            assert cnt >= 1 and kb + cnt <= nbs[r]
            cover.setdefault(r, []).append((kb, cnt))
        for r in range(n):
            parts = sorted(cover.get(r, []))
            assert sum(c for _, c in parts) == nbs[r]
            assert all(a + c == b for (a, c), (b, _) in zip(parts, parts[1:]))  # contiguous, disjoint
        contrib = rng.integers(0, 2**32, len(segs)).tolist()
        want = {}
        for (r, _, _), v in zip(segs, contrib):
            want[r] = want.get(r, 0) ^ v
        for _ in range(3):
            out, left, stores = km.range_accumulate(segs, nbs, contrib, rng)
            assert out == want and not left
        assert all(c == 1 for c in stores.values()) and set(stores) == {r for r in range(n) if nbs[r]}


@pytest.mark.parametrize("shape", ["reads", "tiny", "empties", "few"])
@pytest.mark.parametrize("waves", [2048, 256, 5])
def test_verify_flat_schedule_covers_every_page_once(shape, waves):
    """read_verify_kernel's self-counted schedule (tile counts, static shares at
    page granularity, dynamic chunks, 64-read groups walked from the tile start)
    visits every page of every read exactly once, with the right owner read."""
    rng = np.random.default_rng(len(shape) * 77 + waves)
    if shape == "reads":
        counts = rng.integers(1, 33, 20000)  # 4-128 KiB reads at 4 KiB pages
    elif shape == "tiny":
        counts = rng.integers(1, 3, 30000)
    elif shape == "empties":
        counts = rng.integers(0, 5, 9000)
        counts[::7] = 0  # empty reads and reads past the pool: no pages
        counts[:200] = 0
    else:
        counts = np.array([0, 4097, 1, 0, 33])
    got = km.verify_flat_pages(counts, waves)
    want = [(r, p) for r in range(len(counts)) for p in range(int(counts[r]))]
    assert len(got) == len(want) and sorted(got) == want


@pytest.mark.parametrize("Hall,grid,wv", [(101161, 256, 16), (5000, 40, 16), (37, 4, 16), (900, 17, 12)])
def test_write_log_tail_stealing_rehashes_every_page_once(Hall, grid, wv):
    """The write-log page kernel's tail stealing (log_pages_body): whatever the
    wave speeds (three XCDs ~6 % slow, young waves slower, a late workgroup that
    is not resident at first), every touched page is rehashed by exactly one
    wave, every table slot is cleared once, after the wave that won it read it,
    and with uneven speeds the last wave ends earlier than without stealing."""
    rng = np.random.default_rng(Hall)
    W = grid * wv
    speed = [1.0 + (0.06 if (w // wv) % 8 in (3, 4, 5) else 0.0) + 0.02 * ((w % wv) // 4) + rng.uniform(0, 0.02)
             for w in range(W)]
    start = [0.0] * W
    start[(grid // 2) * wv:(grid // 2 + 1) * wv] = [40.0] * wv
    owner, cleared, ok, end = km.log_steal_schedule(Hall, grid, wv, speed, start=start)
    assert min(owner) >= 0 and all(cleared) and ok
    _, _, _, end0 = km.log_steal_schedule(Hall, grid, wv, speed, max_steals=0, start=start)
    assert max(end) <= max(end0)


@pytest.mark.parametrize("n_segs", [1, 3, 128, 256])
def test_write_log_head_segments_map_every_head_once(n_segs):
    """The write-log page kernel finds head h in the insert blocks' segments
    (per-block head lists, no global counter): every batch of 64 heads maps each
    head to the right (segment, record), across empty segments and segment ends."""
    rng = np.random.default_rng(n_segs)
    for trial in range(30):
        counts = rng.integers(0, 900, n_segs)
        if trial % 3 == 0:
            counts[rng.random(n_segs) < 0.5] = 0  # many empty segments
        if trial % 5 == 0:
            counts[:] = rng.integers(0, 3, n_segs)  # tiny segments: a batch spans dozens
        total = int(counts.sum())
        if total == 0:
            continue
        want = [(s, k) for s in range(n_segs) for k in range(int(counts[s]))]
        for _ in range(20):
            H = int(rng.integers(1, total + 1))
            base = int(rng.integers(0, H))
            got = km.log_head_segments(counts, base, H)
            assert got == want[base:min(base + 64, H)]
