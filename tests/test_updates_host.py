"""Host logic of the partial-write path: ordered batch -> non-overlapping sub-batches."""
import numpy as np
import pytest

from curve_amd.crc import split_nonoverlapping


def apply_in_order(buf, dst, src_data, lens, order):
    out = buf.copy()
    for i in order:
        out[dst[i]:dst[i] + lens[i]] = src_data[i]
    return out


@pytest.mark.parametrize("seed", range(6))
def test_split_equals_in_order_application(seed):
    rng = np.random.default_rng(seed)
    size = 20000
    n = 400
    dst = rng.integers(0, size - 600, n)
    lens = rng.integers(1, 600, n)
    if seed % 2:  # force many overlaps
        dst = rng.integers(0, 2000, n)
    src = [rng.integers(0, 256, l, dtype=np.uint8) for l in lens]
    base = np.zeros(size, dtype=np.uint8)
    want = apply_in_order(base, dst, src, lens, range(n))
    got = base.copy()
    batches = split_nonoverlapping(dst, lens)
    assert sorted(np.concatenate(batches).tolist()) == list(range(n))
    for b in batches:
        iv = sorted((int(dst[i]), int(dst[i] + lens[i])) for i in b)
        assert all(iv[k][1] <= iv[k + 1][0] for k in range(len(iv) - 1))  # no overlaps inside a batch
        for i in reversed(b):  # any order inside a batch gives the same bytes
            got[dst[i]:dst[i] + lens[i]] = src[i]
    assert (got == want).all()


def test_random_pool_writes_need_few_batches():
    rng = np.random.default_rng(5)
    dst = rng.integers(0, (16 << 30) - 4096, 65536)
    lens = rng.integers(512, 4097, 65536)
    b = split_nonoverlapping(dst, lens)
    assert 2 <= len(b) <= 4 and sum(x.size for x in b) == 65536


def test_no_overlap_is_one_batch():
    dst = np.arange(0, 10000, 100)
    assert len(split_nonoverlapping(dst, np.full(dst.size, 100))) == 1
    assert len(split_nonoverlapping(dst, np.full(dst.size, 101))) > 1


@pytest.mark.parametrize("seed", range(6))
def test_cpp_planner_matches_levels(seed):
    """cc_plan_updates (C++) == the Python level assignment, and applying its
    levels in order equals applying the log in order."""
    from curve_amd.crc import _update_dtype, plan_updates
    rng = np.random.default_rng(100 + seed)
    n, size = 3000, 60000 if seed % 2 else 10 ** 9
    dst = rng.integers(0, size, n)
    lens = rng.integers(1, 700, n)
    rec = np.zeros(n, dtype=_update_dtype())
    rec["dst"], rec["src"], rec["len"] = dst, np.arange(n), lens
    out, ends, nb = plan_updates(rec)
    py = split_nonoverlapping(dst, lens)
    assert nb == len(py)
    starts = np.concatenate([[0], ends[:-1]]).astype(int)
    for b, (s0, e0) in enumerate(zip(starts, ends.astype(int))):
        assert sorted(out["src"][s0:e0].tolist()) == py[b].tolist()  # same members, src = write index
        assert (np.diff(out["src"][s0:e0].astype(np.int64)) > 0).all()  # write order kept in a level
    if size < 10 ** 6:
        src = [rng.integers(0, 256, l, dtype=np.uint8) for l in lens]
        want = apply_in_order(np.zeros(size + 800, np.uint8), dst, src, lens, range(n))
        got = np.zeros(size + 800, np.uint8)
        for k in range(n):  # levels in order
            i = int(out["src"][k])
            got[dst[i]:dst[i] + lens[i]] = src[i]
        assert (got == want).all()


def test_cpp_planner_speed():
    import time
    from curve_amd.crc import _update_dtype, plan_updates
    rng = np.random.default_rng(9)
    rec = np.zeros(65536, dtype=_update_dtype())
    rec["dst"] = rng.integers(0, (16 << 30) - 4096, 65536)
    rec["len"] = rng.integers(512, 4097, 65536)
    plan_updates(rec)
    t = time.perf_counter()
    _, _, nb = plan_updates(rec)
    assert 2 <= nb <= 4 and time.perf_counter() - t < 0.05


def _levels_bruteforce(dst, lens):
    """Definition of the level assignment, O(n^2): level(j) = 1 + max level of
    the earlier writes j overlaps, 0 if none."""
    lv = []
    for j in range(len(dst)):
        m = -1
        for i in range(j):
            if dst[i] < dst[j] + lens[j] and dst[j] < dst[i] + lens[i]:
                m = max(m, lv[i])
        lv.append(m + 1)
    return lv


@pytest.mark.parametrize("seed", range(4))
def test_levels_match_definition_on_hot_clusters(seed):
    """The segment-tree level assignment (Python and C++) == the O(n^2)
    definition on logs that pile onto a few hundred bytes."""
    from curve_amd.crc import _update_dtype, plan_updates
    rng = np.random.default_rng(700 + seed)
    n = 300
    dst = rng.integers(0, 400, n)
    lens = rng.integers(1, 120, n)
    want = _levels_bruteforce(dst.tolist(), lens.tolist())
    py = split_nonoverlapping(dst, lens)
    got = np.zeros(n, dtype=int)
    for b, idx in enumerate(py):
        got[idx] = b
    assert got.tolist() == want
    rec = np.zeros(n, dtype=_update_dtype())
    rec["dst"], rec["src"], rec["len"] = dst, np.arange(n), lens
    out, ends, nb = plan_updates(rec)
    starts = np.concatenate([[0], ends[:-1]]).astype(int)
    cpp = np.zeros(n, dtype=int)
    for b, (s0, e0) in enumerate(zip(starts, ends.astype(int))):
        cpp[out["src"][s0:e0].astype(int)] = b
    assert cpp.tolist() == want


def test_cpp_planner_hot_region_is_not_quadratic():
    """20,000 writes hammering one 4 KiB block used to cost a pair
    scan of 2*10^8 checks; the segment tree makes it O(n log n)."""
    import time
    from curve_amd.crc import _update_dtype, plan_updates
    rng = np.random.default_rng(10)
    n = 20000
    rec = np.zeros(n, dtype=_update_dtype())
    rec["dst"] = rng.integers(0, 4096, n)
    rec["len"] = rng.integers(1, 4096, n)
    t = time.perf_counter()
    _, ends, nb = plan_updates(rec, max_batches=n)
    assert time.perf_counter() - t < 0.5
    assert nb > 100 and int(ends[-1]) == n
