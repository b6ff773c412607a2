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
