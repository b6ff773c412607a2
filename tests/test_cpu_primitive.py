"""libcurvecrc's CPU primitive (the drop-in for src/common/crc32.h) vs the oracle."""
import numpy as np
import pytest

import curve_amd as C
from curve_amd import crc as CR
from conftest import copyset_files, rfc_input


def test_rfc_and_extend(golden):
    for e in golden["rfc3720"]:
        assert C.CRC32(rfc_input(e)) == e["crc"]
    assert C.CRC32(b"hello world") == C.CRC32(C.CRC32(b"hello "), b"world")
    assert C.CRC32(b"") == 0


def test_reference_chains(golden):
    crc = 0
    for name in sorted(copyset_files(golden)):
        crc = C.CRC32(crc, copyset_files(golden)[name])
    assert str(crc) == "1355371765"
    import struct
    crc = 0
    for fmt, v in (("<I", 123), ("<I", 1345), ("<Q", 0), ("<Q", 0x6225929368674119)):
        crc = C.CRC32(crc, struct.pack(fmt, v))
    assert crc == 599727352


@pytest.mark.parametrize("n", [0, 1, 7, 8, 15, 16, 63, 503, 504, 768, 1008, 1536, 2040, 3072, 4080, 4095, 4096, 4104,
                               6144, 8191, 12287, 12288, 12289, 3 * 4096 * 5 + 13, 1 << 20])
def test_lengths_and_alignments(oracle, n):
    rng = np.random.default_rng(n)
    buf = rng.integers(0, 256, n + 16, dtype=np.uint8)
    for off in (0, 1, 3, 8):
        chunk = buf[off:off + n].tobytes()
        seed = int(rng.integers(0, 2**32))
        assert C.CRC32(seed, chunk) == oracle.crc32c(chunk, seed)


def test_combine_shift_zeros(oracle):
    rng = np.random.default_rng(3)
    for la, lb in [(0, 0), (1, 0), (0, 9), (100, 4096), (1 << 20, 4097)]:
        a = rng.integers(0, 256, la, dtype=np.uint8).tobytes()
        b = rng.integers(0, 256, lb, dtype=np.uint8).tobytes()
        assert C.combine(C.CRC32(a), C.CRC32(b), lb) == oracle.crc32c(a + b)
    for reg in (0, 1, 0xDEADBEEF, 0xFFFFFFFF):
        for n in (0, 1, 4, 256, 4096, 16 << 20, (16 << 20) + 4096, 10**12):
            assert C.shift(reg, n) == oracle.raw_shift(reg, n)
    assert C.zeros(4096) == 0x98F94189 == oracle.crc32c(bytes(4096))
    assert C.zeros(0) == 0


def test_delta_update_identity(oracle):
    """The identity cc_apply_log_delta_dev relies on, on the oracle: for equal
    lengths V(new) = V(old) ^ raw(old ^ new), raw = zero init, no xorout
    (= V(x) ^ V(0^n)); zero bytes outside the changed range add nothing, so the
    rows a write does not touch need not be read."""
    rng = np.random.default_rng(11)
    for n, lo, hi in [(4096, 0, 1), (4096, 17, 3000), (4096, 4095, 4096), (512, 3, 509), (8192, 0, 8192)]:
        old = rng.integers(0, 256, n, dtype=np.uint8)
        new = old.copy()
        new[lo:hi] = rng.integers(0, 256, hi - lo, dtype=np.uint8)
        delta = (old ^ new).tobytes()
        raw = oracle.crc32c(delta) ^ oracle.crc32c(bytes(n))
        assert oracle.crc32c(new.tobytes()) == oracle.crc32c(old.tobytes()) ^ raw
        # a stale stored CRC stays exactly as stale after the update
        stale = oracle.crc32c(old.tobytes()) ^ 0x10
        assert (stale ^ raw) ^ oracle.crc32c(new.tobytes()) == 0x10


def test_fold_host(oracle, golden):
    s = golden["seeded_pages"]
    pages = oracle.splitmix64_bytes(s["seed"], s["n_pages"] * s["page_bytes"])
    assert CR.fold_host(np.array(s["crcs"], dtype=np.uint32), 4096) == oracle.crc32c(pages.tobytes())
