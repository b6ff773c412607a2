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


@pytest.mark.parametrize("n", [0, 1, 7, 8, 15, 16, 63, 255, 256, 257, 319, 503, 504, 511, 512, 513, 767, 768, 1023, 1024, 1279, 1008, 1536, 2040, 3072, 4080, 4095, 4096, 4104,
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


@pytest.mark.parametrize("page_bytes", [256, 512, 4096, 8192])
def test_fold_host_every_count(oracle, page_bytes):
    """cc_fold_host (four interleaved carry-less Horner chains merged at the
    end) == CRC32 of the concatenation for every page count 1..40 (each
    remainder of the 4-way split, the short path below 8) and 1024 (a 4 MiB slice)."""
    data = oracle.splitmix64_bytes(0xF01D + page_bytes, 1024 * page_bytes)
    crcs = oracle.page_crcs(data, page_bytes)
    for n in list(range(1, 41)) + [1024]:
        want = oracle.crc32c(data[:n * page_bytes].tobytes())
        assert CR.fold_host(crcs[:n], page_bytes) == want, n


def test_shift_random_registers(oracle):
    """The carry-less multiply behind crc32c_shift / combine / zeros against the
    oracle's GF(2) matrix squaring, over random registers and byte counts."""
    rng = np.random.default_rng(0xC1)
    for _ in range(300):
        reg = int(rng.integers(0, 2**32))
        n = int(rng.integers(0, 2**40)) if rng.random() < 0.5 else int(rng.integers(0, 70000))
        assert C.shift(reg, n) == oracle.raw_shift(reg, n)


@pytest.mark.parametrize("seed", range(5))
def test_extend_iov_matches_concatenation(oracle, seed):
    """crc32c_extend_iov (the drop-in for braft::crc32(const butil::IOBuf&),
    raftlog/curve_segment.cpp:405) == CRC32(crc, concatenation of the fragments):
    empty, 1-byte, odd and block-sized fragments at any alignment."""
    rng = np.random.default_rng(seed)
    frags = []
    for _ in range(int(rng.integers(1, 40))):
        n = int(rng.choice([0, 1, 3, 7, 8, 100, 4096, 8192, int(rng.integers(0, 70000))]))
        off = int(rng.integers(0, 8))
        frags.append(rng.integers(0, 256, n + off, dtype=np.uint8)[off:])
    crc0 = int(rng.integers(0, 2**32)) if seed else 0
    whole = b"".join(f.tobytes() for f in frags)
    assert CR.CRC32_iov(frags, crc0) == oracle.crc32c(whole, crc0)
    assert CR.CRC32_iov([], crc0) == crc0


def test_slice_fold_batched(oracle):
    """cc_slice_fold: page CRCs -> slice CRCs == CRC32 of each slice."""
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, 64 * 4096, dtype=np.uint8)
    pc = oracle.page_crcs(data, 4096)
    for pps in (1, 2, 16, 64):
        got = CR.slice_fold(pc, pps, 4096)
        want = [oracle.crc32c(data[s * pps * 4096:(s + 1) * pps * 4096].tobytes()) for s in range(64 // pps)]
        assert got.tolist() == want
    with pytest.raises(CR.CurveCrcError):
        CR.slice_fold(pc[:10], 4, 4096)


# around each path's edges: fold from 256 B; the fold + crc32q split from 8 steps of 752 B, at most 64 a split
_PATH_LENGTHS = [0, 1, 200, 255, 256, 257, 300, 511, 512, 513, 767, 768, 769, 1024, 1279, 1280, 1536, 3007, 3008, 3009,
                 3263, 3264, 3760, 4096, 6015, 6016, 6017, 6271, 6272, 9999, 48127, 48128, 48129, 48384,
                 65535, 65536, 65537, 96256, 96256 + 6016, (1 << 20) + 4101]
_BOTH_PATHS = """
import sys, numpy as np, curve_amd as C
rng = np.random.default_rng(5)
out = []
for n in %s:
    buf = rng.integers(0, 256, n + 64, dtype=np.uint8)
    for off in (0, 1, 5, 13, 63):
        out.append(C.CRC32(int(rng.integers(0, 2**32)), buf[off:off + n].tobytes()))
print(" ".join(map(str, out)))
""" % _PATH_LENGTHS


def test_fold_and_crc32q_paths_agree(oracle):
    """crc32c_cpu.cpp's VPCLMULQDQ fold (used when the CPU has it), the fold +
    crc32q split (AMD hosts; CURVE_CRC_FOLD_SPLIT=1 forces it) and the 3-way
    crc32q loop (CURVE_CRC_NO_FOLD=1) give the same values, and all equal the
    oracle's on the same seeded inputs."""
    import os
    import subprocess
    import sys
    runs = []
    for no_fold, split in (("0", "0"), ("0", "1"), ("1", "0")):
        env = dict(os.environ, CURVE_CRC_NO_FOLD=no_fold, CURVE_CRC_FOLD_SPLIT=split)
        r = subprocess.run([sys.executable, "-c", _BOTH_PATHS], env=env, capture_output=True, text=True, timeout=120,
                           cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        assert r.returncode == 0, r.stderr
        runs.append(r.stdout.split())
    assert runs[0] == runs[1] == runs[2]
    rng = np.random.default_rng(5)
    want = []
    for n in _PATH_LENGTHS:
        buf = rng.integers(0, 256, n + 64, dtype=np.uint8)
        for off in (0, 1, 5, 13, 63):
            seed = int(rng.integers(0, 2**32))
            want.append(str(oracle.crc32c(buf[off:off + n].tobytes(), seed)))
    assert runs[0] == want
