"""WAL segment layout + header walk (CPU) -- mirror of CurveSegment append/load."""
import struct

import numpy as np

from curve_amd import wal


def make_entries(rng, n=40):
    ents = []
    for i in range(n):
        ln = int(rng.choice([0, 1, 27, 4068, 4069, 8000, 65536, int(rng.integers(1, 70000))]))
        ents.append((7 + i // 10, wal.ENTRY_TYPE_DATA if ln else wal.ENTRY_TYPE_NO_OP,
                     rng.integers(0, 256, ln, dtype=np.uint8).tobytes()))
    return ents


def test_layout_and_walk(oracle):
    rng = np.random.default_rng(3)
    ents = make_entries(rng)
    seg = wal.build_segment(ents)
    hs = wal.parse_segment(seg)
    assert len(hs) == len(ents)
    for h, (term, ty, data) in zip(hs, ents):
        assert h.header_ok and h.term == term and h.type == ty and h.checksum_type == wal.CHECKSUM_CRC32
        assert (wal.ENTRY_HEADER_SIZE + h.data_len) % wal.WAL_ALIGN == 0  # 4 KiB aligned entries
        assert h.data_real_len == len(data)
        assert h.data_checksum == oracle.crc32c(data)  # braft::crc32 == butil crc32c Value
        raw = seg[h.offset:h.offset + wal.ENTRY_HEADER_SIZE]
        assert struct.unpack(">I", raw[24:28])[0] == oracle.crc32c(raw[:24])


def test_truncated_tail_and_corrupt_header():
    rng = np.random.default_rng(4)
    ents = make_entries(rng, 6)
    seg = bytearray(wal.build_segment(ents))
    full = wal.parse_segment(bytes(seg))
    # truncated: used-bytes claims the last entry but the file is cut
    cut = bytes(seg[:full[-1].offset + 100])
    assert len(wal.parse_segment(cut)) == len(ents) - 1
    # corrupted header: walk stops there, flagged
    seg[full[2].offset + 3] ^= 1
    hs = wal.parse_segment(bytes(seg))
    assert len(hs) == 3 and not hs[2].header_ok and all(h.header_ok for h in hs[:2])


def test_truncate_then_append(oracle):
    """test_curve_segment.cpp open_segment: append 10 "hello, world: %d"
    entries, truncate(5), append "HELLO, WORLD: %d" for 5..9; the walk sees the
    first five old entries then the five new ones, every checksum intact."""
    old = [(1, wal.ENTRY_TYPE_DATA, (b"hello, world: %d" % i) * 300) for i in range(10)]
    seg = wal.build_segment(old) + bytes(1 << 16)  # preallocated file (prepare_segment)
    hs = wal.parse_segment(seg)
    assert len(hs) == 10
    seg = wal.truncate_segment(seg, hs, 5)
    assert len(wal.parse_segment(seg)) == 5
    new = [(1, wal.ENTRY_TYPE_DATA, (b"HELLO, WORLD: %d" % i) * 7) for i in range(5, 10)]
    seg = wal.append_entries(seg, new)
    hs = wal.parse_segment(seg)
    want = [e[2] for e in old[:5] + new]
    assert len(hs) == 10 and all(h.header_ok for h in hs)
    for h, data in zip(hs, want):
        assert h.data_real_len == len(data)
        assert seg[h.offset + wal.ENTRY_HEADER_SIZE:h.offset + wal.ENTRY_HEADER_SIZE + len(data)] == data
        assert h.data_checksum == oracle.crc32c(data)
