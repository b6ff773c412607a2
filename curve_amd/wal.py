"""Raft WAL segment checksums on the device.

Curve's WAL (src/chunkserver/raftlog/curve_segment.cpp) stores per entry a
28-byte header packed big-endian by butil::RawPacker (:421-428):
    term u64 | meta_field u32 = type<<24 | checksum_type<<16 | data_len u32
    | data_real_len u32 | data_checksum u32 | header_checksum u32
followed by the data zero-padded so that header + data is a multiple of
walAlignSize (4096, :54, :407-414).  data_checksum = braft::crc32(data[:real_len])
and header_checksum = braft::crc32(header[:24]); with CHECKSUM_CRC32 (chosen when
butil::crc32c::IsFastCrc32Supported, curve_segment_log_storage.cpp:76-80)
braft::crc32 is butil::crc32c::Value.  The segment starts with a meta page whose
first 8 bytes hold the used byte count (_load_meta, :231-242).

Replay (CurveSegment::load, :148-190) walks the headers sequentially -- that
walk stays on the host (28 bytes per entry, 24-byte header CRCs on the CPU
primitive) -- and the data checksums of all entries, the bulk bytes, are
verified in ONE device call (cc_crc_ranges_dev).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import List, Sequence, Tuple

from . import crc as C

ENTRY_HEADER_SIZE = 28          # raftlog/define.h:59
WAL_ALIGN = 4096                # FLAGS_walAlignSize, curve_segment.cpp:54
CHECKSUM_MURMURHASH32 = 0       # braft::ChecksumType
CHECKSUM_CRC32 = 1
ENTRY_TYPE_NO_OP = 1            # braft::EntryType
ENTRY_TYPE_DATA = 2
ENTRY_TYPE_CONFIGURATION = 3


@dataclass
class EntryHeader:
    offset: int
    term: int
    type: int
    checksum_type: int
    data_len: int
    data_real_len: int
    data_checksum: int
    header_ok: bool


def pack_entry(term: int, etype: int, data: bytes, align: int = WAL_ALIGN) -> bytes:
    """CurveSegment::append layout (curve_segment.cpp:405-440)."""
    real = len(data)
    to_write = ENTRY_HEADER_SIZE + real
    pad = 0 if to_write % align == 0 else (to_write // align + 1) * align - to_write
    meta_field = (etype << 24) | (CHECKSUM_CRC32 << 16)
    hdr = struct.pack(">qIIII", term, meta_field, real + pad, real, C.CRC32(data))
    hdr += struct.pack(">I", C.CRC32(hdr))
    return hdr + data + bytes(pad)


def build_segment(entries: Sequence[Tuple[int, int, bytes]], meta_page_size: int = 4096) -> bytes:
    """A whole segment file: meta page (used bytes) + packed entries."""
    body = b"".join(pack_entry(t, ty, d) for t, ty, d in entries)
    meta = bytearray(meta_page_size)
    meta[:8] = struct.pack("<q", meta_page_size + len(body))
    return bytes(meta) + body


def append_entries(seg: bytes, entries: Sequence[Tuple[int, int, bytes]], meta_page_size: int = 4096) -> bytes:
    """CurveSegment::append (curve_segment.cpp:405-440) of more entries at the
    meta page's used-bytes offset, which then moves past them (_update_meta_page)."""
    used = struct.unpack_from("<q", seg, 0)[0]
    body = b"".join(pack_entry(t, ty, d) for t, ty, d in entries)
    out = bytearray(seg[:used]) + body + bytearray(seg[used + len(body):])
    out[:8] = struct.pack("<q", used + len(body))
    return bytes(out)


def truncate_segment(seg: bytes, headers: Sequence[EntryHeader], keep: int) -> bytes:
    """CurveSegment::truncate (curve_segment.cpp:663-717): keep the first `keep`
    entries; the meta page's used bytes drop to the first dropped entry's offset.
    The dropped bytes stay in the file (the reference only lseeks) and are
    ignored by the next load and overwritten by the next append."""
    if keep >= len(headers):
        return seg
    out = bytearray(seg)
    out[:8] = struct.pack("<q", headers[keep].offset)
    return bytes(out)


def parse_segment(seg, meta_page_size: int = 4096) -> List[EntryHeader]:
    """Header walk of CurveSegment::load (curve_segment.cpp:148-190): stops at a
    truncated tail or the first corrupted header (reported with header_ok=False)."""
    mv = memoryview(seg)
    # bytes in use per the meta page, bounded by what was actually read: an entry
    # whose data is cut cannot have its data checksum verified (the reference
    # fails that entry's later _load_entry with a short pread, :350-355)
    used = min(struct.unpack_from("<q", mv, 0)[0], len(mv))
    off, out = meta_page_size, []
    while off < used:
        if off + ENTRY_HEADER_SIZE > len(mv):
            break
        term, meta_field, data_len, real, dck, hck = struct.unpack_from(">qIIIII", mv, off)
        ok = C.CRC32(bytes(mv[off:off + ENTRY_HEADER_SIZE - 4])) == hck
        h = EntryHeader(off, term, meta_field >> 24, (meta_field >> 16) & 0xFF, data_len, real, dck, ok)
        out.append(h)
        if not ok:
            break
        if off + ENTRY_HEADER_SIZE + data_len > used:
            out.pop()  # last entry not completely written: truncated on load
            break
        off += ENTRY_HEADER_SIZE + data_len
    return out


@dataclass
class SegmentCheck:
    """Outcome of verify_segment_dev; every index is a position in `headers`."""
    crcs: object                 # int32 device tensor: the data CRC of every CRC32-checked entry, in order
    checked: List[int]           # entries whose data checksum was verified on the device
    bad: List[int]               # ... and did not match (CurveSegment::_load_entry would fail them)
    unverified: List[int]        # entries not verified here: a non-CRC32 checksum type
                                 # (CHECKSUM_MURMURHASH32, braft's other type) or an untrusted header
    corrupt_header: List[int]    # header CRC mismatch: data_real_len is not trusted, data not hashed


def verify_segment_dev(dev_seg, headers: Sequence[EntryHeader], stream=None) -> SegmentCheck:
    """Data checksums of every parsed entry with a trusted header and a CRC32
    checksum, on the device in ONE call (cc_crc_ranges_dev).  Entries whose
    header failed its own CRC are never hashed (their length is not trusted);
    entries of another checksum type are reported as unverified, not skipped
    silently.  Indices refer to `headers`."""
    import numpy as np
    corrupt = [k for k, h in enumerate(headers) if not h.header_ok]
    checked = [k for k, h in enumerate(headers) if h.header_ok and h.checksum_type == CHECKSUM_CRC32]
    unverified = [k for k, h in enumerate(headers) if h.header_ok and h.checksum_type != CHECKSUM_CRC32]
    offs = [headers[k].offset + ENTRY_HEADER_SIZE for k in checked]
    lens = [headers[k].data_real_len for k in checked]
    got = C.crc_ranges(dev_seg, offs, lens, stream=stream)
    vals = np.asarray(C.as_u32(got), dtype=np.uint64)
    want = np.asarray([headers[k].data_checksum for k in checked], dtype=np.uint64)
    bad = [checked[i] for i in np.flatnonzero(vals != want).tolist()]
    return SegmentCheck(got, checked, bad, unverified, corrupt)
