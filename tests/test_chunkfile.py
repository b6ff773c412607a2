"""Chunk-file format, CompareMap semantics, copyset hash over a real directory (CPU parts)."""
import os
import struct

import numpy as np
import pytest

from curve_amd import chunkfile as CF
from curve_amd.scan import ScanMap, compare_maps, scan_schedule


def test_metapage_roundtrip_and_crc_position(oracle):
    m = CF.ChunkFileMetaPage(version=2, sn=7, correctedSn=3)
    page = m.encode()
    hdr = struct.pack("<BQQQ", 2, 7, 3, 0)
    assert page[:25] == hdr
    assert struct.unpack("<I", page[25:29])[0] == oracle.crc32c(hdr)  # CRC at byte 25 (non-clone)
    rc, d = CF.ChunkFileMetaPage.decode(page)
    assert rc == CF.CSErrorCode.Success and (d.version, d.sn, d.correctedSn) == (2, 7, 3)


def test_metapage_clone_and_errors(oracle):
    m = CF.ChunkFileMetaPage(version=1, sn=2, correctedSn=0, location=b"s3@bucket/obj", bitmap_bits=4096,
                             bitmap=bytes(range(256)) * 2)
    page = bytearray(m.encode())
    rc, d = CF.ChunkFileMetaPage.decode(bytes(page))
    assert rc == CF.CSErrorCode.Success and d.location == b"s3@bucket/obj" and d.bitmap_bits == 4096
    page[5] ^= 1  # corrupt sn -> CrcCheckError (chunkserver_chunkfile.cpp:111-118)
    assert CF.ChunkFileMetaPage.decode(bytes(page))[0] == CF.CSErrorCode.CrcCheckError
    bad = CF.ChunkFileMetaPage(version=3).encode()
    assert CF.ChunkFileMetaPage.decode(bad)[0] == CF.CSErrorCode.IncompatibleError


def test_compare_maps_semantics():
    # scan_manager_test.cpp CompareMapSuccessTest / CompareMapFailTest / MismatchedCRCTest shapes
    a = ScanMap(1, 1, 1, 5, 100, 0, 4 << 20)
    assert compare_maps(a, [a, a]) == (True, None)
    b = ScanMap(1, 1, 1, 5, 200, 0, 4 << 20)
    assert compare_maps(a, [a, b]) == (False, a)
    c = ScanMap(1, 1, 1, 6, 100, 0, 4 << 20)  # index differs -> MessageDifferencer says unequal
    assert compare_maps(a, [a, c]) == (False, a)
    assert compare_maps(a, [a]) == (False, None)
    assert compare_maps(None, [a, a]) == (False, None)


def test_scan_schedule_geometry():
    ops = scan_schedule()
    assert len(ops) == 5 and ops[0] == (True, 0, 4096)  # 1 metapage + 4 slices (scan_manager_test.cpp:107-142)
    assert [o[1] for o in ops[1:]] == [0, 4 << 20, 8 << 20, 12 << 20]
    with pytest.raises(ValueError):
        scan_schedule(16 << 20, 3 << 20)


def test_copyset_dir_golden_files(tmp_path, golden):
    """The reference's own 5-file fixture as real files (no chunk files -> CPU chain)."""
    from conftest import copyset_files
    for name, data in copyset_files(golden).items():
        (tmp_path / name).write_bytes(data)
    assert CF.copyset_hash_dir(str(tmp_path)) == "1355371765"


def test_empty_copyset_dir(tmp_path):
    assert CF.copyset_hash_dir(str(tmp_path)) == "0"
