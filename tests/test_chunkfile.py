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
    # lengths that overrun the page: CrcCheckError, never an exception / overread
    good = bytearray(m.encode())
    huge = bytearray(good)
    huge[17:25] = struct.pack("<Q", 1 << 40)
    assert CF.ChunkFileMetaPage.decode(bytes(huge))[0] == CF.CSErrorCode.CrcCheckError
    bits = bytearray(good)
    bits[25 + len(m.location):29 + len(m.location)] = struct.pack("<I", 0xFFFFFFFF)
    assert CF.ChunkFileMetaPage.decode(bytes(bits))[0] == CF.CSErrorCode.CrcCheckError
    assert CF.ChunkFileMetaPage.decode(bytes(good[:20]))[0] == CF.CSErrorCode.CrcCheckError


def test_metapage_crc_is_the_residue_constant(oracle, golden):
    """Every encoded non-clone 4 KiB metapage hashes to the same value (CRC-32C
    residue property), so the metapage ScanMap.crc is 317729701 on every chunk;
    a clone metapage's CRC depends only on its header length."""
    g = golden["metapage_residue"]
    for sn, csn, ver in ((1, 0, 2), (123, 45, 1), (2**64 - 1, 2**63, 2)):
        page = CF.ChunkFileMetaPage(version=ver, sn=sn, correctedSn=csn).encode()
        assert oracle.crc32c(page) == g["crc"]
        hdr = page[:25]
        assert oracle.crc32c(page[:29]) == g["residue"] == oracle.crc32c(hdr + struct.pack("<I", oracle.crc32c(hdr)))
    a = CF.ChunkFileMetaPage(sn=1, location=b"x" * 10, bitmap_bits=16, bitmap=b"\x01\x02").encode()
    b = CF.ChunkFileMetaPage(sn=9, location=b"y" * 10, bitmap_bits=16, bitmap=b"\xff\x00").encode()
    assert oracle.crc32c(a) == oracle.crc32c(b) != g["crc"]


def test_chunk_service_hash_vector(oracle, golden):
    """chunk_service_test.cpp:563-578: hash of the 'a'-filled first block is
    650595490 = CRC32 of the DATA block.  CSChunkFile::GetHash as written
    preads the raw file, whose [0, 4096) is the metapage (-> 317729701); the
    engine follows the code (DevicePool.chunk_hash takes raw file offsets), so
    the reference test's value is reproduced at raw offset 4096."""
    g = golden["chunk_service_hash"]
    assert str(oracle.crc32c(b"a" * 4096)) == g["hash"]
    raw = CF.ChunkFileMetaPage(sn=1).encode() + b"a" * 4096 + bytes(8192)
    assert oracle.chunk_hash(raw, 4096, 4096) == g["hash"]
    assert oracle.chunk_hash(raw, 0, 4096) == str(golden["metapage_residue"]["crc"])


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


def test_get_hash_error_contract(tmp_path, golden):
    """copyset_node_test.cpp:864-997: open/fstat/read failure -> -1; empty -> (0, "0")."""
    from conftest import copyset_files
    assert CF.get_hash(str(tmp_path)) == (0, "0")
    for name, data in copyset_files(golden).items():
        (tmp_path / name).write_bytes(data)
    assert CF.get_hash(str(tmp_path)) == (0, "1355371765")
    os.symlink(str(tmp_path / "missing-target"), str(tmp_path / "test-6.txt"))  # listed, cannot be opened
    assert CF.get_hash(str(tmp_path)) == (-1, "")
    assert CF.get_hash(str(tmp_path / "no-such-dir")) == (-1, "")


def test_empty_copyset_dir(tmp_path):
    assert CF.copyset_hash_dir(str(tmp_path)) == "0"
