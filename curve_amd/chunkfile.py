"""Chunk-file format and the datastore read path around the engine.

Mirrors:
  ChunkFileMetaPage::encode/decode   src/chunkserver/datastore/chunkserver_chunkfile.cpp:64-130
      version u8 | sn u64 | correctedSn u64 | loc_size size_t(u64)
      [| location bytes | bits u32 | bitmap (bits+7)/8 bytes]   (clone chunks only)
      | CRC32 of all of the above (little-endian, memcpy)        -> at byte 25 for non-clone chunks
      decode: CRC mismatch -> CrcCheckError; version not in {1, 2} -> IncompatibleError
  chunk file = metaPageSize (4 KiB) || chunkSize (16 MiB)       conf/chunkserver.conf:13,16
  chunk file names chunk_<id>, chunk_<id>_snap_<sn>            datastore/filename_operator.h:55-62
  CSChunkFile::GetHash (raw FILE range)                        chunkserver_chunkfile.cpp:785-811
  CopysetNode::GetHash over a data directory                   copyset_node.cpp:925-975

Metapage headers are a few dozen bytes: their CRC stays on the CPU primitive.
Whole chunk files go to the GPU engine (cc_scan_host); files of other sizes in
a copyset directory (snapshots of other geometry, stray files) are chained on
the CPU primitive, exactly where the reference would put them in the chain.
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

from . import crc as C

FORMAT_VERSION = 1      # datastore/define.h:39
FORMAT_VERSION_V2 = 2   # datastore/define.h:40


class CSErrorCode:
    """datastore/define.h:44-76 (subset used on this path)."""
    Success = 0
    InternalError = 1
    IncompatibleError = 2
    CrcCheckError = 3
    FileFormatError = 4
    ChunkNotExistError = 8


@dataclass
class ChunkFileMetaPage:
    version: int = FORMAT_VERSION_V2
    sn: int = 1
    correctedSn: int = 0
    location: bytes = b""
    bitmap_bits: int = 0
    bitmap: bytes = b""

    def encode(self, page_size: int = 4096) -> bytes:
        hdr = struct.pack("<BQQQ", self.version, self.sn, self.correctedSn, len(self.location))
        if self.location:
            nbytes = (self.bitmap_bits + 7) >> 3
            bm = (self.bitmap + bytes(nbytes))[:nbytes]
            hdr += self.location + struct.pack("<I", self.bitmap_bits) + bm
        out = bytearray(page_size)
        out[:len(hdr)] = hdr
        out[len(hdr):len(hdr) + 4] = struct.pack("<I", C.CRC32(hdr))
        return bytes(out)

    @classmethod
    def decode(cls, buf: bytes) -> Tuple[int, Optional["ChunkFileMetaPage"]]:
        """(CSErrorCode, metapage) like ChunkFileMetaPage::decode."""
        if len(buf) < 29:
            return CSErrorCode.CrcCheckError, None
        version, sn, csn, loc_size = struct.unpack_from("<BQQQ", buf, 0)
        n = 25
        m = cls(version, sn, csn)
        if loc_size > 0:
            # lengths that overrun the page cannot carry a valid CRC (the
            # reference would read past its buffer here)
            if loc_size > len(buf) - n - 8:
                return CSErrorCode.CrcCheckError, None
            m.location = bytes(buf[n:n + loc_size])
            n += loc_size
            (m.bitmap_bits,) = struct.unpack_from("<I", buf, n)
            n += 4
            nb = (m.bitmap_bits + 7) >> 3
            if nb > len(buf) - n - 4:
                return CSErrorCode.CrcCheckError, None
            m.bitmap = bytes(buf[n:n + nb])
            n += nb
        (rec,) = struct.unpack_from("<I", buf, n)
        if C.CRC32(bytes(buf[:n])) != rec:
            return CSErrorCode.CrcCheckError, None
        if version not in (FORMAT_VERSION, FORMAT_VERSION_V2):
            return CSErrorCode.IncompatibleError, None
        return CSErrorCode.Success, m


def chunk_file_name(chunk_id: int, snap_sn: Optional[int] = None) -> str:
    return f"chunk_{chunk_id}" if snap_sn is None else f"chunk_{chunk_id}_snap_{snap_sn}"


def write_chunk_file(path: str, meta: bytes, data) -> None:
    with open(path, "wb") as f:
        f.write(meta)
        f.write(memoryview(data).cast("B") if not isinstance(data, bytes) else data)


def read_into(path: str, dst) -> int:
    """pread a whole file into a (pinned) numpy buffer; returns bytes read."""
    fd = os.open(path, os.O_RDONLY)
    try:
        mv = memoryview(dst).cast("B")
        got = 0
        while got < mv.nbytes:
            n = os.preadv(fd, [mv[got:]], got)
            if n <= 0:
                break
            got += n
        return got
    finally:
        os.close(fd)


def copyset_hash_dir(data_dir: str, chunk_size: int = C.CHUNK_SIZE, meta_size: int = C.META_PAGE_SIZE,
                     io_threads: int = 0, page_bytes: int = C.PAGE_SIZE) -> str:
    """CopysetNode::GetHash over a real data directory: list, std::sort the
    names, chain CRC32 over whole files.  Chunk files (meta || data of the
    configured geometry: chunkserver.conf's chunk_size / meta_page_size, and
    block_size as the engine's page -- 4096 or 512, datastore_mock_unittest.cpp:4270-4279)
    are read AND hashed by the engine (cc_scan_files:
    native pread into pinned staging overlapped with the GPU scan); any other
    file -- or one the engine could not read -- is hashed on the CPU primitive.
    The chain is assembled with crc32c_combine in sorted-name order, identical
    to `crc = CRC32(crc, file)` over the same order."""
    names = sorted(os.listdir(data_dir))  # std::sort on std::string: bytewise
    if not names:
        return "0"
    fsize = chunk_size + meta_size
    sizes = [os.stat(os.path.join(data_dir, n)).st_size for n in names]
    file_crc: Dict[int, int] = {}
    chunk_idx = [i for i, s in enumerate(sizes) if s == fsize]
    if chunk_idx:
        st, _, _, fc = C.scan_files([os.path.join(data_dir, names[i]) for i in chunk_idx], chunk_size, meta_size,
                                    page_bytes, min(C.SCAN_SIZE, chunk_size), io_threads)
        for k, i in enumerate(chunk_idx):
            if st[k] == 0:
                file_crc[i] = int(fc[k])
    crc = 0
    for i, n in enumerate(names):
        if i in file_crc:
            crc = C.combine(crc, file_crc[i], sizes[i])
        else:
            with open(os.path.join(data_dir, n), "rb") as f:
                crc = C.CRC32(crc, f.read())
    return str(crc)


def get_hash(data_dir: str, chunk_size: int = C.CHUNK_SIZE, meta_size: int = C.META_PAGE_SIZE) -> Tuple[int, str]:
    """CopysetNode::GetHash's contract (copyset_node.cpp:925-975): (0, hash) on
    success, (-1, "") when listing, opening, fstat or reading any file fails
    (copyset_node_test.cpp:864-997 pins these cases)."""
    try:
        return 0, copyset_hash_dir(data_dir, chunk_size, meta_size)
    except OSError:
        return -1, ""
