"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

Python face of the CPU oracle (oracle/crc32c_oracle.c).  Imported only by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, always as the
checker; the product package ``curve_amd`` never imports this module.

Besides the CRC primitive it restates the reference's *geometry* on top of it:

* scan slices    -- ScanManager::ScanJobProcess (src/chunkserver/scan_manager.cpp:233-291):
                    1 metapage op + chunkSize/scanSize data slices per chunk, each
                    slice CRC = CRC32(buf, size) (src/chunkserver/op_request.cpp:794, :847)
* chunk hash     -- CSChunkFile::GetHash (src/chunkserver/datastore/chunkserver_chunkfile.cpp:785-811):
                    CRC32(0, rawfile[offset, offset+length)) -- raw *file* offset, metapage included
* copyset hash   -- CopysetNode::GetHash (src/chunkserver/copyset_node.cpp:925-975):
                    std::sort(names); crc = CRC32(crc, whole file) chained from 0
* conf epoch CRC -- ConfEpochFile::ConfEpochCrc (src/chunkserver/conf_epoch_file.cpp:148-164)
"""
from __future__ import annotations

import ctypes
import os
import struct
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u32, u64, sz, vp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p
        for name in ("oc_crc32c_bitwise", "oc_crc32c_table", "oc_crc32c_sse42"):
            f = getattr(L, name)
            f.argtypes = [u32, vp, sz]
            f.restype = u32
        L.oc_crc32c_value.argtypes = [vp, sz]
        L.oc_crc32c_value.restype = u32
        L.oc_raw_shift.argtypes = [u32, u64]
        L.oc_raw_shift.restype = u32
        L.oc_crc32c_combine.argtypes = [u32, u32, u64]
        L.oc_crc32c_combine.restype = u32
        L.oc_page_crcs.argtypes = [vp, u64, u32, vp]
        L.oc_page_crcs.restype = None
        L.oc_page_crcs_mt.argtypes = [vp, u64, u32, vp, ctypes.c_int]
        L.oc_page_crcs_mt.restype = ctypes.c_int
        _lib = L
    return _lib


def _buf(data):
    """(pointer, nbytes, keepalive) for bytes / bytearray / numpy arrays."""
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data)
        return a.ctypes.data_as(ctypes.c_void_p), a.nbytes, a
    if isinstance(data, (bytes, bytearray, memoryview)):
        b = bytes(data)
        return ctypes.c_char_p(b), len(b), b
    raise TypeError(type(data))


def crc32c(data, crc: int = 0, impl: str = "sse42") -> int:
    """curve::common::CRC32(crc, p, n) == butil::crc32c::Extend (src/common/crc32.h:53-55).
    With crc=0 this is CRC32(p, n) == butil::crc32c::Value (src/common/crc32.h:40-42)."""
    p, n, _keep = _buf(data)
    f = {"sse42": lib().oc_crc32c_sse42, "table": lib().oc_crc32c_table,
         "bitwise": lib().oc_crc32c_bitwise}[impl]
    return int(f(crc & 0xFFFFFFFF, p, n))


def crc32c_py(data: bytes, crc: int = 0) -> int:
    """Pure-Python bitwise CRC32C (small inputs only): a fourth, dependency-free formulation."""
    l = (crc ^ 0xFFFFFFFF) & 0xFFFFFFFF
    for b in bytes(data):
        l ^= b
        for _ in range(8):
            l = (l >> 1) ^ (0x82F63B78 if l & 1 else 0)
    return l ^ 0xFFFFFFFF


def combine(crc_a: int, crc_b: int, len_b: int) -> int:
    return int(lib().oc_crc32c_combine(crc_a, crc_b, len_b))


def raw_shift(reg: int, nbytes: int) -> int:
    return int(lib().oc_raw_shift(reg, nbytes))


def page_crcs(pages: np.ndarray, page_bytes: int = 4096, threads: int = 1) -> np.ndarray:
    a = np.ascontiguousarray(pages).view(np.uint8).reshape(-1)
    assert a.nbytes % page_bytes == 0
    n = a.nbytes // page_bytes
    out = np.empty(n, dtype=np.uint32)
    if threads > 1:
        lib().oc_page_crcs_mt(a.ctypes.data_as(ctypes.c_void_p), n, page_bytes,
                              out.ctypes.data_as(ctypes.c_void_p), threads)
    else:
        lib().oc_page_crcs(a.ctypes.data_as(ctypes.c_void_p), n, page_bytes,
                           out.ctypes.data_as(ctypes.c_void_p))
    return out


# --------------------------------------------------------------------------
# deterministic synthetic data (splitmix64, seed 0xC0FFEE ^ chunk)
# --------------------------------------------------------------------------
_M64 = (1 << 64) - 1


def splitmix64_bytes(seed: int, nbytes: int) -> np.ndarray:
    """nbytes of splitmix64 output (little-endian u64 stream) from `seed`."""
    n64 = (nbytes + 7) // 8
    with np.errstate(over="ignore"):
        idx = np.arange(1, n64 + 1, dtype=np.uint64)
        z = np.uint64(seed & _M64) + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.view(np.uint8)[:nbytes].copy()


# --------------------------------------------------------------------------
# reference geometry restated over the oracle CRC
# --------------------------------------------------------------------------
CHUNK_SIZE = 16 * 1024 * 1024      # conf/chunkserver.conf:13 (chunksize)
META_PAGE_SIZE = 4096              # conf/chunkserver.conf:16 (metapagesize)
SCAN_SIZE = 4 * 1024 * 1024        # conf/chunkserver.conf:114 (copyset.scan_size_byte)


def scan_slices(meta_page: bytes, data: bytes, scan_size: int = SCAN_SIZE):
    """(offset, len, crc) for every scan op of one chunk, in ScanJobProcess order:
    the metapage op (len = metapage size, offset 0) then data slices at offset k*scan_size
    (src/chunkserver/scan_manager.cpp:250-283).  crc = CRC32(buf, size) (op_request.cpp:794)."""
    out = [(0, len(meta_page), crc32c(meta_page))]
    for off in range(0, len(data), scan_size):
        out.append((off, scan_size, crc32c(data[off:off + scan_size])))
    return out


def chunk_hash(raw_file: bytes, offset: int, length: int) -> str:
    """CSChunkFile::GetHash: to_string(CRC32(0, rawfile[offset:offset+length]))."""
    return str(crc32c(raw_file[offset:offset + length], 0))


def copyset_hash(files: dict) -> str:
    """CopysetNode::GetHash over {name: bytes}: sorted names, chained CRC from 0."""
    crc = 0
    for name in sorted(files):
        crc = crc32c(files[name], crc)
    return str(crc)


def conf_epoch_crc(logic_pool_id: int, copyset_id: int, epoch: int,
                   magic: int = 0x6225929368674119) -> int:
    """ConfEpochFile::ConfEpochCrc (conf_epoch_file.cpp:148-164), chained per field."""
    crc = 0
    crc = crc32c(struct.pack("<I", logic_pool_id), crc)
    crc = crc32c(struct.pack("<I", copyset_id), crc)
    crc = crc32c(struct.pack("<Q", epoch), crc)
    crc = crc32c(struct.pack("<Q", magic), crc)
    return crc
