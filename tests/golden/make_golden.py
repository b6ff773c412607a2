"""Generate tests/golden/*.json fixtures (committed; rerun to regenerate).

Two kinds of vectors:
  * known answers copied (as data) from the reference's own tests -- these PIN
    the oracle: RFC 3720 B.4 (test/common/crc32_test.cpp:49-84), Extend identity
    (:90-93), copyset hash 1355371765 (test/chunkserver/copyset_node_test.cpp:811-835),
    conf-epoch CRC 599727352 (test/chunkserver/conf_epoch_file_test.cpp:103-106);
  * vectors computed by the oracle AFTER it reproduces the pinned ones, cross-
    checked by an independent pure-Python bitwise CRC where small enough.

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle as O  # noqa: E402

RFC_PDU = [0x01, 0xc0, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
           0x14, 0x00, 0x00, 0x00, 0x00, 0x00, 0x04, 0x00, 0x00, 0x00, 0x00, 0x14, 0x00, 0x00, 0x00, 0x18,
           0x28, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x02, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00]

COPYSET_FILES = {  # copyset_node_test.cpp:811-835 (echo adds '\n'; dd bs=512 count=15)
    "test-1.txt": "wwwww\n",
    "test-2.txt": "abcddddddddd333\n",
    "test-3.txt": None,  # 7680 zero bytes
    "test-4.txt": "mmmmmmmm\n",
    "test-5.txt": "eeeeeeeeeee\n",
}


def copyset_bytes():
    return {k: (bytes(7680) if v is None else v.encode()) for k, v in COPYSET_FILES.items()}


def metapage_v2(sn: int = 1, corrected_sn: int = 0, page_size: int = 4096) -> bytes:
    """ChunkFileMetaPage::encode for a non-clone chunk (chunkserver_chunkfile.cpp:64-88):
    version(u8)=2 sn(u64) correctedSn(u64) loc_size(size_t=0), CRC32 of those 25 B at byte 25."""
    hdr = struct.pack("<BQQQ", 2, sn, corrected_sn, 0)
    assert len(hdr) == 25
    crc = O.crc32c(hdr)
    page = bytearray(page_size)
    page[:25] = hdr
    page[25:29] = struct.pack("<I", crc)
    return bytes(page)


def synthetic_chunk(seed: int):
    data = O.splitmix64_bytes(seed, O.CHUNK_SIZE)
    return metapage_v2(), data


def main():
    g = {}
    # ---- pinned known answers (reference test data) ----
    g["rfc3720"] = [
        {"input": "zeros32", "crc": 0x8a9136aa},
        {"input": "ff32", "crc": 0x62a8ab43},
        {"input": "inc32", "crc": 0x46dd794e},
        {"input": "dec32", "crc": 0x113fdb5c},
        {"input_hex": bytes(RFC_PDU).hex(), "crc": 0xd9963a56},
    ]
    g["extend"] = {"a": "hello ", "b": "world"}
    g["copyset_hash"] = {"files": COPYSET_FILES, "zero_file_bytes": 7680, "hash": "1355371765"}
    g["conf_epoch"] = {"logicPoolId": 123, "copysetId": 1345, "epoch": 0,
                       "magic": 0x6225929368674119, "crc": 599727352}
    # GetChunkHash of a chunk whose first 4 KiB block was written with 'a'
    # (test/chunkserver/chunk_service_test.cpp:505-523 write, :563-578 hash)
    g["chunk_service_hash"] = {"data_byte": "a", "bytes": 4096, "hash": "650595490",
                               "note": "= CRC32('a' x 4096), i.e. the DATA block; CSChunkFile::GetHash "
                                       "preads the raw file (chunkserver_chunkfile.cpp:796, mock test "
                                       "datastore_mock_unittest.cpp:4238 pins Read(fd, buf, 0, 4096)), "
                                       "which at offset 0 returns the metapage -- see metapage_residue"}
    # GetCopysetStatus(queryhash) after 25 x 4 KiB writes of 'b' at offsets
    # 4096*i to chunk 1 of a one-chunk copyset, 16 MiB chunks, 4 KiB metapage
    # (test/chunkserver/chunkserver_snapshot_test.cpp:339-388; writes:
    # test/integration/common/peer_cluster.cpp:459-495)
    g["copyset_hash_one_chunk"] = {"chunk_bytes": 16 << 20, "meta_bytes": 4096, "fill": "b", "blocks": 25,
                                   "block_bytes": 4096, "file": "chunk_1", "hash": "3049021227"}
    # verify the oracle reproduces them before deriving anything else
    assert O.copyset_hash(copyset_bytes()) == g["copyset_hash"]["hash"]
    assert O.conf_epoch_crc(123, 1345, 0) == 599727352
    assert O.crc32c(bytes(32)) == 0x8a9136aa
    assert str(O.crc32c(b"a" * 4096)) == g["chunk_service_hash"]["hash"]
    one = metapage_v2() + b"b" * (25 * 4096) + bytes((16 << 20) - 25 * 4096)
    assert O.copyset_hash({"chunk_1": one}) == g["copyset_hash_one_chunk"]["hash"]

    # ---- derived vectors ----
    g["zero_page"] = {"bytes": 4096, "crc": O.crc32c(bytes(4096))}
    assert g["zero_page"]["crc"] == O.crc32c_py(bytes(4096)) == 0x98F94189

    pages = O.splitmix64_bytes(0x5EED, 64 * 4096)
    crcs = O.page_crcs(pages, 4096)
    g["seeded_pages"] = {"generator": "splitmix64", "seed": 0x5EED, "page_bytes": 4096, "n_pages": 64,
                         "crcs": [int(c) for c in crcs]}
    for i in (0, 17, 63):
        assert O.crc32c_py(pages[i * 4096:(i + 1) * 4096].tobytes()) == crcs[i]

    # 512-B pages (blocksize 512 is allowed, conf/chunkserver.conf:17-22)
    p512 = O.splitmix64_bytes(0x512, 64 * 512)
    g["seeded_pages_512"] = {"generator": "splitmix64", "seed": 0x512, "page_bytes": 512, "n_pages": 64,
                             "crcs": [int(c) for c in O.page_crcs(p512, 512)]}

    # every zero-padded metapage of a given header length has the same CRC:
    # encode appends CRC32(header) little-endian, so CRC32(header || crc) is
    # the CRC-32C residue whatever the header bytes, and the zero padding to
    # 4 KiB shifts it by an amount fixed by the header length (25 B non-clone)
    res = {O.crc32c(metapage_v2(sn, csn)) for sn, csn in ((1, 0), (7, 3), (2**63, 5))}
    assert len(res) == 1
    hdr = struct.pack("<BQQQ", 1, 3, 1, 0)
    residue = O.crc32c(hdr + struct.pack("<I", O.crc32c(hdr)))
    clone_hdr = struct.pack("<BQQQ", 2, 9, 0, 13) + b"curvefs:/f@1x" + struct.pack("<I", 20) + bytes([0xA5, 0x0F, 0x03])
    assert O.crc32c(clone_hdr + struct.pack("<I", O.crc32c(clone_hdr))) == residue
    g["metapage_residue"] = {"page_bytes": 4096, "crc": res.pop(), "residue": residue,
                             "note": "CRC32 of ANY encoded non-clone 4 KiB metapage (ScanMap.crc of the metapage "
                                     "op; GetChunkHash(offset 0, 4096)); residue = CRC32(h || CRC32(h)_le) for "
                                     "every header h"}

    # one synthetic 16 MiB chunk: slices, metapage, chunk hash, page CRCs
    meta, data = synthetic_chunk(0xC0FFEE)
    raw = meta + data.tobytes()
    slices = O.scan_slices(meta, data.tobytes())
    pc = O.page_crcs(data, 4096)
    pc.astype("<u4").tofile(os.path.join(HERE, "chunk_c0ffee_pages.u32"))
    g["chunk_c0ffee"] = {
        "generator": "splitmix64", "seed": 0xC0FFEE, "chunk_bytes": O.CHUNK_SIZE,
        "metapage": {"version": 2, "sn": 1, "correctedSn": 0, "crc": O.crc32c(meta)},
        "scan_slices": [{"offset": o, "len": n, "crc": c} for (o, n, c) in slices],
        "chunk_hash_0_chunksize": O.chunk_hash(raw, 0, O.CHUNK_SIZE),
        "chunk_hash_4096_8192": O.chunk_hash(raw, 4096, 8192),
        "whole_file_crc": O.crc32c(raw),
        "page_crcs_file": "chunk_c0ffee_pages.u32",
        "page_crcs_crc": O.crc32c(pc.astype("<u4").tobytes()),
    }

    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(g, f, indent=1)
    print("wrote", os.path.join(HERE, "golden.json"))


if __name__ == "__main__":
    main()
