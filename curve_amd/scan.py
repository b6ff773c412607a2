"""Scan-service / hash surfaces of the chunkserver, on the device engine.

Mirrors, with the reference's names and semantics:
  ScanMap                        proto/scan.proto:23-31
  ScanChunkRequest::OnApply      src/chunkserver/op_request.cpp:769-820 (slice CRC -> ScanMap)
  ScanManager slice schedule     src/chunkserver/scan_manager.cpp:250-283 (metapage op + data slices)
  CSChunkFile::GetHash           src/chunkserver/datastore/chunkserver_chunkfile.cpp:785-811
  CopysetNode::GetHash           src/chunkserver/copyset_node.cpp:925-975
Data lives in HBM as a `DevicePool`: one [n_chunks, chunk_size] data tensor and
one [n_chunks, meta_page_size] metapage tensor (a chunk file is
metapage || data, chunkserver_chunkfile.cpp:497-536).  All arithmetic is in
libcurvecrc's kernels; torch only owns the memory and the stream.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

from . import crc as C

CHUNK_SIZE = C.CHUNK_SIZE
META_PAGE_SIZE = C.META_PAGE_SIZE
SCAN_SIZE = C.SCAN_SIZE
PAGE_SIZE = C.PAGE_SIZE
FORMAT_VERSION_V2 = 2  # datastore/define.h:40


@dataclass(frozen=True)
class ScanMap:
    """proto/scan.proto:23-31 (all fields required)."""
    logicalPoolId: int
    copysetId: int
    chunkId: int
    index: int
    crc: int
    offset: int
    len: int


def compare_maps(local: Optional[ScanMap], followers: Sequence[ScanMap]) -> Tuple[bool, Optional[ScanMap]]:
    """ScanManager::CompareMap (scan_manager.cpp:367-409): the leader's map must
    equal BOTH followers' maps in every field (MessageDifferencer::Equals,
    `index` included).  Returns (consistent, map to push to FailedScanMap)."""
    if local is None or len(followers) != 2:
        return False, None  # "waitingNum is 0 but there isn't three scanmap": logged, not failed
    if local == followers[0] and local == followers[1]:
        return True, None
    return False, local


def chunk_file_name(chunk_id: int, snap_sn: Optional[int] = None) -> str:
    """FileNameOperator (src/chunkserver/datastore/filename_operator.h:55-62)."""
    return f"chunk_{chunk_id}" if snap_sn is None else f"chunk_{chunk_id}_snap_{snap_sn}"


def copyset_after_bytes(names: Sequence[str], sizes: Sequence[int]) -> List[int]:
    """For each file (in the caller's order): bytes of the copyset's files that
    sort after it.  CopysetNode::GetHash uses std::sort on the names
    (lexicographic: chunk_10 < chunk_2, copyset_node.cpp:938)."""
    order = sorted(range(len(names)), key=lambda i: names[i])
    after = [0] * len(names)
    acc = 0
    for i in reversed(order):
        after[i] = acc
        acc += sizes[i]
    return after


def scan_schedule(chunk_size: int = CHUNK_SIZE, scan_size: int = SCAN_SIZE, meta_page_size: int = META_PAGE_SIZE):
    """(readMetaPage, offset, len) for each scan op of one chunk, in ScanJobProcess
    order; Init requires scanSize <= chunkSize and chunkSize % scanSize == 0
    (scan_manager.cpp:43-48)."""
    if scan_size > chunk_size or chunk_size % scan_size:
        raise ValueError("scanSize must divide chunkSize")
    ops = [(True, 0, meta_page_size)]
    ops += [(False, off, scan_size) for off in range(0, chunk_size, scan_size)]
    return ops


class DevicePool:
    """A device-resident set of chunk files (one copyset-agnostic batch)."""

    def __init__(self, data, meta, chunk_ids: Sequence[int], page_bytes: int = PAGE_SIZE,
                 scan_size: int = SCAN_SIZE):
        import torch
        self.torch = torch
        self.data = data          # [n, chunk_size] uint8, device
        self.meta = meta          # [n, meta_page_size] uint8, device
        self.n = data.shape[0]
        self.chunk_size = data.shape[1]
        self.meta_size = meta.shape[1]
        self.page_bytes = page_bytes
        self.scan_size = scan_size
        self.chunk_ids = list(chunk_ids)
        assert len(self.chunk_ids) == self.n == meta.shape[0]
        assert self.chunk_size % scan_size == 0 and scan_size % page_bytes == 0
        dev = data.device
        self.page_crcs = torch.empty(self.n * self.chunk_size // page_bytes, dtype=torch.int32, device=dev)
        self.meta_crcs = torch.empty(self.n * max(1, self.meta_size // page_bytes), dtype=torch.int32, device=dev)
        self.slice_crcs = torch.empty(self.n * self.chunk_size // scan_size, dtype=torch.int32, device=dev)
        self.data_crcs = torch.empty(self.n, dtype=torch.int32, device=dev)
        self.file_crcs = torch.empty(self.n, dtype=torch.int32, device=dev)

    # -- the hot path ------------------------------------------------------
    def hash_pages(self, stream=None):
        C.page_crc(self.data, self.page_bytes, out=self.page_crcs, stream=stream)
        return self.page_crcs

    def epilogue_ok(self) -> bool:
        ppc, pps = self.chunk_size // self.page_bytes, self.scan_size // self.page_bytes
        if ppc % 256:
            return False
        q = ppc // 256
        return pps % q == 0 and (pps // q) & (pps // q - 1) == 0 and pps // q <= 256

    def scan(self, stream=None, after_bytes=None, group=None, digest=None):
        """Page CRCs -> 4 MiB slice CRCs (ScanMap.crc), metapage CRCs and
        chunk-file CRCs (+ optionally the per-copyset digest partials); all on
        the device.  The epilogue is ONE fused launch (cc_scan_epilogue_dev)
        when the geometry allows, else fold + fold + combine (+ digest)."""
        self.hash_pages(stream)
        C.page_crc(self.meta, self.meta_size, out=self.meta_crcs[: self.n], stream=stream)
        per_slice = self.scan_size // self.page_bytes
        if self.epilogue_ok():
            mult = C.xpow8(after_bytes, stream=stream) if digest is not None else None
            C.scan_epilogue(self.page_crcs, self.meta_crcs[: self.n], self.n, self.chunk_size // self.page_bytes,
                            self.page_bytes, per_slice, self.slice_crcs, self.file_crcs,
                            mult, group, digest, stream=stream)
            return self.slice_crcs
        C.fold(self.page_crcs, per_slice, self.page_bytes, out=self.slice_crcs, stream=stream)
        C.fold(self.slice_crcs, self.chunk_size // self.scan_size, self.scan_size, out=self.data_crcs, stream=stream)
        C.combine_dev(self.meta_crcs[: self.n], self.data_crcs, self.chunk_size, out=self.file_crcs, stream=stream)
        if digest is not None:
            C.digest_dev(self.file_crcs, after_bytes, group, digest.numel(), out=digest, stream=stream)
        return self.slice_crcs

    def verify(self, expected_page_crcs, stream=None):
        return C.page_verify(self.data, expected_page_crcs, self.page_bytes, stream=stream)

    def bad_pages(self, expected_page_crcs, max_bad: int = 4096, stream=None):
        """Every mismatching page as sorted (chunk index, page in chunk) pairs
        -- what a scan reports per chunk (FailedScanMap granularity is the
        chunk; the page pinpoints the repair).  Raises if more than max_bad."""
        cnt, lst = C.page_verify_list(self.data, expected_page_crcs, self.page_bytes, max_bad, stream=stream)
        n = int(cnt[0])
        if n > max_bad:
            raise C.CurveCrcError(-74, f"{n} bad pages > max_bad={max_bad}")
        ppc = self.chunk_size // self.page_bytes
        pages = sorted(int(p) for p in lst[:n].cpu().tolist())
        return [(p // ppc, p % ppc) for p in pages]

    # -- reference surfaces built on the device results ----------------------
    def scan_maps(self, logical_pool_id: int, copyset_id: int, first_index: int = 0) -> List[ScanMap]:
        """ScanMaps as ScanChunkRequest::OnApply builds them (op_request.cpp:795-803),
        one per scan op in ScanJobProcess order; `index` is the raft log index,
        here a running counter from first_index.  Chunks whose metapage version
        is not FORMAT_VERSION_V2 are not scanned (scan_manager.cpp:228-231)."""
        slices = C.as_u32(self.slice_crcs)
        metas = C.as_u32(self.meta_crcs[: self.n])
        versions = self.meta[:, 0].cpu().tolist()
        per_chunk = self.chunk_size // self.scan_size
        out, idx = [], first_index
        for c, cid in enumerate(self.chunk_ids):
            if versions[c] != FORMAT_VERSION_V2:
                continue
            out.append(ScanMap(logical_pool_id, copyset_id, cid, idx, metas[c], 0, self.meta_size))
            idx += 1
            for k in range(per_chunk):
                out.append(ScanMap(logical_pool_id, copyset_id, cid, idx, slices[c * per_chunk + k],
                                   k * self.scan_size, self.scan_size))
                idx += 1
        return out

    def chunk_hash(self, c: int, offset: int = 0, length: Optional[int] = None) -> str:
        """CSChunkFile::GetHash(offset, length): to_string(CRC32(0, rawfile[offset,
        offset+length))) over the raw FILE (metapage at file offset 0, data after
        it: chunkserver_chunkfile.cpp:785-811), any offset/length inside the file.
        The metapage part and the data part are hashed on the device
        (cc_crc_ranges_dev) and combined."""
        if length is None:
            length = self.chunk_size
        end = offset + length
        if offset < 0 or end > self.meta_size + self.chunk_size:
            raise ValueError("range beyond the chunk file")
        crc, parts = 0, []
        if offset < self.meta_size:
            parts.append((self.meta[c], offset, min(end, self.meta_size) - offset))
        if end > self.meta_size:
            d0 = max(offset, self.meta_size) - self.meta_size
            parts.append((self.data[c], d0, end - self.meta_size - d0))
        for buf, o, n in parts:
            v = C.as_u32(C.crc_ranges(buf, [o], [n]))[0]
            crc = C.combine(crc, v, n)
        return str(crc)

    def copyset_digest_partial(self, names: Sequence[str], after_bytes: Sequence[int], group: Sequence[int],
                               n_groups: int, stream=None):
        """XOR partials of the per-copyset chained hash for the files this pool
        holds; XOR over all holders == CopysetNode::GetHash."""
        torch = self.torch
        dev = self.data.device
        after = torch.tensor(list(after_bytes), dtype=torch.int64, device=dev)
        grp = torch.tensor(list(group), dtype=torch.int32, device=dev)
        return C.digest_dev(self.file_crcs, after, grp, n_groups, stream=stream)


def scan_copyset_dir(data_dir: str, logical_pool_id: int, copyset_id: int, first_index: int = 0,
                     chunk_size: int = CHUNK_SIZE, meta_size: int = META_PAGE_SIZE, scan_size: int = SCAN_SIZE,
                     io_threads: int = 0, page_bytes: int = PAGE_SIZE) -> List[ScanMap]:
    """ScanManager::ScanJobProcess over a copyset's chunk files on disk
    (scan_manager.cpp:210-296): for every chunk (`chunk_<id>`, the ChunkMap;
    snapshots are not scanned) with a V2 metapage, the metapage op then the
    data slices, each a ScanMap as ScanChunkRequest::OnApply builds it.  The
    engine reads the files itself and hashes them on the GPU (cc_scan_files);
    the reference's per-slice CRC32(readBuffer, size) (op_request.cpp:794) is
    the same value.  Chunks in ascending id order (the reference iterates an
    unordered map).  Unreadable chunk files raise OSError (InternalError ->
    LOG(FATAL) in the reference, op_request.cpp:813-815)."""
    import os
    import re
    if scan_size > chunk_size or chunk_size % scan_size:
        raise ValueError("scanSize must divide chunkSize")
    pat = re.compile(r"^chunk_(\d+)$")
    ids = sorted(int(m.group(1)) for n in os.listdir(data_dir) if (m := pat.match(n)))
    paths = [os.path.join(data_dir, chunk_file_name(i)) for i in ids]
    st, mc, sc, _ = C.scan_files(paths, chunk_size, meta_size, page_bytes, scan_size, io_threads)
    out, idx = [], first_index
    for k, cid in enumerate(ids):
        if st[k] != 0:
            raise OSError(-int(st[k]) if st[k] < 0 else 22, f"cannot scan {paths[k]}")
        with open(paths[k], "rb") as f:
            version = f.read(1)[0]
        if version != FORMAT_VERSION_V2:
            continue
        out.append(ScanMap(logical_pool_id, copyset_id, cid, idx, int(mc[k]), 0, meta_size))
        idx += 1
        for j in range(chunk_size // scan_size):
            out.append(ScanMap(logical_pool_id, copyset_id, cid, idx, int(sc[k, j]), j * scan_size, scan_size))
            idx += 1
    return out
