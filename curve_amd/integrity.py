"""Per-page CRC persistence + integrity jobs.

The reference computes no per-page data CRC and has nowhere to keep one (the
chunk metapage holds version/sn/correctedSn/location/bitmap + a header CRC,
chunkserver_chunkfile.cpp:64-88), so verify-on-read needs a NEW artefact.  This
module defines it and drives it through the engine:

Sidecar `<copyset dir>/pcrc/<chunk file name>.pcrc` -- deliberately NOT in the
data directory, because CopysetNode::GetHash (copyset_node.cpp:931-970) chains
every file listed there and a sidecar would change the copyset hash.
Layout (little-endian):
    0  magic  b"CVPCRC01"
    8  version u32 (=1) | page_bytes u32 | n_pages u32 | reserved u32
   24  chunk_sn u64       (sn of the chunk when the table was computed)
   32  header_crc u32     (CRC32C of bytes [0, 32))
   36  table_crc u32      (CRC32C of the page-CRC array)
   40  page CRCs, n_pages x u32
A table is trusted only if both CRCs check; a bad table is reported as
`TableCorrupt`, never used to condemn data.

Jobs mirror proto/integrity.proto (IntegrityService: ScheduleJob / CancelJob /
PauseJob / ResumeJob / ListJobs; IntegrityJob{id, copyset, state, progress,
sched_time, start_time}; INTEGRITY_JOB_STATE) -- declared and compiled in the
reference (proto/BUILD:78) with no implementation anywhere in src/.  A job walks
one copyset data directory: every chunk file is read into pinned memory,
hashed page by page on the GPU, and compared with its sidecar (or the sidecar is
created when missing).  Bad pages are recorded per file (first bad page, count).
"""
from __future__ import annotations

import enum
import os
import struct
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from . import crc as C

MAGIC = b"CVPCRC01"
HEADER_BYTES = 40


class IntegrityJobState(enum.IntEnum):  # proto/integrity.proto:23-30
    WAITING = 0
    RUNNING = 1
    CANCELED = 2
    FINISHED = 3
    PAUSED = 4
    FAILED = 5


class IntegrityOpStatus(enum.IntEnum):  # proto/integrity.proto:45-48
    SUCCESS = 0
    FAILURE_UNKNOWN = 1


class TableCorrupt(Exception):
    pass


def encode_table(page_crcs: np.ndarray, page_bytes: int, chunk_sn: int) -> bytes:
    crcs = np.ascontiguousarray(page_crcs, dtype="<u4")
    head = MAGIC + struct.pack("<IIIIQ", 1, page_bytes, crcs.size, 0, chunk_sn)
    body = crcs.tobytes()
    return head + struct.pack("<II", C.CRC32(head), C.CRC32(body)) + body


def decode_table(buf: bytes):
    """-> (page_bytes, chunk_sn, page CRCs as uint32 array); TableCorrupt if bad."""
    if len(buf) < HEADER_BYTES or buf[:8] != MAGIC:
        raise TableCorrupt("bad magic / short header")
    ver, page_bytes, n, _, sn = struct.unpack_from("<IIIIQ", buf, 8)
    hcrc, tcrc = struct.unpack_from("<II", buf, 32)
    if C.CRC32(buf[:32]) != hcrc or ver != 1:
        raise TableCorrupt("header checksum / version")
    body = buf[HEADER_BYTES:HEADER_BYTES + 4 * n]
    if len(body) != 4 * n or C.CRC32(body) != tcrc:
        raise TableCorrupt("table checksum")
    return page_bytes, sn, np.frombuffer(body, dtype="<u4").copy()


def table_dir_for(data_dir: str) -> str:
    """<copyset>/data -> <copyset>/pcrc (sibling of the data directory)."""
    return os.path.join(os.path.dirname(os.path.abspath(data_dir)), "pcrc")


def sidecar_path(chunk_path: str, table_dir: Optional[str] = None) -> str:
    d = table_dir or table_dir_for(os.path.dirname(os.path.abspath(chunk_path)))
    return os.path.join(d, os.path.basename(chunk_path) + ".pcrc")


@dataclass
class FileResult:
    name: str
    pages: int
    bad_pages: int = 0
    first_bad: int = -1
    table: str = "ok"          # ok | created | corrupt


@dataclass
class IntegrityJob:  # proto/integrity.proto:32-39
    id: int
    copyset: int
    data_dir: str
    state: IntegrityJobState = IntegrityJobState.WAITING
    progress: int = 0          # percent of chunk files done
    sched_time: int = 0
    start_time: int = 0
    results: List[FileResult] = field(default_factory=list)
    error: str = ""


def hash_chunk_files(paths: List[str], chunk_size: int, meta_size: int, page_bytes: int):
    """Page CRCs of the DATA part of each chunk file (file = metapage || data;
    CSChunkFile::Read reads at offset + metaPageSize).  The engine preads the
    files itself (cc_scan_files, slice = one page, so the per-slice CRCs ARE the
    page CRCs).  -> list of uint32 arrays; IOError for an unreadable file."""
    st, _, pcs, _ = C.scan_files(paths, chunk_size, meta_size, page_bytes, page_bytes)
    bad = np.flatnonzero(st)
    if bad.size:
        raise IOError(f"cannot read {paths[bad[0]]}: status {int(st[bad[0]])}")
    return [pcs[k].copy() for k in range(len(paths))]


class IntegrityService:
    """In-process IntegrityService (ScheduleJob/CancelJob/PauseJob/ResumeJob/
    ListJobs).  One worker thread runs jobs FIFO; Pause/Cancel take effect at
    chunk-file batch boundaries."""

    def __init__(self, chunk_size: int = C.CHUNK_SIZE, meta_size: int = C.META_PAGE_SIZE,
                 page_bytes: int = C.PAGE_SIZE, batch: int = 16, create_missing: bool = True):
        self.chunk_size, self.meta_size, self.page_bytes = chunk_size, meta_size, page_bytes
        self.batch, self.create_missing = batch, create_missing
        self._jobs: Dict[int, IntegrityJob] = {}
        self._order: List[int] = []
        self._cv = threading.Condition()
        self._stop = False
        self._worker = threading.Thread(target=self._run, daemon=True)
        self._worker.start()

    # -- RPC surface -----------------------------------------------------
    def ScheduleJob(self, job_id: int, copyset: int, data_dir: str) -> IntegrityOpStatus:
        with self._cv:
            if job_id in self._jobs:
                return IntegrityOpStatus.FAILURE_UNKNOWN
            self._jobs[job_id] = IntegrityJob(job_id, copyset, data_dir, sched_time=int(time.time()))
            self._order.append(job_id)
            self._cv.notify_all()
        return IntegrityOpStatus.SUCCESS

    def _set(self, job_id: int, frm, to) -> IntegrityOpStatus:
        with self._cv:
            j = self._jobs.get(job_id)
            if j is None or j.state not in frm:
                return IntegrityOpStatus.FAILURE_UNKNOWN
            j.state = to
            self._cv.notify_all()
        return IntegrityOpStatus.SUCCESS

    def CancelJob(self, job_id: int) -> IntegrityOpStatus:
        S = IntegrityJobState
        return self._set(job_id, (S.WAITING, S.RUNNING, S.PAUSED), S.CANCELED)

    def PauseJob(self, job_id: int) -> IntegrityOpStatus:
        S = IntegrityJobState
        return self._set(job_id, (S.WAITING, S.RUNNING), S.PAUSED)

    def ResumeJob(self, job_id: int) -> IntegrityOpStatus:
        S = IntegrityJobState
        return self._set(job_id, (S.PAUSED,), S.WAITING)

    def ListJobs(self) -> List[IntegrityJob]:
        with self._cv:
            return [self._jobs[i] for i in self._order]

    def wait(self, job_id: int, timeout: float = 60.0) -> IntegrityJob:
        end = time.time() + timeout
        with self._cv:
            while self._jobs[job_id].state in (IntegrityJobState.WAITING, IntegrityJobState.RUNNING):
                left = end - time.time()
                if left <= 0:
                    break
                self._cv.wait(left)
            return self._jobs[job_id]

    def close(self):
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        self._worker.join(timeout=10)

    # -- worker ------------------------------------------------------------
    def _next(self) -> Optional[IntegrityJob]:
        for i in self._order:
            if self._jobs[i].state == IntegrityJobState.WAITING:
                return self._jobs[i]
        return None

    def _run(self):
        import torch
        if torch.cuda.is_available():
            torch.cuda.set_device(0)
        while True:
            with self._cv:
                while not self._stop and self._next() is None:
                    self._cv.wait()
                if self._stop:
                    return
                job = self._next()
                job.state = IntegrityJobState.RUNNING
                if not job.start_time:
                    job.start_time = int(time.time())
            try:
                self._do(job)
            except Exception as e:  # noqa: BLE001 -- reported through the job state
                with self._cv:
                    job.state, job.error = IntegrityJobState.FAILED, repr(e)
                    self._cv.notify_all()

    def _do(self, job: IntegrityJob):
        fsize = self.chunk_size + self.meta_size
        names = sorted(n for n in os.listdir(job.data_dir) if os.path.getsize(os.path.join(job.data_dir, n)) == fsize)
        os.makedirs(table_dir_for(job.data_dir), exist_ok=True)
        done = {r.name for r in job.results}
        todo = [n for n in names if n not in done]
        for b0 in range(0, len(todo), self.batch):
            with self._cv:
                if job.state != IntegrityJobState.RUNNING:  # paused or canceled at a batch boundary
                    self._cv.notify_all()
                    return
            part = todo[b0:b0 + self.batch]
            paths = [os.path.join(job.data_dir, n) for n in part]
            crcs = hash_chunk_files(paths, self.chunk_size, self.meta_size, self.page_bytes)
            for n, p, pc in zip(part, paths, crcs):
                job.results.append(self._check(n, p, pc))
            with self._cv:
                job.progress = int(100 * len(job.results) / max(1, len(names)))
        with self._cv:
            if job.state == IntegrityJobState.RUNNING:
                job.state, job.progress = IntegrityJobState.FINISHED, 100
            self._cv.notify_all()

    def _check(self, name: str, path: str, pc: np.ndarray) -> FileResult:
        from .chunkfile import ChunkFileMetaPage
        side = sidecar_path(path)
        res = FileResult(name, pc.size)
        with open(path, "rb") as f:
            rc, meta = ChunkFileMetaPage.decode(f.read(self.meta_size))
        sn = meta.sn if meta else 0
        if not os.path.exists(side):
            if self.create_missing:
                with open(side, "wb") as f:
                    f.write(encode_table(pc, self.page_bytes, sn))
                res.table = "created"
            return res
        try:
            with open(side, "rb") as f:
                page_bytes, _, want = decode_table(f.read())
            if page_bytes != self.page_bytes or want.size != pc.size:
                raise TableCorrupt("geometry")
        except TableCorrupt:
            res.table = "corrupt"
            return res
        bad = np.flatnonzero(want != pc)
        res.bad_pages = int(bad.size)
        res.first_bad = int(bad[0]) if bad.size else -1
        return res
