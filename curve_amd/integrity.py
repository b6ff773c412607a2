"""Per-page CRC persistence + integrity jobs, Python mirror.

The product surface is libcurvecrc's C ABI (include/curve_crc.h, section
"Per-page CRC persistence": cc_pcrc_* codec / atomic store / load,
cc_integrity_check) and the C++ IntegrityService of the host layer
(curve_amd/host/integrity_service.h).  This module binds the same ABI for the
tests and tools; it does no checksum arithmetic of its own.

The reference computes no per-page data CRC and has nowhere to keep one (the
chunk metapage holds version/sn/correctedSn/location/bitmap + a header CRC,
chunkserver_chunkfile.cpp:64-88), so verify-on-read needs a NEW artefact: the
sidecar `<copyset dir>/pcrc/<chunk file name>.pcrc` -- deliberately NOT in the
data directory, because CopysetNode::GetHash (copyset_node.cpp:931-970) chains
every file listed there and a sidecar would change the copyset hash.  Layout:
curve_amd/csrc/integrity.cpp.  A table records the chunk's sn and the chunk
file's mtime / size when it was written; a table whose chunk changed since is
"stale" (refreshed by policy) and never condemns data, and a table that fails
its own CRCs is "corrupt".

Jobs mirror proto/integrity.proto (IntegrityService: ScheduleJob / CancelJob /
PauseJob / ResumeJob / ListJobs; IntegrityJob{id, copyset, state, progress,
sched_time, start_time}; INTEGRITY_JOB_STATE) -- declared and compiled in the
reference (proto/BUILD:78) with no implementation anywhere in src/.  A job walks
one copyset data directory in batches; each batch is one cc_integrity_check
call (native pread into pinned staging, every page rehashed on the GPU, compared
with its table).
"""
from __future__ import annotations

import ctypes
import enum
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from . import _lib
from . import crc as C
from ._lib import check, lib


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


def encode_table(page_crcs: np.ndarray, page_bytes: int, chunk_sn: int, data_mtime_ns: int = 0,
                 data_size: int = 0) -> bytes:
    """cc_pcrc_encode."""
    crcs = np.ascontiguousarray(page_crcs, dtype="<u4")
    h = _lib.CcPcrcHeader(page_bytes, crcs.size, chunk_sn, data_mtime_ns, data_size)
    out = ctypes.create_string_buffer(int(lib().cc_pcrc_encoded_bytes(crcs.size)))
    check(lib().cc_pcrc_encode(ctypes.byref(h), crcs.ctypes.data, out, len(out)), "cc_pcrc_encode")
    return out.raw


def decode_table(buf: bytes):
    """cc_pcrc_decode -> (header, page CRCs as uint32); TableCorrupt if bad."""
    h = _lib.CcPcrcHeader()
    rc = lib().cc_pcrc_decode(buf, len(buf), ctypes.byref(h), None, 0)
    if rc == _lib.CC_ECORRUPT:
        raise TableCorrupt("sidecar table fails its checks")
    check(rc, "cc_pcrc_decode")
    out = np.empty(h.n_pages, dtype=np.uint32)
    check(lib().cc_pcrc_decode(buf, len(buf), ctypes.byref(h), out.ctypes.data, out.size), "cc_pcrc_decode")
    return h, out


def table_dir_for(data_dir: str) -> str:
    """<copyset>/data -> <copyset>/pcrc (sibling of the data directory)."""
    return os.path.join(os.path.dirname(os.path.abspath(data_dir)), "pcrc")


def sidecar_path(chunk_path: str, table_dir: Optional[str] = None) -> str:
    d = table_dir or table_dir_for(os.path.dirname(os.path.abspath(chunk_path)))
    return os.path.join(d, os.path.basename(chunk_path) + ".pcrc")


def store_table(chunk_path: str, page_crcs, page_bytes: int = C.PAGE_SIZE, meta_bytes: int = C.META_PAGE_SIZE,
                table_path: Optional[str] = None) -> str:
    """cc_pcrc_store: persist the page CRCs of `chunk_path` (host array, or a
    device tensor -- e.g. the slice of a DevicePool's CRC table that
    cc_apply_log_delta_dev keeps current) after the write they describe."""
    if hasattr(page_crcs, "is_cuda"):
        page_crcs = page_crcs.detach().cpu().numpy()
    a = np.ascontiguousarray(page_crcs).view(np.uint32)
    path = table_path or sidecar_path(chunk_path)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    check(lib().cc_pcrc_store(os.fsencode(chunk_path), meta_bytes, os.fsencode(path), a.ctypes.data, a.size,
                              page_bytes), "cc_pcrc_store")
    return path


def load_table(table_path: str):
    """cc_pcrc_load -> (header, page CRCs)."""
    with open(table_path, "rb") as f:
        return decode_table(f.read())


@dataclass
class FileResult:
    name: str
    pages: int
    bad_pages: int = 0
    first_bad: int = -1
    table: str = "ok"          # ok | created | corrupt | stale | refreshed | missing | rebuilt
    status: int = 0
    bad_list: List[int] = field(default_factory=list)


def check_files(paths: List[str], table_paths: List[str], chunk_size: int = C.CHUNK_SIZE,
                meta_size: int = C.META_PAGE_SIZE, page_bytes: int = C.PAGE_SIZE, create_missing: bool = True,
                refresh_stale: bool = True, io_threads: int = 8, bad_cap: int = 4096) -> List[FileResult]:
    """cc_integrity_check over one batch of chunk files."""
    n = len(paths)
    if n == 0:
        return []
    cp = (ctypes.c_char_p * n)(*[os.fsencode(p) for p in paths])
    tp = (ctypes.c_char_p * n)(*[os.fsencode(p) for p in table_paths])
    o = _lib.CcIntegrityOpts(chunk_size, meta_size, page_bytes, io_threads, int(create_missing), int(refresh_stale))
    res = (_lib.CcIntegrityResult * n)()
    bad = np.zeros(max(1, bad_cap), dtype=np.uint64)
    nb = ctypes.c_uint64(0)
    check(lib().cc_integrity_check(cp, tp, n, ctypes.byref(o), res, bad.ctypes.data, bad_cap, ctypes.byref(nb)),
          "cc_integrity_check")
    out = [FileResult(os.path.basename(p), int(r.n_pages), int(r.bad_pages), int(r.first_bad),
                      _lib.TABLE_STATES.get(int(r.table_state), "?"), int(r.status)) for p, r in zip(paths, res)]
    for v in bad[:min(int(nb.value), bad_cap)].tolist():
        out[v >> 32].bad_list.append(v & 0xFFFFFFFF)
    return out


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


class IntegrityService:
    """In-process IntegrityService (ScheduleJob/CancelJob/PauseJob/ResumeJob/
    ListJobs), the Python twin of curve_amd/host/integrity_service.h.  One
    worker thread runs jobs FIFO; Pause/Cancel take effect at chunk-file batch
    boundaries.  Work happens on the calling process's current HIP device."""

    def __init__(self, chunk_size: int = C.CHUNK_SIZE, meta_size: int = C.META_PAGE_SIZE,
                 page_bytes: int = C.PAGE_SIZE, batch: int = 16, create_missing: bool = True,
                 refresh_stale: bool = True):
        self.chunk_size, self.meta_size, self.page_bytes = chunk_size, meta_size, page_bytes
        self.batch, self.create_missing, self.refresh_stale = batch, create_missing, refresh_stale
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
        tdir = table_dir_for(job.data_dir)
        os.makedirs(tdir, exist_ok=True)
        done = {r.name for r in job.results}
        todo = [n for n in names if n not in done]
        for b0 in range(0, len(todo), self.batch):
            with self._cv:
                if job.state != IntegrityJobState.RUNNING:  # paused or canceled at a batch boundary
                    self._cv.notify_all()
                    return
            part = todo[b0:b0 + self.batch]
            paths = [os.path.join(job.data_dir, n) for n in part]
            res = check_files(paths, [sidecar_path(p, tdir) for p in paths], self.chunk_size, self.meta_size,
                              self.page_bytes, self.create_missing, self.refresh_stale)
            bad = [r for r in res if r.status]
            if bad:
                raise IOError(f"cannot check {bad[0].name}: status {bad[0].status}")
            job.results.extend(res)
            with self._cv:
                job.progress = int(100 * len(job.results) / max(1, len(names)))
        with self._cv:
            if job.state == IntegrityJobState.RUNNING:
                job.state, job.progress = IntegrityJobState.FINISHED, 100
            self._cv.notify_all()
