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
reference (proto/BUILD:78) with no implementation anywhere in src/.  The
service is the C++ one (curve_amd/host/integrity_service.cpp) behind
include/curve_integrity.h; `IntegrityService` below is a ctypes facade over it.
A job walks one copyset data directory in batches; each batch is one
cc_integrity_check call (native pread into pinned staging, every page rehashed
on the GPU, compared with its table).  A chunk's own failure (metapage header
CRC, deleted mid-job) is that file's result; only a failing batch call fails
the job.
"""
from __future__ import annotations

import ctypes
import enum
import os
from dataclasses import dataclass, field
from typing import List, Optional

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
                refresh_stale: bool = True, io_threads: int = 0, bad_cap: int = 4096) -> List[FileResult]:
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
    state: IntegrityJobState = IntegrityJobState.WAITING
    progress: int = 0          # percent of chunk files done
    sched_time: int = 0
    start_time: int = 0
    results: List[FileResult] = field(default_factory=list)
    error: str = ""


class IntegrityService:
    """IntegrityService (ScheduleJob / CancelJob / PauseJob / ResumeJob /
    ListJobs) -- a ctypes facade over the C++ service of the host layer
    (curve_amd/host/integrity_service.h through include/curve_integrity.h,
    libcurvehost.so).  The job state machine, its worker thread and its
    batches live in C++ only; this class converts arguments and results.
    Work happens on the process's current HIP device."""

    def __init__(self, chunk_size: int = C.CHUNK_SIZE, meta_size: int = C.META_PAGE_SIZE,
                 page_bytes: int = C.PAGE_SIZE, batch: int = 16, create_missing: bool = True,
                 refresh_stale: bool = True, io_threads: int = 0):
        self._H = _lib.host_lib()
        o = _lib.CcIsvcOpts(chunk_size, meta_size, page_bytes, batch, io_threads, int(create_missing),
                            int(refresh_stale))
        self._s = self._H.cc_isvc_create(ctypes.byref(o))
        if not self._s:
            raise C.CurveCrcError(_lib.CC_EINVAL, "cc_isvc_create")
        self.page_bytes, self.pages = page_bytes, chunk_size // page_bytes

    # -- RPC surface -----------------------------------------------------
    def ScheduleJob(self, job_id: int, copyset: int, data_dir: str) -> IntegrityOpStatus:
        return IntegrityOpStatus(self._H.cc_isvc_schedule(self._s, job_id, copyset, os.fsencode(data_dir)))

    def CancelJob(self, job_id: int) -> IntegrityOpStatus:
        return IntegrityOpStatus(self._H.cc_isvc_cancel(self._s, job_id))

    def PauseJob(self, job_id: int) -> IntegrityOpStatus:
        return IntegrityOpStatus(self._H.cc_isvc_pause(self._s, job_id))

    def ResumeJob(self, job_id: int) -> IntegrityOpStatus:
        return IntegrityOpStatus(self._H.cc_isvc_resume(self._s, job_id))

    def ListJobs(self) -> List[IntegrityJob]:
        n = ctypes.c_uint64(0)
        check(self._H.cc_isvc_list(self._s, None, 0, ctypes.byref(n)), "cc_isvc_list")
        ids = (ctypes.c_int32 * max(1, n.value))()
        check(self._H.cc_isvc_list(self._s, ids, n.value, ctypes.byref(n)), "cc_isvc_list")
        return [self.job(int(ids[k])) for k in range(min(n.value, len(ids)))]

    def job(self, job_id: int) -> IntegrityJob:
        info = _lib.CcIsvcJob()
        check(self._H.cc_isvc_job_info(self._s, job_id, ctypes.byref(info)), "cc_isvc_job_info")
        j = IntegrityJob(info.id, info.copyset, IntegrityJobState(info.state), info.progress, info.sched_time,
                         info.start_time, error=info.error.decode(errors="replace"))
        f = _lib.CcIsvcFile()
        for k in range(info.n_results):
            check(self._H.cc_isvc_file_result(self._s, job_id, k, ctypes.byref(f), None, 0), "cc_isvc_file_result")
            bad = np.zeros(max(1, f.n_bad_listed), dtype=np.uint32)
            check(self._H.cc_isvc_file_result(self._s, job_id, k, ctypes.byref(f), bad.ctypes.data, bad.size),
                  "cc_isvc_file_result")
            j.results.append(FileResult(f.name.decode(errors="replace"), self.pages, int(f.bad_pages), int(f.first_bad),
                                        _lib.TABLE_STATES.get(int(f.table_state), "?"), int(f.status),
                                        bad[:f.n_bad_listed].tolist()))
        return j

    def wait(self, job_id: int, timeout: float = 60.0) -> IntegrityJob:
        rc = self._H.cc_isvc_wait(self._s, job_id, int(timeout * 1000))
        if rc < 0:
            raise C.CurveCrcError(rc, "cc_isvc_wait")
        return self.job(job_id)

    def close(self):
        if self._s:
            s, self._s = self._s, None
            self._H.cc_isvc_destroy(s)

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass
