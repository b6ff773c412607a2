"""ctypes binding of libcurvecrc.so (include/curve_crc.h).

The library is built in-tree (curve_amd/libcurvecrc.so, `make -C curve_amd/csrc`)
and loaded from there; if it is missing, importing any device entry point raises
-- there is deliberately no CPU fallback for the device path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
# $CURVE_AMD_LIB / $CURVE_AMD_HOST_LIB name another build of the same libraries
# (scripts/sanitize.sh runs the CPU suite on ASan/UBSan builds)
LIB_PATH = os.environ.get("CURVE_AMD_LIB") or os.path.join(_HERE, "libcurvecrc.so")
CSRC = os.path.join(_HERE, "csrc")

CC_OK = 0
CC_EINVAL = -22
CC_ENODEV = -19
CC_ENOMEM = -12
CC_EHIP = -5
CC_ECORRUPT = -74
CC_ECOMM = -71
CC_EIO = -5001
CC_ESTALE = -116
CC_ETIMEDOUT = -110
CC_EFORMAT = -5002
CC_ENOENT = -2
CC_COMM_ID_BYTES = 128

# every symbol include/curve_crc.h declares: (name, restype, argtypes)
_u32, _u64, _sz, _vp, _int = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int


class CcOpts(ctypes.Structure):
    _fields_ = [("page_bytes", _u32), ("slice_bytes", _u32), ("staging_bytes", _u64)]


class CcFileResult(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("meta_crc", _u32), ("file_crc", _u32), ("reserved", _u32)]


class CcChunkSrc(ctypes.Structure):
    _fields_ = [("meta", _vp), ("data", _vp)]


class CcScanDigest(ctypes.Structure):  # include/curve_crc.h cc_scan_digest
    _fields_ = [("h_after_bytes", _vp), ("h_group", _vp), ("n_groups", _u64), ("h_digest", _vp)]


class IoVec(ctypes.Structure):  # struct iovec
    _fields_ = [("iov_base", _vp), ("iov_len", _sz)]


class CcPcrcHeader(ctypes.Structure):  # include/curve_crc.h cc_pcrc_header
    _fields_ = [("page_bytes", _u32), ("n_pages", _u32), ("chunk_sn", _u64), ("data_mtime_ns", ctypes.c_int64),
                ("data_size", _u64), ("stamp_ns", ctypes.c_int64)]


class CcIntegrityOpts(ctypes.Structure):
    _fields_ = [("chunk_bytes", _u32), ("meta_bytes", _u32), ("page_bytes", _u32), ("io_threads", _u32),
                ("create_missing", _u32), ("refresh_stale", _u32)]


class CcIntegrityResult(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("table_state", _u32), ("n_pages", _u32), ("bad_pages", _u32),
                ("first_bad", ctypes.c_int64)]


CC_PCRC_HEADER_BYTES = 64
TABLE_STATES = {0: "ok", 1: "created", 2: "corrupt", 3: "stale", 4: "refreshed", 5: "missing", 6: "rebuilt"}


class CcLogBatch(ctypes.Structure):
    """cc_log_batch (include/curve_crc.h): one write log of a cc_apply_logs_dev queue."""
    _fields_ = [("d_src", ctypes.c_void_p), ("d_log", ctypes.c_void_p), ("n_updates", ctypes.c_uint64)]


class CcPoolShard(ctypes.Structure):  # include/curve_crc.h cc_pool_shard
    _fields_ = [("d_data", _vp), ("d_meta", _vp), ("n_chunks", _u64), ("chunk_bytes", _u32),
                ("meta_bytes", _u32), ("page_bytes", _u32), ("slice_bytes", _u32), ("d_after_mult", _vp),
                ("d_group", _vp), ("n_groups", _u64), ("d_page_crcs", _vp), ("d_meta_crcs", _vp),
                ("d_slice_crcs", _vp), ("d_file_crcs", _vp), ("d_digest", _vp), ("ev_pages_begin", _vp),
                ("ev_pages_end", _vp), ("ev_exchange_begin", _vp), ("ev_exchange_end", _vp)]


SIGNATURES = {
    "crc32c_value": (_u32, [_vp, _sz]),
    "crc32c_extend": (_u32, [_u32, _vp, _sz]),
    "crc32c_combine": (_u32, [_u32, _u32, _u64]),
    "crc32c_shift": (_u32, [_u32, _u64]),
    "crc32c_zeros": (_u32, [_u64]),
    "cc_fold_host": (_u32, [_vp, _u64, _u64]),
    "crc32c_extend_iov": (_u32, [_u32, _vp, _sz]),
    "cc_slice_fold": (_int, [_vp, _u64, _u32, _u32, _vp]),
    "cc_crc_bufs_host": (_int, [_vp, _vp, _u64, _vp]),
    "cc_digest_fold_dev": (_int, [_vp, _u32, _u64, _vp, _vp]),
    "cc_scan_host_digest": (_int, [ctypes.POINTER(CcChunkSrc), _u64, _u32, _u32, _u32, _u32, _vp, _vp, _vp,
                                   ctypes.POINTER(CcScanDigest)]),
    "cc_engine_init": (_int, [ctypes.POINTER(CcOpts)]),
    "cc_engine_fini": (_int, []),
    "cc_engine_trim": (_int, []),
    "cc_device_count": (_int, []),
    "cc_strerror": (ctypes.c_char_p, [_int]),
    "cc_version": (ctypes.c_char_p, []),
    "cc_page_crc_dev": (_int, [_vp, _u64, _u32, _vp, _vp]),
    "cc_page_verify_dev": (_int, [_vp, _u64, _u32, _vp, _vp, _vp, _vp]),
    "cc_hbm_read_probe_dev": (_int, [_vp, _u64, _vp, _vp]),
    "cc_page_load_probe_dev": (_int, [_vp, _u64, _vp, _vp]),
    "cc_page_verify_list_dev": (_int, [_vp, _u64, _u32, _vp, _vp, _vp, _vp, _u64, _vp]),
    "cc_fold_dev": (_int, [_vp, _u64, _u32, _u64, _vp, _vp]),
    "cc_shift_dev": (_int, [_vp, _vp, _u64, _vp, _vp]),
    "cc_crc_ranges_dev": (_int, [_vp, _vp, _u64, _vp, _vp]),
    "cc_xpow8_dev": (_int, [_vp, _u64, _vp, _vp]),
    "cc_scan_epilogue_dev": (_int, [_vp, _vp, _u64, _u32, _u32, _u32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "cc_combine_dev": (_int, [_vp, _vp, _u64, _u64, _vp, _vp]),
    "cc_digest_dev": (_int, [_vp, _vp, _vp, _u64, _vp, _vp]),
    "cc_page_crc_host": (_int, [_vp, _u64, _u32, _vp]),
    "cc_lds_image": (_int, [_vp, _sz]),
    "cc_scan_files": (_int, [ctypes.POINTER(ctypes.c_char_p), _u64, _u32, _u32, _u32, _u32, _u32, _vp,
                              ctypes.POINTER(CcFileResult)]),
    "cc_default_io_threads": (_u32, []),
    "cc_scan_host": (_int, [ctypes.POINTER(CcChunkSrc), _u64, _u32, _u32, _u32, _u32, _vp, _vp, _vp]),
    "cc_apply_log_work_bytes": (_u64, [_u64, _u32, _u32]),
    "cc_apply_log_dev": (_int, [_vp, _u64, _u32, _vp, _vp, _u64, _u32, _vp, _vp, _u64, _vp]),
    "cc_apply_log_delta_dev": (_int, [_vp, _u64, _u32, _vp, _vp, _u64, _u32, _vp, _vp, _u64, _vp]),
    "cc_engine_stream_entries": (_u64, []),
    "cc_apply_log_probe_dev": (_int, [_vp, _u64, _vp, _vp, _u64, _vp, _vp]),
    "cc_apply_logs_work_bytes": (_u64, [_u64, _u32, _u32]),
    "cc_page_list_probe_dev": (_int, [_vp, _u64, _vp, _u64, _vp, _vp]),
    "cc_apply_logs_dev": (_int, [_vp, _u64, _u32, _vp, _u32, _u32, _vp, _int, _vp, _u64, _vp]),
    "cc_verify_reads_work_bytes": (_u64, [_u64]),
    "cc_verify_reads_dev": (_int, [_vp, _u64, _u32, _vp, _u64, _vp, _vp, _vp, _vp, _u64, _vp]),
    "cc_comm_unique_id": (_int, [_vp, _sz]),
    "cc_comm_init": (_int, [ctypes.POINTER(_vp), _int, _int, _vp, _sz]),
    "cc_comm_init_timeout": (_int, [ctypes.POINTER(_vp), _int, _int, _vp, _sz, _u32]),
    "cc_comm_destroy": (_int, [_vp]),
    "cc_comm_abort": (_int, [_vp]),
    "cc_comm_size": (_int, [_vp]),
    "cc_comm_rank": (_int, [_vp]),
    "cc_comm_wait": (_int, [_vp, _vp, _u32]),
    "cc_digest_allreduce_dev": (_int, [_vp, _vp, _u64, _vp]),
    "cc_pool_scan_dev": (_int, [ctypes.POINTER(CcPoolShard), _vp, _vp]),
    "cc_pcrc_encoded_bytes": (_u64, [_u32]),
    "cc_pcrc_encode": (_int, [ctypes.POINTER(CcPcrcHeader), _vp, _vp, _u64]),
    "cc_pcrc_decode": (_int, [_vp, _u64, ctypes.POINTER(CcPcrcHeader), _vp, _u32]),
    "cc_chunk_meta_sn": (_int, [_vp, _u32, ctypes.POINTER(_u64)]),
    "cc_pcrc_store": (_int, [ctypes.c_char_p, _u32, ctypes.c_char_p, _vp, _u32, _u32]),
    "cc_pcrc_load": (_int, [ctypes.c_char_p, ctypes.POINTER(CcPcrcHeader), _vp, _u32]),
    "cc_pcrc_store_expect": (_int, [ctypes.c_char_p, _u32, ctypes.c_char_p, _vp, _u32, _u32,
                                    ctypes.POINTER(CcPcrcHeader)]),
    "cc_pcrc_is_racy": (_int, [ctypes.POINTER(CcPcrcHeader)]),
    "cc_integrity_check": (_int, [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_char_p), _u64,
                                  ctypes.POINTER(CcIntegrityOpts), ctypes.POINTER(CcIntegrityResult), _vp, _u64,
                                  ctypes.POINTER(_u64)]),
}

# ---- the host layer's C ABI (include/curve_integrity.h, curve_amd/host/libcurvehost.so)
HOST_LIB_PATH = os.environ.get("CURVE_AMD_HOST_LIB") or os.path.join(_HERE, "host", "libcurvehost.so")


class CcIsvcOpts(ctypes.Structure):
    _fields_ = [("chunk_bytes", _u32), ("meta_bytes", _u32), ("page_bytes", _u32), ("batch", _u32),
                ("io_threads", _u32), ("create_missing", _u32), ("refresh_stale", _u32)]


class CcIsvcJob(ctypes.Structure):
    _fields_ = [("id", ctypes.c_int32), ("copyset", ctypes.c_int32), ("state", ctypes.c_int32),
                ("progress", ctypes.c_int32), ("sched_time", ctypes.c_int32), ("start_time", ctypes.c_int32),
                ("n_results", _u64), ("error", ctypes.c_char * 256)]


class CcIsvcFile(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 256), ("status", ctypes.c_int32), ("table_state", _u32),
                ("bad_pages", _u32), ("n_bad_listed", _u32), ("first_bad", ctypes.c_int64)]


HOST_SIGNATURES = {
    "cc_isvc_create": (_vp, [ctypes.POINTER(CcIsvcOpts)]),
    "cc_isvc_destroy": (None, [_vp]),
    "cc_isvc_schedule": (_int, [_vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p]),
    "cc_isvc_cancel": (_int, [_vp, ctypes.c_int32]),
    "cc_isvc_pause": (_int, [_vp, ctypes.c_int32]),
    "cc_isvc_resume": (_int, [_vp, ctypes.c_int32]),
    "cc_isvc_list": (_int, [_vp, _vp, _u64, ctypes.POINTER(_u64)]),
    "cc_isvc_job_info": (_int, [_vp, ctypes.c_int32, ctypes.POINTER(CcIsvcJob)]),
    "cc_isvc_file_result": (_int, [_vp, ctypes.c_int32, _u64, ctypes.POINTER(CcIsvcFile), _vp, _u64]),
    "cc_isvc_wait": (_int, [_vp, ctypes.c_int32, ctypes.c_int32]),
}

_lib = None
_host = None


def _one_hip_runtime():
    """Load torch (if present) BEFORE libcurvecrc: torch's wheel carries its own
    libamdhip64.so.7 / libhsa-runtime64 and loads them by path, so a process
    that loaded /opt/rocm's first (through libcurvecrc) ends up with TWO HIP
    runtimes, and the one libcurvecrc bound to finds no usable device
    (CC_ENODEV on every call; scripts/load_order_probe.py).  With torch first,
    libcurvecrc's libamdhip64.so.7 resolves to the runtime already loaded."""
    try:
        import torch  # noqa: F401
    except Exception:  # absent, or a broken install (OSError / RuntimeError at import): the plain load order
        pass


def host_lib():
    """libcurvehost.so (the C++ IntegrityService behind include/curve_integrity.h)."""
    global _host
    if _host is None:
        lib()  # libcurvecrc first (the host library links it)
        if not os.path.exists(HOST_LIB_PATH):
            raise OSError(f"{HOST_LIB_PATH} missing: build it with `make -C {os.path.join(_HERE, 'host')}`")
        H = ctypes.CDLL(HOST_LIB_PATH)
        for name, (res, args) in HOST_SIGNATURES.items():
            f = getattr(H, name)
            f.restype = res
            f.argtypes = args
        _host = H
    return _host


class CurveCrcError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = _lib.cc_strerror(code).decode() if _lib is not None else str(code)
        super().__init__(f"{what}: {msg} ({code})" if what else f"{msg} ({code})")


def build(arch: str = "gfx950") -> str:
    subprocess.run(["make", "-s", "-C", CSRC, f"ARCH={arch}"], check=True)
    return LIB_PATH


def lib():
    """The loaded libcurvecrc; raises OSError (loudly) if it was never built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} missing: build it with `make -C {CSRC}` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
        _one_hip_runtime()
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != CC_OK:
        raise CurveCrcError(rc, what)
