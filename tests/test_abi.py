"""The C-ABI library loads and exports every symbol include/*.h declares
(no compute calls that need a GPU)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


HOST_HEADERS = ("curve_integrity.h",)  # the host layer's C ABI: curve_amd/host/libcurvehost.so


def declared_symbols(host=False):
    """Functions a header declares: libcurvecrc's headers, or (host=True) the
    host layer's."""
    names = set()
    inc = os.path.join(ROOT, "include")
    for fn in os.listdir(inc):
        if not fn.endswith(".h") or (fn in HOST_HEADERS) != host:
            continue
        txt = open(os.path.join(inc, fn)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b([a-z_][a-z0-9_]*)\s*\(", txt, re.M):
            if m.group(1) not in ("if", "sizeof"):
                names.add(m.group(1))
    return names


def test_header_parses():
    names = declared_symbols()
    for must in ("crc32c_value", "crc32c_extend", "cc_page_crc_dev", "cc_page_verify_dev",
                 "cc_fold_dev", "cc_page_crc_host", "cc_engine_init", "cc_engine_fini"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from curve_amd import _lib
    L = _lib.lib()
    missing = [n for n in sorted(declared_symbols()) if not hasattr(L, n)]
    assert not missing, missing
    # and the python binding describes every one of them
    assert declared_symbols() <= set(_lib.SIGNATURES)


def test_host_library_exports_every_declared_symbol():
    """libcurvehost.so (the C++ IntegrityService's C ABI) loads beside
    libcurvecrc and exports what include/curve_integrity.h declares."""
    from curve_amd import _lib
    H = _lib.host_lib()
    names = declared_symbols(host=True)
    assert "cc_isvc_create" in names and "cc_isvc_wait" in names
    missing = [n for n in sorted(names) if not hasattr(H, n)]
    assert not missing, missing
    assert names <= set(_lib.HOST_SIGNATURES)


def test_no_gpu_fails_loudly_here():
    """Without a device the device entry points return CC_ENODEV (never a CPU fallback)."""
    from curve_amd import _lib
    L = _lib.lib()
    if L.cc_device_count() > 0:
        pytest.skip("a GPU is visible")
    buf = ctypes.create_string_buffer(4096)
    out = ctypes.create_string_buffer(4)
    assert L.cc_page_crc_dev(buf, 1, 4096, out, None) == _lib.CC_ENODEV
    assert L.cc_page_crc_host(buf, 1, 4096, out) == _lib.CC_ENODEV
    assert L.cc_engine_init(None) == _lib.CC_ENODEV
    paths = (ctypes.c_char_p * 1)(b"/nonexistent")
    res = (_lib.CcFileResult * 1)()
    assert L.cc_scan_files(paths, 1, 1 << 20, 4096, 4096, 4096, 2, None, res) == _lib.CC_ENODEV


def test_argument_checks_need_no_gpu():
    from curve_amd import _lib
    L = _lib.lib()
    buf = ctypes.create_string_buffer(4096)
    out = ctypes.create_string_buffer(4)
    assert L.cc_page_crc_dev(buf, 1, 100, out, None) == _lib.CC_EINVAL   # not a multiple of 256
    assert L.cc_page_crc_dev(buf, 1, 0, out, None) == _lib.CC_EINVAL
    assert L.cc_page_crc_dev(None, 1, 4096, out, None) == _lib.CC_EINVAL
    assert L.cc_page_crc_dev(buf, 0, 4096, out, None) == _lib.CC_OK       # empty batch is a no-op
    assert L.cc_lds_image(None, 0) == _lib.CC_EINVAL
    res = (_lib.CcFileResult * 1)()
    assert L.cc_scan_files(None, 1, 1 << 20, 4096, 4096, 4096, 2, None, res) == _lib.CC_EINVAL
    assert L.cc_scan_files(None, 0, 1 << 20, 4096, 4096, 4096, 2, None, res) == _lib.CC_OK
    assert L.cc_strerror(_lib.CC_ENODEV) == b"no usable HIP device"


def test_write_log_work_sizing_limits():
    """cc_apply_log_work_bytes (host arithmetic only): the caller's buffer holds
    a list link per piece and the insert blocks' head segments (the hash table is the
    engine's: >= 8 entries per piece in a power of two up to 2^32 slots, never
    fewer than 4 per piece), and a log whose table would need more than 2^32
    slots at 4 per piece (32-bit slot indices) is refused with 0, not truncated."""
    from curve_amd import _lib
    L = _lib.lib()
    small = L.cc_apply_log_work_bytes(65536, 4096, 4096)  # 2 pieces per write
    assert small >= 2 * 131072 * 4
    assert L.cc_apply_log_work_bytes(1 << 29, 4096, 4096) > 0          # 2^30 pieces -> 2^32 slots
    assert L.cc_apply_log_work_bytes((1 << 29) + 1, 4096, 4096) == 0   # would need 2^33 slots
    assert L.cc_apply_log_work_bytes(0, 4096, 4096) == 0
    assert L.cc_apply_log_work_bytes(10, 0, 4096) == 0
    # the buffer holds a 4-byte link per piece, the head segments (one per insert
    # block, each as long as the pieces of the 512-piece chunks that block takes:
    # at most 256 blocks, grid-stride beyond) and 256 segment counts
    for n, max_len in ((1, 1), (65536, 4096), (200000, 3 * 4096), (1 << 20, 4096)):
        pieces = n * ((max_len - 1) // 4096 + 2)
        chunks = -(-pieces // 512)
        segs = min(chunks, 256)
        cap = -(-chunks // segs) * 512
        need = L.cc_apply_log_work_bytes(n, max_len, 4096)
        assert need >= pieces * 4 + segs * cap * 8 + 256 * 4, (n, max_len, need)
        assert need <= pieces * 4 + segs * cap * 8 + 256 * 4 + 3 * 256, (n, max_len, need)


def test_default_io_threads_from_affinity_and_quota():
    """cc_default_io_threads (host arithmetic, no GPU): half the CPUs this
    process may use -- its affinity mask, capped by the cgroup v2 cpu.max quota
    -- within [2, 8]; scan_files(io_threads=0) uses it."""
    from curve_amd import _lib
    from curve_amd import crc as C
    cpus = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max" and int(q) // int(per) >= 1:
            cpus = min(cpus, int(q) // int(per))
    except (OSError, ValueError):
        pass
    want = min(8, max(2, cpus // 2))
    assert _lib.lib().cc_default_io_threads() == want == C.default_io_threads()


def test_log_probe_and_stream_entries_need_no_gpu():
    """The diagnostic entry points check their arguments before touching a
    device; with no context the engine holds no per-stream entries."""
    from curve_amd import _lib
    L = _lib.lib()
    assert L.cc_apply_log_probe_dev(None, 4096, None, None, 0, None, None) == _lib.CC_OK  # empty list
    assert L.cc_apply_log_probe_dev(None, 4096, None, None, 1, None, None) == _lib.CC_EINVAL
    buf = ctypes.create_string_buffer(8192)
    assert L.cc_apply_log_probe_dev(buf, 100, buf, buf, 1, buf, None) == _lib.CC_EINVAL  # pool not whole pages
    if L.cc_device_count() == 0:
        assert L.cc_engine_stream_entries() == 0


def test_log_queue_sizing_and_arguments_need_no_gpu():
    """cc_apply_logs_work_bytes (host arithmetic): two regions, each a link per
    piece plus head segments for either grouping -- the insert kernel's, or a
    page kernel's tail over <= 256 workgroups of <= 1024 threads taking up to
    twice their even share in takes of 2 chunks -- and 256 counts, then the
    three chunk counters;
    cc_apply_logs_dev checks its arguments before it needs a device."""
    import ctypes
    from curve_amd import _lib
    L = _lib.lib()
    for n, max_len in ((1, 1), (65536, 4096), (200000, 3 * 4096)):
        pieces = n * ((max_len - 1) // 4096 + 2)
        recs = 2 * (pieces + 1024 * 257) + (2 - 1) * 1024 * 256  # kGroupTake = 2
        region = -(-pieces * 4 // 256) * 256 + -(-recs * 8 // 256) * 256 + 1024
        assert L.cc_apply_logs_work_bytes(n, max_len, 4096) == 2 * region + 256, (n, max_len)
    assert L.cc_apply_logs_work_bytes(0, 4096, 4096) == 0
    assert L.cc_apply_logs_work_bytes(10, 0, 4096) == 0
    assert L.cc_apply_logs_work_bytes((1 << 29) + 1, 4096, 4096) == 0
    arr = (_lib.CcLogBatch * 1)()
    arr[0].n_updates = 3  # records but no pointers
    buf = ctypes.c_void_p(4096)
    assert L.cc_apply_logs_dev(None, 4096, 4096, None, 0, 4096, None, 0, None, 0, None) == _lib.CC_OK
    assert L.cc_apply_logs_dev(buf, 4096, 4096, None, 1, 4096, buf, 0, buf, 1 << 30, None) == _lib.CC_EINVAL
    assert L.cc_apply_logs_dev(buf, 4096, 4096, ctypes.cast(arr, ctypes.c_void_p), 1, 4096, buf, 0, buf, 1 << 30,
                               None) == _lib.CC_EINVAL
    assert L.cc_apply_logs_dev(buf, 4096, 1000, ctypes.cast(arr, ctypes.c_void_p), 1, 4096, buf, 0, buf, 1 << 30,
                               None) == _lib.CC_EINVAL  # page size
