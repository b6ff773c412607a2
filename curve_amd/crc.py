"""Host-side mirror of the reference's CRC32C surface.

`CRC32` mirrors curve::common::CRC32 (src/common/crc32.h:40-55): the two
overloads become one function with an optional leading `crc`.  Device batch
operations work on torch CUDA tensors (device memory + the current stream are
plumbing; the compute is libcurvecrc's HIP kernels) and raise `CurveCrcError`
on any failure -- there is no CPU fallback for them.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Union

from . import _lib
from ._lib import CurveCrcError, check, lib

PAGE_SIZE = 4096                # conf/chunkserver.conf:22 (blocksize / page)
CHUNK_SIZE = 16 * 1024 * 1024   # conf/chunkserver.conf:13
META_PAGE_SIZE = 4096           # conf/chunkserver.conf:16
SCAN_SIZE = 4 * 1024 * 1024     # conf/chunkserver.conf:114


def _host_buf(data):
    if isinstance(data, (bytes, bytearray)):
        b = bytes(data)
        return ctypes.c_char_p(b), len(b), b
    if isinstance(data, memoryview):
        b = data.tobytes()
        return ctypes.c_char_p(b), len(b), b
    try:  # numpy array
        import numpy as np
        if isinstance(data, np.ndarray):
            a = np.ascontiguousarray(data)
            return ctypes.c_void_p(a.ctypes.data), a.nbytes, a
    except ImportError:  # pragma: no cover
        pass
    if isinstance(data, str):
        b = data.encode()
        return ctypes.c_char_p(b), len(b), b
    raise TypeError(f"unsupported buffer type {type(data)!r}")


def CRC32(*args) -> int:
    """CRC32(data) == curve::common::CRC32(pData, iLen)           (crc32.h:40-42)
       CRC32(crc, data) == curve::common::CRC32(crc, pData, iLen)  (crc32.h:53-55)
    CPU primitive for small buffers (metapage headers, conf-epoch, ...)."""
    if len(args) == 1:
        crc, data = 0, args[0]
    elif len(args) == 2:
        crc, data = args
    else:
        raise TypeError("CRC32(data) or CRC32(crc, data)")
    p, n, _keep = _host_buf(data)
    return int(lib().crc32c_extend(int(crc) & 0xFFFFFFFF, p, n))


def CRC32_iov(fragments, crc: int = 0) -> int:
    """crc32c_extend_iov: one CRC over a scattered buffer, as braft::crc32(const
    butil::IOBuf&) extends it across the IOBuf's blocks (raftlog/curve_segment.cpp:405)."""
    keep = [_host_buf(f) for f in fragments]
    iov = (_lib.IoVec * max(1, len(keep)))()
    for i, (p, n, _k) in enumerate(keep):
        iov[i].iov_base = ctypes.cast(p, ctypes.c_void_p).value if n else None
        iov[i].iov_len = n
    return int(lib().crc32c_extend_iov(int(crc) & 0xFFFFFFFF, iov, len(keep)))


def slice_fold(page_crcs, pages_per_slice: int, page_bytes: int = PAGE_SIZE):
    """cc_slice_fold: page CRCs -> one CRC per slice of pages_per_slice pages (host)."""
    import numpy as np
    a = np.ascontiguousarray(page_crcs, dtype=np.uint32)
    if pages_per_slice <= 0 or a.size % pages_per_slice:
        raise CurveCrcError(_lib.CC_EINVAL, "page count is not a multiple of pages_per_slice")
    out = np.empty(a.size // pages_per_slice, dtype=np.uint32)
    check(lib().cc_slice_fold(ctypes.c_void_p(a.ctypes.data), a.size, pages_per_slice, page_bytes,
                              ctypes.c_void_p(out.ctypes.data)), "cc_slice_fold")
    return out


def crc_bufs_host(bufs):
    """cc_crc_bufs_host: CRC32 of every host buffer in one blocking device call."""
    import numpy as np
    keep = [_host_buf(b) for b in bufs]
    n = len(keep)
    ptrs = (ctypes.c_void_p * max(1, n))(*[ctypes.cast(p, ctypes.c_void_p).value for p, _, _ in keep])
    lens = np.array([k[1] for k in keep], dtype=np.uint64)
    out = np.empty(n, dtype=np.uint32)
    check(lib().cc_crc_bufs_host(ptrs, ctypes.c_void_p(lens.ctypes.data), n, ctypes.c_void_p(out.ctypes.data)),
          "cc_crc_bufs_host")
    return out


def combine(crc_a: int, crc_b: int, len_b: int) -> int:
    return int(lib().crc32c_combine(crc_a & 0xFFFFFFFF, crc_b & 0xFFFFFFFF, int(len_b)))


def shift(crc: int, nbytes: int) -> int:
    return int(lib().crc32c_shift(crc & 0xFFFFFFFF, int(nbytes)))


def zeros(nbytes: int) -> int:
    return int(lib().crc32c_zeros(int(nbytes)))


def fold_host(page_crcs, page_bytes: int) -> int:
    import numpy as np
    a = np.ascontiguousarray(page_crcs, dtype=np.uint32)
    return int(lib().cc_fold_host(ctypes.c_void_p(a.ctypes.data), a.size, int(page_bytes)))


def device_count() -> int:
    return int(lib().cc_device_count())


def engine_init(page_bytes: int = 0, slice_bytes: int = 0, staging_bytes: int = 0) -> None:
    o = _lib.CcOpts(page_bytes, slice_bytes, staging_bytes)
    check(lib().cc_engine_init(ctypes.byref(o)), "cc_engine_init")


def engine_fini() -> None:
    check(lib().cc_engine_fini(), "cc_engine_fini")


# ---------------------------------------------------------------------------
# device batch operations (torch tensors as device-memory handles)
# ---------------------------------------------------------------------------
def _torch():
    import torch
    return torch


def _stream_handle(stream) -> Optional[int]:
    torch = _torch()
    if stream is None:
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


def _on_stream(stream):
    """Context in which tensors are created on `stream` (the stream the native
    call enqueues on), so an output's initialisation (torch.full / zeros) is
    ordered before the kernel that writes it."""
    import contextlib
    torch = _torch()
    return torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()


def _stream_key(device, stream):
    """Cache key of per-stream scratch: (device, HIP stream handle)."""
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return (device, s.cuda_stream)


def _dev_ptr(t, what: str):
    if not t.is_cuda:
        raise CurveCrcError(_lib.CC_EINVAL, f"{what} must be a device tensor")
    if not t.is_contiguous():
        raise CurveCrcError(_lib.CC_EINVAL, f"{what} must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


def _nbytes(t) -> int:
    return t.numel() * t.element_size()


def page_crc(pages, page_bytes: int = PAGE_SIZE, out=None, stream=None):
    """CRC32C of every `page_bytes` page of the device tensor `pages` (any dtype,
    contiguous, size a multiple of page_bytes) -> int32 tensor of CRC bits
    (uint32 values viewed as int32; `.view(torch.uint32)` / `& 0xFFFFFFFF` to read)."""
    torch = _torch()
    nb = _nbytes(pages)
    if nb % page_bytes:
        raise CurveCrcError(_lib.CC_EINVAL, "pages size is not a multiple of page_bytes")
    n = nb // page_bytes
    if out is None:
        with _on_stream(stream):  # created on the stream the kernel writes it on
            out = torch.empty(n, dtype=torch.int32, device=pages.device)
    elif out.numel() < n or out.element_size() != 4:
        raise CurveCrcError(_lib.CC_EINVAL, "out too small or not 32-bit")
    with torch.cuda.device(pages.device):
        check(lib().cc_page_crc_dev(_dev_ptr(pages, "pages"), n, page_bytes, _dev_ptr(out, "out"),
                                    _stream_handle(stream)), "cc_page_crc_dev")
    return out


def page_verify(pages, expected, page_bytes: int = PAGE_SIZE, stream=None, counters=None):
    """Recompute and compare.  Returns a 2-element int64 device tensor
    [bad_count, first_bad] (first_bad = 2^64-1 -> -1 when clean); no host sync."""
    torch = _torch()
    nb = _nbytes(pages)
    if nb % page_bytes:
        raise CurveCrcError(_lib.CC_EINVAL, "pages size is not a multiple of page_bytes")
    n = nb // page_bytes
    if expected.numel() < n or expected.element_size() != 4:
        raise CurveCrcError(_lib.CC_EINVAL, "expected must hold one 32-bit CRC per page")
    if counters is None:
        with _on_stream(stream):
            counters = torch.tensor([0, -1], dtype=torch.int64, device=pages.device)
    base = counters.data_ptr()
    with torch.cuda.device(pages.device):
        check(lib().cc_page_verify_dev(_dev_ptr(pages, "pages"), n, page_bytes, _dev_ptr(expected, "expected"),
                                       ctypes.c_void_p(base), ctypes.c_void_p(base + 8),
                                       _stream_handle(stream)), "cc_page_verify_dev")
    return counters


def hbm_read_probe(buf, sink, stream=None):
    """cc_hbm_read_probe_dev (diagnostic): pure nt read of `buf`; sink must hold
    2*CUs*16 int32."""
    check(lib().cc_hbm_read_probe_dev(_dev_ptr(buf, "buf"), _nbytes(buf), _dev_ptr(sink, "sink"),
                                      _stream_handle(stream)), "cc_hbm_read_probe_dev")


def page_load_probe(pages, out, stream=None):
    """cc_page_load_probe_dev (diagnostic): the page kernel's schedule and
    traffic over the 4 KiB pages of `pages` without the CRC arithmetic; `out`
    (one int32 per page) receives meaningless words."""
    n = _nbytes(pages) // PAGE_SIZE
    if out.numel() < n or out.element_size() != 4:
        raise CurveCrcError(_lib.CC_EINVAL, "out too small or not 32-bit")
    check(lib().cc_page_load_probe_dev(_dev_ptr(pages, "pages"), n, _dev_ptr(out, "out"), _stream_handle(stream)),
          "cc_page_load_probe_dev")


def page_verify_list(pages, expected, page_bytes: int = PAGE_SIZE, max_bad: int = 4096, stream=None):
    """cc_page_verify_list_dev: -> (counters [bad_count, first_bad] int64 device
    tensor, bad page indices int64 device tensor of max_bad slots; the first
    min(bad_count, max_bad) are valid, unordered).  No host sync."""
    torch = _torch()
    nb = _nbytes(pages)
    if nb % page_bytes:
        raise CurveCrcError(_lib.CC_EINVAL, "pages size is not a multiple of page_bytes")
    n = nb // page_bytes
    if expected.numel() < n or expected.element_size() != 4:
        raise CurveCrcError(_lib.CC_EINVAL, "expected must hold one 32-bit CRC per page")
    with _on_stream(stream):
        counters = torch.tensor([0, -1], dtype=torch.int64, device=pages.device)
        bad = torch.full((max(1, max_bad),), -1, dtype=torch.int64, device=pages.device)
    base = counters.data_ptr()
    with torch.cuda.device(pages.device):
        check(lib().cc_page_verify_list_dev(_dev_ptr(pages, "pages"), n, page_bytes, _dev_ptr(expected, "expected"),
                                            ctypes.c_void_p(base), ctypes.c_void_p(base + 8),
                                            ctypes.c_void_p(bad.data_ptr()), max_bad,
                                            _stream_handle(stream)), "cc_page_verify_list_dev")
    return counters, bad


def fold(crcs, per_group: int, unit_bytes: int, out=None, stream=None):
    """Group fold on device: out[g] = CRC of the concatenation of `per_group`
    consecutive units (each `unit_bytes`) given their CRCs."""
    torch = _torch()
    n = crcs.numel()
    if per_group <= 0 or n % per_group:
        raise CurveCrcError(_lib.CC_EINVAL, "crcs count is not a multiple of per_group")
    g = n // per_group
    if out is None:
        with _on_stream(stream):  # created on the stream the kernel writes it on
            out = torch.empty(g, dtype=torch.int32, device=crcs.device)
    with torch.cuda.device(crcs.device):
        check(lib().cc_fold_dev(_dev_ptr(crcs, "crcs"), g, per_group, int(unit_bytes), _dev_ptr(out, "out"),
                                _stream_handle(stream)), "cc_fold_dev")
    return out


def shift_dev(crcs, shift_bytes, out=None, stream=None):
    """out[i] = shift(crcs[i], shift_bytes[i]) on device (int64 shift counts)."""
    torch = _torch()
    n = crcs.numel()
    if shift_bytes.numel() != n or shift_bytes.element_size() != 8:
        raise CurveCrcError(_lib.CC_EINVAL, "shift_bytes must be int64, one per crc")
    if out is None:
        with _on_stream(stream):  # created on the stream the kernel writes it on
            out = torch.empty(n, dtype=torch.int32, device=crcs.device)
    with torch.cuda.device(crcs.device):
        check(lib().cc_shift_dev(_dev_ptr(crcs, "crcs"), _dev_ptr(shift_bytes, "shift_bytes"), n,
                                 _dev_ptr(out, "out"), _stream_handle(stream)), "cc_shift_dev")
    return out


def crc_ranges(buf, offsets, lengths, out=None, stream=None):
    """CRC32C (Value) of arbitrary byte ranges of the device tensor `buf`
    (cc_crc_ranges_dev) -> int32 device tensor."""
    import numpy as np
    torch = _torch()
    offs = np.asarray(offsets, dtype=np.uint64)
    lens = np.asarray(lengths, dtype=np.uint64)
    if offs.size != lens.size:
        raise CurveCrcError(_lib.CC_EINVAL, "offsets / lengths mismatch")
    if (offs + lens > _nbytes(buf)).any():
        raise CurveCrcError(_lib.CC_EINVAL, "range beyond the buffer")
    rec = np.empty((offs.size, 2), dtype=np.uint64)
    rec[:, 0], rec[:, 1] = offs, lens
    with _on_stream(stream):
        d_rec = torch.from_numpy(rec.view(np.uint8).reshape(-1)).to(buf.device)
        if out is None:
            out = torch.empty(offs.size, dtype=torch.int32, device=buf.device)
    with torch.cuda.device(buf.device):
        check(lib().cc_crc_ranges_dev(_dev_ptr(buf, "buf"), _dev_ptr(d_rec, "ranges"), offs.size,
                                      _dev_ptr(out, "out"), _stream_handle(stream)), "cc_crc_ranges_dev")
    if stream is not None:
        d_rec.record_stream(stream)
    return out


def xpow8(nbytes, out=None, stream=None):
    """x^(8*n) mod P per element (cc_xpow8_dev): the shift multipliers of a static layout."""
    torch = _torch()
    if out is None:
        with _on_stream(stream):  # created on the stream the kernel writes it on
            out = torch.empty(nbytes.numel(), dtype=torch.int32, device=nbytes.device)
    with torch.cuda.device(nbytes.device):
        check(lib().cc_xpow8_dev(_dev_ptr(nbytes, "nbytes"), nbytes.numel(), _dev_ptr(out, "out"),
                                 _stream_handle(stream)), "cc_xpow8_dev")
    return out


def scan_epilogue(page_crcs, meta_crcs, n_chunks: int, pages_per_chunk: int, page_bytes: int,
                  pages_per_slice: int, slice_out, file_out=None, after_mult=None, group=None, digest=None,
                  stream=None):
    """Fused epilogue (cc_scan_epilogue_dev): slices, file CRCs, digest partials in
    one launch.  after_mult = xpow8(after_bytes) (int32 view of the multipliers)."""
    torch = _torch()
    opt = lambda t, w: _dev_ptr(t, w) if t is not None else None  # noqa: E731
    with torch.cuda.device(page_crcs.device):
        check(lib().cc_scan_epilogue_dev(_dev_ptr(page_crcs, "page_crcs"), _dev_ptr(meta_crcs, "meta_crcs"),
                                         n_chunks, pages_per_chunk, page_bytes, pages_per_slice,
                                         _dev_ptr(slice_out, "slice_out"), opt(file_out, "file_out"),
                                         opt(after_mult, "after_mult"), opt(group, "group"), opt(digest, "digest"),
                                         _stream_handle(stream)), "cc_scan_epilogue_dev")
    return slice_out


def combine_dev(a, b, len_b: int, out=None, stream=None):
    """out[i] = combine(a[i], b[i], len_b) on device."""
    torch = _torch()
    n = a.numel()
    if b.numel() != n:
        raise CurveCrcError(_lib.CC_EINVAL, "a / b length mismatch")
    if out is None:
        with _on_stream(stream):  # created on the stream the kernel writes it on
            out = torch.empty(n, dtype=torch.int32, device=a.device)
    with torch.cuda.device(a.device):
        check(lib().cc_combine_dev(_dev_ptr(a, "a"), _dev_ptr(b, "b"), int(len_b), n, _dev_ptr(out, "out"),
                                   _stream_handle(stream)), "cc_combine_dev")
    return out


def digest_fold_dev(gathered, nranks: int, out=None, stream=None):
    """cc_digest_fold_dev: gathered [nranks * n] int32 device partials -> XOR over ranks [n]."""
    torch = _torch()
    if nranks <= 0 or gathered.numel() % nranks:
        raise CurveCrcError(_lib.CC_EINVAL, "gathered size is not a multiple of nranks")
    n = gathered.numel() // nranks
    if out is None:
        with _on_stream(stream):  # created on the stream the kernel writes it on
            out = torch.empty(n, dtype=torch.int32, device=gathered.device)
    with torch.cuda.device(gathered.device):
        check(lib().cc_digest_fold_dev(_dev_ptr(gathered, "gathered"), nranks, n, _dev_ptr(out, "out"),
                                       _stream_handle(stream)), "cc_digest_fold_dev")
    return out


def digest_dev(file_crcs, after_bytes, group, n_groups: int, out=None, stream=None):
    """Per-copyset digest partials: out[group[i]] ^= shift(file_crcs[i], after_bytes[i])."""
    torch = _torch()
    n = file_crcs.numel()
    if after_bytes.numel() != n or group.numel() != n:
        raise CurveCrcError(_lib.CC_EINVAL, "file_crcs / after_bytes / group length mismatch")
    if out is None:
        with _on_stream(stream):  # created on the stream the kernel writes it on
            out = torch.zeros(n_groups, dtype=torch.int32, device=file_crcs.device)
    with torch.cuda.device(file_crcs.device):
        check(lib().cc_digest_dev(_dev_ptr(file_crcs, "file_crcs"), _dev_ptr(after_bytes, "after_bytes"),
                                  _dev_ptr(group, "group"), n, _dev_ptr(out, "out"), _stream_handle(stream)),
              "cc_digest_dev")
    return out


def page_crc_host(data, page_bytes: int = PAGE_SIZE):
    """Host in / host out (blocking): numpy uint8 buffer -> numpy uint32 CRCs."""
    import numpy as np
    a = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    if a.nbytes % page_bytes:
        raise CurveCrcError(_lib.CC_EINVAL, "size is not a multiple of page_bytes")
    n = a.nbytes // page_bytes
    out = np.empty(n, dtype=np.uint32)
    check(lib().cc_page_crc_host(ctypes.c_void_p(a.ctypes.data), n, page_bytes,
                                 ctypes.c_void_p(out.ctypes.data)), "cc_page_crc_host")
    return out


def scan_host(chunks, chunk_bytes: int = CHUNK_SIZE, meta_bytes: int = META_PAGE_SIZE,
              page_bytes: int = PAGE_SIZE, slice_bytes: int = SCAN_SIZE, after_bytes=None, group=None,
              n_groups: int = 0):
    """Streaming scan of host-resident chunk files (cc_scan_host / cc_scan_host_digest).
    `chunks`: sequence of (meta, data) numpy uint8 arrays (pinned or pageable, mixed).
    Returns (meta_crcs[n], slice_crcs[n, chunk/slice], file_crcs[n]) as uint32 numpy;
    with after_bytes / group / n_groups also the per-copyset digests [n_groups]
    computed on the device (4th element)."""
    import numpy as np
    n = len(chunks)
    arr = (_lib.CcChunkSrc * max(n, 1))()
    keep = []
    for i, (m, d) in enumerate(chunks):
        m = np.ascontiguousarray(m)
        d = np.ascontiguousarray(d)
        if m.nbytes != meta_bytes or d.nbytes != chunk_bytes:
            raise CurveCrcError(_lib.CC_EINVAL, f"chunk {i}: wrong metapage/data size")
        keep += [m, d]
        arr[i].meta = m.ctypes.data
        arr[i].data = d.ctypes.data
    S = chunk_bytes // slice_bytes
    mc = np.empty(n, dtype=np.uint32)
    sc = np.empty((n, S), dtype=np.uint32)
    fc = np.empty(n, dtype=np.uint32)
    if after_bytes is None:
        check(lib().cc_scan_host(arr, n, chunk_bytes, meta_bytes, page_bytes, slice_bytes,
                                 ctypes.c_void_p(mc.ctypes.data), ctypes.c_void_p(sc.ctypes.data),
                                 ctypes.c_void_p(fc.ctypes.data)), "cc_scan_host")
        return mc, sc, fc
    ab = np.ascontiguousarray(after_bytes, dtype=np.uint64)
    gr = np.ascontiguousarray(group, dtype=np.uint32)
    if ab.size != n or gr.size != n:
        raise CurveCrcError(_lib.CC_EINVAL, "after_bytes / group must hold one entry per chunk")
    dig = np.empty(max(1, n_groups), dtype=np.uint32)
    d = _lib.CcScanDigest(ab.ctypes.data, gr.ctypes.data, n_groups, dig.ctypes.data)
    check(lib().cc_scan_host_digest(arr, n, chunk_bytes, meta_bytes, page_bytes, slice_bytes,
                                    ctypes.c_void_p(mc.ctypes.data), ctypes.c_void_p(sc.ctypes.data),
                                    ctypes.c_void_p(fc.ctypes.data), ctypes.byref(d)), "cc_scan_host_digest")
    return mc, sc, fc, dig[:n_groups]


UPDATE_DTYPE = None


def _update_dtype():
    global UPDATE_DTYPE
    if UPDATE_DTYPE is None:
        import numpy as np
        UPDATE_DTYPE = np.dtype([("dst", "<u8"), ("src", "<u8"), ("len", "<u4"), ("reserved", "<u4")])
    return UPDATE_DTYPE


def log_records(dst_off, src_off, lens):
    """Write log (in write order) as cc_update records (numpy structured array)."""
    import numpy as np
    dst_off = np.asarray(dst_off, dtype=np.uint64)
    rec = np.zeros(dst_off.size, dtype=_update_dtype())
    rec["dst"], rec["src"], rec["len"] = dst_off, np.asarray(src_off, dtype=np.uint64), np.asarray(lens, np.uint32)
    return rec


_log_work = {}


def apply_log(pool, page_crcs, src, d_log, n_updates: int, max_len: int, page_bytes: int = PAGE_SIZE, stream=None,
              delta: bool = False):
    """cc_apply_log_dev: the write log `d_log` (device tensor of n_updates
    cc_update records, WRITE order, overlaps allowed) applied to `pool` with
    later writes winning, and the CRC of every touched page recomputed in
    `page_crcs` -- ordering, apply and rehash all on the device.
    delta=True -> cc_apply_log_delta_dev: `page_crcs` must hold the CRCs of the
    pages before the batch; they are updated by linearity from the touched rows
    only (a stale CRC stays stale instead of being refreshed)."""
    torch = _torch()
    need = int(lib().cc_apply_log_work_bytes(n_updates, max_len, page_bytes))
    if need == 0:
        raise CurveCrcError(_lib.CC_EINVAL, "unsupported log geometry")
    # scratch per (device, stream): calls on different streams may run at the
    # same time (the apply-thread model) and must not share keys / heads
    key = _stream_key(pool.device, stream)
    work = _log_work.get(key)
    if work is None or work.numel() < need:
        with _on_stream(stream):
            work = torch.empty(need, dtype=torch.uint8, device=pool.device)
        _log_work[key] = work
    with torch.cuda.device(pool.device):
        fn = "cc_apply_log_delta_dev" if delta else "cc_apply_log_dev"
        check(getattr(lib(), fn)(_dev_ptr(pool, "pool"), _nbytes(pool), page_bytes, _dev_ptr(src, "src"),
                                 _dev_ptr(d_log, "log"), n_updates, max_len, _dev_ptr(page_crcs, "page_crcs"),
                                 _dev_ptr(work, "work"), work.numel(), _stream_handle(stream)), fn)
    if stream is not None:
        work.record_stream(stream)
    return 1


def read_pages_list(offs, lens, page_bytes: int = PAGE_SIZE):
    """Diagnostic helper (host): the pages a batch of reads touches, read after
    read -- the list cc_page_list_probe_dev walks (int64 page indices; an empty
    read adds none)."""
    import numpy as np
    offs = np.asarray(offs, dtype=np.int64)
    lens = np.asarray(lens, dtype=np.int64)
    keep = lens > 0
    p0 = offs[keep] // page_bytes
    cnt = (offs[keep] + lens[keep] - 1) // page_bytes - p0 + 1
    start = np.repeat(p0 - np.concatenate(([0], np.cumsum(cnt)[:-1])), cnt)
    return start + np.arange(int(cnt.sum()), dtype=np.int64)


def page_list_probe(pool, d_pages, n: int, out, stream=None):
    """cc_page_list_probe_dev (diagnostic): the read traffic of a page list alone
    -- the ceiling of verify-on-read's access pattern.  `out` gets a word per page."""
    torch = _torch()
    with torch.cuda.device(pool.device):
        check(lib().cc_page_list_probe_dev(_dev_ptr(pool, "pool"), _nbytes(pool), _dev_ptr(d_pages, "pages"), n,
                                           _dev_ptr(out, "out"), _stream_handle(stream)), "cc_page_list_probe_dev")


def apply_logs(pool, page_crcs, batches, max_len: int, page_bytes: int = PAGE_SIZE, stream=None,
               delta: bool = False):
    """cc_apply_logs_dev: a QUEUE of write logs applied in order -- the same
    pool bytes and page CRCs as one apply_log call per batch, pipelined (each
    batch's page kernel also groups the next batch's pieces).  `batches`: a
    list of (src, d_log, n_updates) -- device tensors as for apply_log."""
    import ctypes
    torch = _torch()
    if not batches:
        return 0
    n_max = max(int(n) for _, _, n in batches)
    need = int(lib().cc_apply_logs_work_bytes(max(n_max, 1), max_len, page_bytes))
    if need == 0:
        raise CurveCrcError(_lib.CC_EINVAL, "unsupported log geometry")
    key = ("logs",) + tuple(_stream_key(pool.device, stream))
    work = _log_work.get(key)
    if work is None or work.numel() < need:
        with _on_stream(stream):
            work = torch.empty(need, dtype=torch.uint8, device=pool.device)
        _log_work[key] = work
    arr = (_lib.CcLogBatch * len(batches))()
    for i, (src, d_log, n) in enumerate(batches):
        arr[i].d_src = _dev_ptr(src, "src").value if int(n) else None
        arr[i].d_log = _dev_ptr(d_log, "log").value if int(n) else None
        arr[i].n_updates = int(n)
    with torch.cuda.device(pool.device):
        check(lib().cc_apply_logs_dev(_dev_ptr(pool, "pool"), _nbytes(pool), page_bytes, ctypes.cast(arr, ctypes.c_void_p),
                                      len(batches), max_len, _dev_ptr(page_crcs, "page_crcs"), 1 if delta else 0,
                                      _dev_ptr(work, "work"), work.numel(), _stream_handle(stream)), "cc_apply_logs_dev")
    if stream is not None:
        work.record_stream(stream)
    return 1


def apply_updates(pool, page_crcs, src, dst_off, src_off, lens, page_bytes: int = PAGE_SIZE, stream=None,
                  delta: bool = False):
    """Client partial-write path: host-side write log -> device (one copy of the
    records) -> cc_apply_log_dev (cc_apply_log_delta_dev with delta=True).
    Returns the number of device calls (1)."""
    import numpy as np
    torch = _torch()
    lens = np.asarray(lens, dtype=np.uint32)
    dst_off = np.asarray(dst_off, dtype=np.uint64)
    src_off = np.asarray(src_off, dtype=np.uint64)
    if not (dst_off.size == src_off.size == lens.size):
        raise CurveCrcError(_lib.CC_EINVAL, "dst/src/len size mismatch")
    if lens.size == 0:
        return 0
    if (lens == 0).any() or (dst_off + lens > _nbytes(pool)).any() or (src_off + lens > _nbytes(src)).any():
        raise CurveCrcError(_lib.CC_EINVAL, "update out of range or empty")
    rec = log_records(dst_off, src_off, lens)
    with _on_stream(stream):
        d_log = torch.from_numpy(rec.view(np.uint8)).to(pool.device)
    n = apply_log(pool, page_crcs, src, d_log, rec.size, int(lens.max()), page_bytes, stream, delta)
    if stream is not None:
        d_log.record_stream(stream)
    return n


def log_probe_descs(dst_off, src_off, lens, page_bytes: int = PAGE_SIZE):
    """Descriptors of cc_apply_log_probe_dev (the write log's page traffic
    alone) for one write log, built on the host: one per touched page, in the
    order of the first write touching it (the page pass's head order).  A page
    with ONE piece reads the rows that piece covers whole from the source (as
    cc_apply_log_dev does) and the rest from the page; every page stores back
    the rows its pieces touch.  Diagnostic: not part of the write path."""
    import numpy as np
    if page_bytes != 4096:
        raise CurveCrcError(_lib.CC_EINVAL, "the probe is built for 4 KiB pages")
    dst = np.asarray(dst_off, dtype=np.uint64)
    src = np.asarray(src_off, dtype=np.uint64)
    ln = np.asarray(lens, dtype=np.uint64)
    pb = np.uint64(page_bytes)
    p0, p1 = dst // pb, (dst + ln - np.uint64(1)) // pb
    span = int((p1 - p0).max()) + 1 if dst.size else 0
    pg, upd = [], []
    for k in range(span):  # piece k of every write that reaches its k-th page
        m = p0 + np.uint64(k) <= p1
        pg.append(p0[m] + np.uint64(k))
        upd.append(np.nonzero(m)[0])
    pg, upd = np.concatenate(pg), np.concatenate(upd)
    pbase = pg * pb
    rlo = (np.maximum(dst[upd], pbase) - pbase).astype(np.int64)
    rhi = (np.minimum(dst[upd] + ln[upd], pbase + pb) - pbase).astype(np.int64)
    r0, r1 = rlo >> 8, (rhi - 1) >> 8
    dirty = ((np.int64(2) << r1) - 1) & ~((np.int64(1) << r0) - 1)
    f0, f1 = (rlo + 255) >> 8, rhi >> 8
    cov = np.where(f1 > f0, ((np.int64(1) << f1) - 1) & ~((np.int64(1) << f0) - 1), 0)
    soff = src[upd] - dst[upd] + pbase  # modular, as cc_apply_log_dev's per-piece source pointer
    order = np.lexsort((upd, pg))  # pieces grouped by page, log order inside
    pg, upd, dirty, cov, soff = pg[order], upd[order], dirty[order], cov[order], soff[order]
    starts = np.flatnonzero(np.r_[True, pg[1:] != pg[:-1]])
    counts = np.diff(np.r_[starts, pg.size])
    out = np.zeros(starts.size, dtype=[("page", "<u8"), ("src_off", "<u8"), ("covered", "<u4"), ("dirty", "<u4")])
    out["page"] = pg[starts]
    out["dirty"] = np.bitwise_or.reduceat(dirty, starts).astype(np.uint32)
    single = counts == 1
    out["covered"] = np.where(single, cov[starts], 0).astype(np.uint32)
    out["src_off"] = np.where(single, soff[starts], 0)
    return out[np.argsort(upd[starts], kind="stable")]  # head order: by the first write touching the page


def log_probe(pool, src, d_desc, n: int, out, stream=None):
    """cc_apply_log_probe_dev over `n` descriptors resident on the device."""
    with _torch().cuda.device(pool.device):
        check(lib().cc_apply_log_probe_dev(_dev_ptr(pool, "pool"), _nbytes(pool), _dev_ptr(src, "src"),
                                           _dev_ptr(d_desc, "desc"), n, _dev_ptr(out, "out"),
                                           _stream_handle(stream)), "cc_apply_log_probe_dev")


_reads_work = {}


def verify_read_records(pool, page_crcs, d_reads, n_reads: int, bad, total, page_bytes: int = PAGE_SIZE,
                        stream=None):
    """cc_verify_reads_dev on a batch already resident on the device: `d_reads`
    = int64 device tensor of n_reads (offset, length) pairs; mismatches are
    ADDED to `bad` (int32 [n_reads], -1 marks a read past the pool) and
    `total` (int64 [1]).  Work buffer cached per (device, stream).  No host sync."""
    torch = _torch()
    need = int(lib().cc_verify_reads_work_bytes(n_reads))
    if need == 0:
        raise CurveCrcError(_lib.CC_EINVAL, "unsupported read batch")
    key = _stream_key(pool.device, stream)
    work = _reads_work.get(key)
    if work is None or work.numel() < need:
        with _on_stream(stream):
            work = torch.empty(need, dtype=torch.uint8, device=pool.device)
        _reads_work[key] = work
    with torch.cuda.device(pool.device):
        check(lib().cc_verify_reads_dev(_dev_ptr(pool, "pool"), _nbytes(pool), page_bytes, _dev_ptr(d_reads, "reads"),
                                        n_reads, _dev_ptr(page_crcs, "page_crcs"), _dev_ptr(bad, "bad"),
                                        _dev_ptr(total, "total"), _dev_ptr(work, "work"), work.numel(),
                                        _stream_handle(stream)), "cc_verify_reads_dev")
    if stream is not None:
        work.record_stream(stream)


def verify_reads(pool, page_crcs, offsets, lengths, page_bytes: int = PAGE_SIZE, stream=None):
    """cc_verify_reads_dev: verify-on-read for a batch of reads of the pool.
    Returns (bad pages per read: int32 device tensor, -1 = read past the pool;
    total bad pages: int64 device tensor [1]).  No host sync."""
    import numpy as np
    torch = _torch()
    off = np.asarray(offsets, dtype=np.uint64)
    ln = np.asarray(lengths, dtype=np.uint64)
    if off.size != ln.size:
        raise CurveCrcError(_lib.CC_EINVAL, "offsets/lengths size mismatch")
    n = off.size
    with _on_stream(stream):
        bad = torch.zeros(max(n, 1), dtype=torch.int32, device=pool.device)
        total = torch.zeros(1, dtype=torch.int64, device=pool.device)
        if n == 0:
            return bad[:0], total
        rng = torch.from_numpy(np.stack([off, ln], axis=1).reshape(-1).view(np.int64)).to(pool.device)
        need = int(lib().cc_verify_reads_work_bytes(n))
        work = torch.empty(need, dtype=torch.uint8, device=pool.device)
    with torch.cuda.device(pool.device):
        check(lib().cc_verify_reads_dev(_dev_ptr(pool, "pool"), _nbytes(pool), page_bytes, _dev_ptr(rng, "reads"), n,
                                        _dev_ptr(page_crcs, "page_crcs"), _dev_ptr(bad, "bad"),
                                        _dev_ptr(total, "total"), _dev_ptr(work, "work"), need,
                                        _stream_handle(stream)), "cc_verify_reads_dev")
    if stream is not None:
        for t in (rng, work):
            t.record_stream(stream)
    return bad, total


def scan_files(paths, chunk_bytes: int = CHUNK_SIZE, meta_bytes: int = META_PAGE_SIZE,
               page_bytes: int = PAGE_SIZE, slice_bytes: int = SCAN_SIZE, io_threads: int = 0):
    """cc_scan_files: native pread + scan of chunk files.
    Returns (status[n] int32, meta_crcs[n], slice_crcs[n, S], file_crcs[n]) numpy."""
    import numpy as np
    n = len(paths)
    arr = (ctypes.c_char_p * max(n, 1))(*[os.fsencode(p) for p in paths])
    res = (_lib.CcFileResult * max(n, 1))()
    S = chunk_bytes // slice_bytes
    sc = np.zeros((n, S), dtype=np.uint32)
    check(lib().cc_scan_files(arr, n, chunk_bytes, meta_bytes, page_bytes, slice_bytes, io_threads,
                              ctypes.c_void_p(sc.ctypes.data), res), "cc_scan_files")
    st = np.array([res[i].status for i in range(n)], dtype=np.int32)
    mc = np.array([res[i].meta_crc for i in range(n)], dtype=np.uint32)
    fc = np.array([res[i].file_crc for i in range(n)], dtype=np.uint32)
    return st, mc, sc, fc


def default_io_threads() -> int:
    """cc_default_io_threads: the reader count scan_files(io_threads=0) uses."""
    return int(lib().cc_default_io_threads())


def as_u32(t) -> "list[int]":
    """Device/host int32 CRC tensor -> python ints in [0, 2^32)."""
    return [int(x) & 0xFFFFFFFF for x in t.detach().cpu().tolist()]
