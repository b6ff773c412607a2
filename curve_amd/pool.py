"""Full-pool integrity scan sharded across GPUs (BASELINE config 5).

One process per GPU.  Chunk files are sharded by contiguous chunk-index range;
each rank hashes its own files on its own GPU with no data-path collective.  The
only exchange is the per-copyset digest: CopysetNode::GetHash
(src/chunkserver/copyset_node.cpp:925-975) is an ORDERED chain over files in
std::sort name order, but in the linear GF(2) domain each file contributes
shift(V(file), bytes after it in that order), so every rank computes order-free
XOR partials for the files it holds and one all_gather of 4 B per copyset per
rank (RCCL over xGMI on GPUs, gloo on CPU) finishes it.  A commutative XOR is
not an RCCL reduction op, hence all_gather + local XOR rather than all_reduce.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Sequence

from .scan import chunk_file_name, copyset_after_bytes


def shard_range(n_total: int, rank: int, world: int):
    """Contiguous chunk-index range [lo, hi) of `rank` (sizes differ by <= 1)."""
    base, rem = divmod(n_total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


@dataclass
class CopysetLayout:
    """Which copyset each chunk file belongs to and its digest shift."""
    names: List[str]
    group: List[int]          # copyset index per file
    after_bytes: List[int]    # bytes of the same copyset sorting after the file
    n_groups: int


def copyset_layout(chunk_ids: Sequence[int], copyset_of: Sequence[int], file_bytes: Sequence[int]) -> CopysetLayout:
    """Geometry of the whole pool (every rank computes the same layout)."""
    names = [chunk_file_name(c) for c in chunk_ids]
    groups = sorted(set(copyset_of))
    gidx = {g: i for i, g in enumerate(groups)}
    group = [gidx[g] for g in copyset_of]
    after = [0] * len(names)
    members: Dict[int, List[int]] = {}
    for i, g in enumerate(group):
        members.setdefault(g, []).append(i)
    for g, mem in members.items():
        for i, a in zip(mem, copyset_after_bytes([names[i] for i in mem], [file_bytes[i] for i in mem])):
            after[i] = a
    return CopysetLayout(names, group, after, len(groups))


def reduce_digests(partial, dist, group=None):
    """XOR-reduce per-copyset partials (int32 tensor [n_groups]) over all ranks:
    all_gather_into_tensor (RCCL, or gloo through host memory) then the XOR
    fold -- on the device through libcurvecrc (cc_digest_fold_dev) when the
    partials live there, on the host for host tensors.  Returns the full digests
    on every rank, on the partials' device."""
    import torch
    world = dist.get_world_size(group)
    if world == 1:
        return partial
    dev = partial.device
    src = partial
    if dist.get_backend(group) == "gloo" and partial.is_cuda:
        src = partial.cpu()  # gloo moves host tensors; RCCL works on device tensors
    gathered = torch.empty(world * src.numel(), dtype=src.dtype, device=src.device)
    dist.all_gather_into_tensor(gathered, src.contiguous(), group=group)
    if partial.is_cuda:
        from .crc import digest_fold_dev
        return digest_fold_dev(gathered.to(dev), world)
    g = gathered.view(world, -1)
    out = g[0].clone()
    for r in range(1, world):
        out.bitwise_xor_(g[r])
    return out


def digests_as_hash_strings(digests) -> List[str]:
    """Per-copyset digests -> GetCopysetStatus(queryhash) strings (std::to_string(uint32))."""
    return [str(int(x) & 0xFFFFFFFF) for x in digests.detach().cpu().tolist()]


# ---------------------------------------------------------------------------
# Native path (libcurvecrc): RCCL communicator + one-call shard scan.  This is
# what a C++ chunkserver binds (include/curve_crc.h cc_comm_* / cc_pool_scan_dev);
# torch is only the device-memory / stream / rendezvous plumbing here.
# ---------------------------------------------------------------------------
class Comm:
    """An RCCL communicator created and owned by libcurvecrc (cc_comm_init_timeout:
    non-blocking RCCL init polled against a deadline, aborted when it expires)."""

    def __init__(self, nranks: int, rank: int, uid: bytes, timeout_ms: int = 0):
        import ctypes
        from . import _lib
        if len(uid) != _lib.CC_COMM_ID_BYTES:
            raise ValueError("unique id must be CC_COMM_ID_BYTES long")
        self._h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(bytes(uid), len(uid))
        _lib.check(_lib.lib().cc_comm_init_timeout(ctypes.byref(self._h), nranks, rank, buf, len(uid),
                                                   int(timeout_ms)), "cc_comm_init")
        self.nranks, self.rank = nranks, rank

    @staticmethod
    def unique_id() -> bytes:
        import ctypes
        from . import _lib
        buf = ctypes.create_string_buffer(_lib.CC_COMM_ID_BYTES)
        _lib.check(_lib.lib().cc_comm_unique_id(buf, _lib.CC_COMM_ID_BYTES), "cc_comm_unique_id")
        return buf.raw

    @property
    def handle(self):
        return self._h

    def allreduce_digest(self, digest, stream=None):
        """In place: digest[g] <- XOR over ranks (cc_digest_allreduce_dev)."""
        from . import _lib
        from .crc import _dev_ptr, _stream_handle
        _lib.check(_lib.lib().cc_digest_allreduce_dev(self._h, _dev_ptr(digest, "digest"), digest.numel(),
                                                      _stream_handle(stream)), "cc_digest_allreduce_dev")
        return digest

    def wait(self, stream=None, timeout_ms: int = 0):
        """Bounded wait for the stream's work so far, the digest exchanges
        included (cc_comm_wait): raises CurveCrcError(CC_ETIMEDOUT) -- the
        communicator aborted -- when a peer stopped participating."""
        from . import _lib
        from .crc import _stream_handle
        _lib.check(_lib.lib().cc_comm_wait(self._h, _stream_handle(stream), int(timeout_ms)), "cc_comm_wait")

    def close(self):
        from . import _lib
        if self._h:
            h, self._h = self._h, None
            _lib.check(_lib.lib().cc_comm_destroy(h), "cc_comm_destroy")

    def abort(self):
        """Leave without waiting for the peers (cc_comm_abort)."""
        from . import _lib
        if self._h:
            h, self._h = self._h, None
            _lib.lib().cc_comm_abort(h)

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


# Failure injection for the agreement protocol (the reference's libfiu
# failpoints play this role, test/failpoint/): when this environment variable
# holds a rank number, that rank's native init fails before it reaches RCCL,
# as a rank whose device or RCCL setup broke would.
FAIL_INIT_RANK_ENV = "CC_INJECT_COMM_INIT_FAIL_RANK"


def comm_from_dist(dist, group=None, timeout_ms: int = 0) -> Comm:
    """Rank 0 makes the RCCL unique id, torch.distributed carries its 128 bytes
    to every rank (as the MDS or any out-of-band channel would), then every
    rank joins the native communicator on its current device."""
    import os
    from . import _lib
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    obj = [None]
    if rank == 0:  # a failure here is broadcast too: the other ranks must not wait for an id forever
        try:
            obj = [Comm.unique_id()]
        except Exception as e:
            obj = [f"rank 0 could not create the RCCL id: {e}"]
    dist.broadcast_object_list(obj, src=0, group=group)
    if not isinstance(obj[0], bytes):
        raise _lib.CurveCrcError(_lib.CC_ECOMM, f"cc_comm_unique_id ({obj[0]})")
    if os.environ.get(FAIL_INIT_RANK_ENV, "") == str(rank):
        raise _lib.CurveCrcError(_lib.CC_ECOMM, f"cc_comm_init (injected failure on rank {rank})")
    return Comm(world, rank, obj[0], timeout_ms=timeout_ms)


def agreed_comm(dist, device=None, group=None, timeout_ms: int = 0):
    """Every rank takes the SAME digest-exchange path, or a mismatched
    collective hangs: each rank tries the native communicator (bounded by
    `timeout_ms`), then the ranks all-reduce(MIN) a success flag.  If any
    rank failed, the ranks that succeeded abort theirs and every rank returns
    None (the torch.distributed exchange, reduce_digests).  Returns
    (comm or None, note saying which path runs and why)."""
    import torch
    err = None
    comm = None
    try:
        comm = comm_from_dist(dist, group=group, timeout_ms=timeout_ms)
    except Exception as e:  # CurveCrcError (ECOMM / ETIMEDOUT / ENODEV) or a rendezvous error
        err = e
    on_dev = dist.get_backend(group) != "gloo" and device is not None
    flag = torch.tensor([0 if err else 1], dtype=torch.int32, device=device if on_dev else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    ok_all = bool(int(flag.item()))
    if ok_all:
        return comm, "native RCCL (cc_comm_init_timeout + cc_digest_allreduce_dev)"
    if comm is not None:
        comm.abort()
    why = f"this rank: {err}" if err else "another rank's native init failed"
    return None, f"torch.distributed all_gather_into_tensor + cc_digest_fold_dev (native comm not agreed: {why})"


def pool_scan(pool, after_mult, group, digest, comm: "Comm" = None, stream=None, events=None,
              exchange_events=None):
    """One integrity scan pass over a DevicePool shard as ONE native call
    (cc_pool_scan_dev): page CRCs, metapage CRCs, slice/file CRCs, digest
    partials and -- with a Comm -- the RCCL digest exchange.  `events` =
    (begin, end) torch.cuda.Event pair recorded around the page kernel (they
    must already exist: record each once beforehand); `exchange_events` the
    same around the exchange (all-gather + XOR fold; recorded only with a Comm)."""
    import ctypes
    from . import _lib
    from .crc import _dev_ptr, _stream_handle
    s = _lib.CcPoolShard()
    s.d_data = _dev_ptr(pool.data, "data").value
    s.d_meta = _dev_ptr(pool.meta, "meta").value
    s.n_chunks = pool.n
    s.chunk_bytes, s.meta_bytes = pool.chunk_size, pool.meta_size
    s.page_bytes, s.slice_bytes = pool.page_bytes, pool.scan_size
    s.d_after_mult = _dev_ptr(after_mult, "after_mult").value if after_mult is not None else None
    s.d_group = _dev_ptr(group, "group").value if group is not None else None
    s.n_groups = digest.numel() if digest is not None else 0
    s.d_page_crcs = _dev_ptr(pool.page_crcs, "page_crcs").value
    s.d_meta_crcs = _dev_ptr(pool.meta_crcs, "meta_crcs").value
    s.d_slice_crcs = _dev_ptr(pool.slice_crcs, "slice_crcs").value
    s.d_file_crcs = _dev_ptr(pool.file_crcs, "file_crcs").value
    s.d_digest = _dev_ptr(digest, "digest").value if digest is not None else None
    if events is not None:
        s.ev_pages_begin, s.ev_pages_end = events[0].cuda_event, events[1].cuda_event
    if exchange_events is not None:
        s.ev_exchange_begin, s.ev_exchange_end = exchange_events[0].cuda_event, exchange_events[1].cuda_event
    _lib.check(_lib.lib().cc_pool_scan_dev(ctypes.byref(s), comm.handle if comm is not None else None,
                                           _stream_handle(stream)), "cc_pool_scan_dev")
    return digest
