"""The shared-memory RCCL stand-in that lets one-GPU tests run the multi-rank
native digest exchange (tests/native/rccl_stub.cpp; GPU use in
tests/test_distributed_gpu.py::test_bench_world8_native_exchange_over_stub_rccl).
Its communicator set-up needs no GPU: N processes meet at the init barrier and
the last one out removes the segment; a rank whose peer never comes gets an
error at the bound instead of hanging."""
import ctypes
import multiprocessing as mp
import os

import pytest

from conftest import ROOT

STUB = os.path.join(ROOT, "build", "stub", "librccl_stub.so")


class UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


def _lib():
    L = ctypes.CDLL(STUB)
    L.ncclGetUniqueId.argtypes = [ctypes.POINTER(UniqueId)]
    L.ncclCommInitRankConfig.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, UniqueId, ctypes.c_int,
                                         ctypes.c_void_p]
    L.ncclCommDestroy.argtypes = [ctypes.c_void_p]
    return L


def _rank(uid_bytes, nranks, rank, q):
    L = _lib()
    uid = UniqueId()
    uid.internal = uid_bytes
    comm = ctypes.c_void_p()
    rc = L.ncclCommInitRankConfig(ctypes.byref(comm), nranks, uid, rank, None)
    rd = L.ncclCommDestroy(comm) if rc == 0 else -1
    q.put((rank, rc, rd))


@pytest.fixture(scope="module")
def stub():
    if not os.path.exists(STUB):
        pytest.skip("make -C curve_amd/csrc stubrccl")
    return _lib()


def test_stub_ranks_meet_and_clean_up(stub):
    uid = UniqueId()
    assert stub.ncclGetUniqueId(ctypes.byref(uid)) == 0
    name = uid.internal.decode()
    assert name.startswith("/ccrcclstub-")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(uid.internal, 4, r, q)) for r in range(4)]
    for p in ps:
        p.start()
    got = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    assert got == [(r, 0, 0) for r in range(4)]
    assert not os.path.exists("/dev/shm" + name)  # the last rank out unlinked it


def test_stub_missing_peer_is_an_error_not_a_hang(stub, monkeypatch):
    monkeypatch.setenv("CC_RCCL_STUB_WAIT_S", "1")
    uid = UniqueId()
    assert stub.ncclGetUniqueId(ctypes.byref(uid)) == 0
    comm = ctypes.c_void_p()
    rc = stub.ncclCommInitRankConfig(ctypes.byref(comm), 2, uid, 0, None)
    assert rc == 2  # ncclSystemError: rank 1 never came
    assert not os.path.exists("/dev/shm" + uid.internal.decode())
