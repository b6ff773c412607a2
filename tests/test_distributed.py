"""N>1 path on CPU: world_size-2 gloo, chunk-range sharding + per-copyset digest
exchange (all_gather + XOR) reproduces CopysetNode::GetHash's chained CRC.
File CRCs here come from libcurvecrc's CPU primitive (no GPU in this container);
the GPU path feeds the same partials from cc_digest_dev."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def make_pool(n_chunks=13, data_bytes=64 << 10, meta_bytes=4096):
    rng = np.random.default_rng(123)
    ids = [1, 2, 3, 10, 11, 20, 100, 5, 7, 9, 12, 21, 1000][:n_chunks]
    copyset_of = [i % 3 for i in range(n_chunks)]
    files = [rng.integers(0, 256, meta_bytes + data_bytes, dtype=np.uint8).tobytes() for _ in range(n_chunks)]
    return ids, copyset_of, files


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import curve_amd.crc as C
        from curve_amd.pool import copyset_layout, reduce_digests, shard_range, digests_as_hash_strings
        ids, copyset_of, files = make_pool()
        lay = copyset_layout(ids, copyset_of, [len(f) for f in files])
        lo, hi = shard_range(len(ids), rank, world)
        partial = torch.zeros(lay.n_groups, dtype=torch.int64)
        for i in range(lo, hi):
            v = C.shift(C.CRC32(files[i]), lay.after_bytes[i])
            partial[lay.group[i]] ^= v
        full = reduce_digests(partial.to(torch.int32), dist)
        q.put((rank, digests_as_hash_strings(full)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_digest_matches_chained_copyset_hash(oracle, world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in ps]
    res = dict(q.get(timeout=120) for _ in range(world))
    [p.join(timeout=60) for p in ps]
    assert all(p.exitcode == 0 for p in ps)
    from curve_amd.pool import copyset_layout
    ids, copyset_of, files = make_pool()
    lay = copyset_layout(ids, copyset_of, [len(f) for f in files])
    want = []
    for g in sorted(set(copyset_of)):
        members = {f"chunk_{ids[i]}": files[i] for i in range(len(ids)) if copyset_of[i] == g}
        want.append(oracle.copyset_hash(members))
    for r in range(world):
        assert res[r] == want


def test_shard_range_partitions():
    from curve_amd.pool import shard_range
    for n in (0, 1, 7, 1024, 8193):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1


def test_lexicographic_order_quirk():
    """std::sort on names: chunk_10 sorts before chunk_2 (copyset_node.cpp:938)."""
    from curve_amd.scan import copyset_after_bytes
    names = ["chunk_2", "chunk_10", "chunk_1"]
    after = copyset_after_bytes(names, [1, 10, 100])
    # sorted: chunk_1 (100), chunk_10 (10), chunk_2 (1)
    assert after == [0, 1, 11]


def _agree_worker(rank, world, port, inject, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if inject is not None:
        os.environ["CC_INJECT_COMM_INIT_FAIL_RANK"] = str(inject)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from curve_amd.pool import agreed_comm
        comm, note = agreed_comm(dist, timeout_ms=2000)
        q.put((rank, comm is None, note))
    except Exception as e:
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("inject", [None, 0, 1])
def test_exchange_path_agreement_no_gpu(inject):
    """The ranks agree on ONE digest-exchange path before any collective
    (pool.agreed_comm): here no rank has a GPU (rank 0 cannot even make the
    RCCL id, and says so to the others instead of leaving them in the
    broadcast), and with a failure injected on one rank, every rank returns the
    torch.distributed path -- and nobody hangs."""
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_agree_worker, args=(r, world, port, inject, q)) for r in range(world)]
    [p.start() for p in ps]
    try:
        res = dict((r, (fell_back, note)) for r, fell_back, note in (q.get(timeout=60) for _ in range(world)))
    finally:
        [p.join(timeout=30) for p in ps]
        for p in ps:
            if p.is_alive():
                p.kill()
    assert all(res[r][0] is True for r in range(world)), res
    assert all("torch.distributed" in res[r][1] for r in range(world)), res
