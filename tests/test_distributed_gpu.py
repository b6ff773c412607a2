"""BASELINE config 5 (the node-level pool scan) with more than one
rank, on the one-GPU test box: two (and three) gloo ranks share cuda:0; each
runs the native one-call shard scan (cc_pool_scan_dev) over its chunk range, the
per-copyset XOR partials are all-gathered over gloo and folded ON THE DEVICE by
cc_digest_fold_dev -- the same fold cc_digest_allreduce_dev runs after its RCCL
all-gather (RCCL itself refuses two ranks on one device, "Duplicate GPU
detected", so the RCCL transport is exercised at world 1 in test_pool_native.py
and at N GPUs by the driver's multi-GPU bench).  The reduced digests must equal
CopysetNode::GetHash's sorted-name chain (copyset_node.cpp:925-975) over the
WHOLE pool, computed by the oracle."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


N_CHUNKS, CHUNK = 13, 1 << 20


def _pool_arrays():
    rng = np.random.default_rng(2024)
    data = rng.integers(0, 256, (N_CHUNKS, CHUNK), dtype=np.uint8)
    meta = rng.integers(0, 256, (N_CHUNKS, 4096), dtype=np.uint8)
    meta[:, 0] = 2
    ids = [1, 2, 3, 10, 11, 20, 100, 5, 7, 9, 12, 21, 1000]
    groups = [i % 4 for i in range(N_CHUNKS)]
    return data, meta, ids, groups


def _rank_main(rank, world, port, q, agreed=False, inject=None):
    import sys
    import time
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if inject is not None:
        os.environ["CC_INJECT_COMM_INIT_FAIL_RANK"] = str(inject)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from curve_amd import crc as C
        from curve_amd.pool import (agreed_comm, copyset_layout, digests_as_hash_strings, pool_scan, reduce_digests,
                                    shard_range)
        from curve_amd.scan import DevicePool
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        data, meta, ids, groups = _pool_arrays()
        lay = copyset_layout(ids, groups, [CHUNK + 4096] * N_CHUNKS)
        lo, hi = shard_range(N_CHUNKS, rank, world)
        pool = DevicePool(torch.from_numpy(data[lo:hi]).to(dev), torch.from_numpy(meta[lo:hi]).to(dev), ids[lo:hi],
                          scan_size=256 << 10)
        after = torch.tensor(lay.after_bytes[lo:hi], dtype=torch.int64, device=dev)
        grp = torch.tensor(lay.group[lo:hi], dtype=torch.int32, device=dev)
        digest = torch.full((lay.n_groups,), -1, dtype=torch.int32, device=dev)
        comm, note, t_agree = None, "plain", 0.0
        if agreed:  # the bench's protocol: bounded native init, then ONE path for all ranks
            t0 = time.perf_counter()
            comm, note = agreed_comm(dist, device=dev, timeout_ms=4000)
            t_agree = time.perf_counter() - t0
        pool_scan(pool, C.xpow8(after), grp, digest, comm=comm)  # one native call: pages, slices, files, partials
        # without a native comm: gloo all-gather + cc_digest_fold_dev
        full = digest if comm is not None else reduce_digests(digest, dist)
        torch.cuda.synchronize()
        if comm is not None:
            comm.close()
        q.put((rank, digests_as_hash_strings(full), [int(x) & 0xFFFFFFFF for x in pool.file_crcs.cpu().tolist()],
               note, t_agree))
    except Exception as e:  # report to the parent instead of hanging it
        q.put((rank, repr(e), None, None, None))
    finally:
        dist.destroy_process_group()


def _run_ranks(world, agreed=False, inject=None):
    import torch.multiprocessing as mp
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, q, agreed, inject)) for r in range(world)]
    [p.start() for p in ps]
    try:
        res = {}
        for _ in range(world):
            r, dig, fcs, note, t_agree = q.get(timeout=100)
            res[r] = (dig, fcs, note, t_agree)
    finally:
        [p.join(timeout=30) for p in ps]
        for p in ps:
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    return res


def _check_against_oracle(oracle, res, world):
    from curve_amd.pool import copyset_layout, shard_range
    from curve_amd.scan import chunk_file_name
    data, meta, ids, groups = _pool_arrays()
    lay = copyset_layout(ids, groups, [CHUNK + 4096] * N_CHUNKS)
    want = []
    for g in range(lay.n_groups):
        files = {chunk_file_name(ids[i]): meta[i].tobytes() + data[i].tobytes()
                 for i in range(N_CHUNKS) if lay.group[i] == g}
        want.append(oracle.copyset_hash(files))
    for r in range(world):
        assert res[r][0] == want, (r, res[r][0])
        lo, hi = shard_range(N_CHUNKS, r, world)
        assert res[r][1] == [oracle.crc32c(meta[i].tobytes() + data[i].tobytes()) for i in range(lo, hi)]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_pool_scan_device_fold_matches_whole_pool_chain(oracle, world):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _check_against_oracle(oracle, _run_ranks(world), world)


@pytest.mark.parametrize("inject", [None, 0, 1])
def test_exchange_agreement_with_one_rank_failing_native_init(oracle, inject):
    """The N>1 bench's exchange protocol (pool.agreed_comm) on one GPU: a
    failure injected into ONE rank's native init (rank 0 after it made the
    RCCL id, or rank 1), or none (RCCL then refuses two ranks on one device
    by itself).  The other rank's bounded init gives up (4 s here) instead of
    waiting for its peer forever, the ranks reduce a success flag, all take
    the torch.distributed exchange, and the digests equal the oracle's
    whole-pool chain: no mismatched collectives, no hang."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = _run_ranks(2, agreed=True, inject=inject)
    for r in range(2):
        assert res[r][2] is not None and "torch.distributed" in res[r][2], res[r]
        assert res[r][3] < 30.0, res[r][3]  # bounded: the 4 s init timeout + bootstrap
    _check_against_oracle(oracle, res, 2)


@pytest.mark.parametrize("nranks", [1, 2, 3, 8])
def test_digest_fold_dev_any_rank_count(nranks):
    """cc_digest_fold_dev (the device XOR fold of the exchange) at 1..8 ranks'
    worth of gathered partials, against numpy's XOR."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from curve_amd import crc as C
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(nranks)
    for n in (1, 64, 5000):
        g = rng.integers(0, 2**32, (nranks, n), dtype=np.uint64).astype(np.uint32)
        out = C.digest_fold_dev(torch.from_numpy(g.reshape(-1).view(np.int32)).to(dev), nranks)
        want = np.bitwise_xor.reduce(g, axis=0)
        assert (out.cpu().numpy().view(np.uint32) == want).all()


def test_bench_rank_lost_after_init_ends_with_an_error_line(tmp_path):
    """A peer that stops participating in the digest exchange AFTER init (the
    bench's CC_INJECT_SKIP_EXCHANGE_RANK failpoint: rank 1 skips its exchange
    every step) must end the N>1 bench with a JSON error line and a non-zero
    exit within its bound -- not a hang until the driver's limit with no line.
    Two gloo ranks on cuda:0 (RCCL refuses two ranks on one device, so the
    ranks agree on the torch.distributed exchange, bounded by the group
    timeout, BENCH_DIST_TIMEOUT_S; the native exchange's bound, cc_comm_wait,
    is tested in test_pool_native.py)."""
    import json
    import subprocess
    import sys
    import time
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo", CC_INJECT_SKIP_EXCHANGE_RANK="1", BENCH_DIST_TIMEOUT_S="15")
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--chunks", "16", "--steps", "3",
           "--warmup", "1", "--clock-warm-ms", "0", "--comm-timeout-ms", "5000", "--no-cpu-baseline", "--no-e2e",
           "--no-pmc", "--updates", "0", "--reads", "0", "--wal-entries", "0", "--stream-chunks", "0",
           "--file-chunks", "0"]
    t0 = time.perf_counter()
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=240)
    el = time.perf_counter() - t0
    assert r.returncode != 0, r.stdout[-2000:]
    # rank 0's error line on stdout (the driver's), the other rank's on stderr
    errs = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{") and '"error"' in x]
    assert len(errs) == 1 and errs[0]["error"].startswith("rank 0:"), r.stdout[-2000:]
    assert all(e["value"] is None and "digest exchange failed" in e["error"] for e in errs), r.stdout[-2000:]
    assert el < 200, el  # the 15 s group timeout, rendezvous and two torch imports


def _bench_world8(tmp_path, log_name, extra_env=None):
    """`bench.py --gpus 8` (it starts torch.distributed.run itself, as a child),
    8 gloo ranks sharing cuda:0, 16 chunks a rank; returns rank 0's line after
    checking everything the N>1 line must hold."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    world, chunks = 8, 16
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo", BENCH_DIST_TIMEOUT_S="240", **(extra_env or {}))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", str(world), "--chunks", str(chunks),
           "--steps", "3", "--warmup", "1", "--clock-warm-ms", "0", "--comm-timeout-ms", "5000", "--no-pmc",
           "--stream-chunks-per-rank", "4", "--file-chunks", "0"]
    # the ranks' output goes to a file that grows while they run (a GPU box's
    # runner takes a call that prints nothing for minutes to be hung)
    out_dir = os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out") if "GRAFT_REPO_ROOT" in os.environ \
        else str(tmp_path)
    os.makedirs(out_dir, exist_ok=True)
    log_path = os.path.join(out_dir, log_name)
    with open(log_path, "w") as logf:
        r = subprocess.run(cmd, cwd=str(tmp_path), env=env, stdout=logf, stderr=subprocess.STDOUT, timeout=360)
    text = open(log_path).read()
    assert r.returncode == 0, text[-4000:]
    lines = [json.loads(x) for x in text.splitlines() if x.startswith("{")]
    assert len(lines) == 1, text[-4000:]  # rank 0 prints the one line
    d = lines[0]
    assert d["n_gpus"] == world and d["value"] > 0 and d["scaling"] == "weak"
    roof = d["roofline"]
    assert len(roof["rank_kernel_ms"]) == world and all(x > 0 for x in roof["rank_kernel_ms"])
    assert roof["aggregate_peak"] == 8000.0 * world
    want_agg = world * roof["alg_bytes_per_launch"] / (max(roof["rank_kernel_ms"]) * 1e-3) / 1e9
    assert abs(roof["aggregate_achieved"] - want_agg) <= 0.2 + 1e-3 * want_agg
    assert d["digest_check_cpu"]["ok"] is True
    ex = d["digest_exchange"]
    assert ex["matches_cpu_chain"] is True
    # the exchange's own time per timed step and its share of the step
    assert len(ex["ms_each"]) == 3 and all(x > 0 for x in ex["ms_each"]), ex
    assert len(ex["rank_ms_avg"]) == world and all(x > 0 for x in ex["rank_ms_avg"]), ex
    assert 0 < ex["share_of_step"] <= ex["share_of_step_max_rank"] + 1e-9, ex
    assert ex["share_of_step_max_rank"] < 1.5, ex  # an exchange inside the step (host wall may include some slack)
    sa = d["stream_all_ranks"]
    assert sa.get("digest_check_ok") is True and sa["ranks"] == world, sa
    # every chunk of the whole pool in exactly one rank's shard, in rank order
    ranges = d["shard_ranges"]
    assert len(ranges) == world
    covered = [c for lo, hi in ranges for c in range(lo, hi)]
    assert covered == list(range(world * chunks))
    assert d["verify"]["bad_pages"] == 0
    assert "bound" in d["numa_binding_rank0"]  # the rank's NUMA binding is reported (bound or why not)
    return d


@pytest.mark.timeout(420)
def test_bench_world8_gloo_rehearsal(tmp_path):
    """The driver's 8-GPU bench path rehearsed at world 8 on the one-GPU box.
    Everything the N>1 line holds is produced by the same code the driver's
    node runs -- the shard layout, the digest exchange and its checks (against
    torch.distributed and against libcurvecrc's CPU chain over the whole pool),
    the stream leg of every rank, the aggregate roofline over every rank's
    kernel time -- only the transport differs: RCCL refuses 8 ranks on one
    device, so the ranks agree on the torch.distributed exchange
    (pool.agreed_comm).  Reference exchange: CopysetNode::GetHash,
    copyset_node.cpp:925-975."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = _bench_world8(tmp_path, "bench_world8_gloo.log")
    assert "torch.distributed" in d["digest_exchange"]["path"]


@pytest.mark.timeout(420)
def test_bench_world8_native_exchange_over_stub_rccl(tmp_path):
    """The same world-8 run with the NATIVE digest exchange taken: a build of
    libcurvecrc linked against tests/native/rccl_stub.cpp (the seven RCCL calls
    pool.hip makes, over shared memory, synchronous) instead of librccl, which
    refuses 8 ranks on one GPU.  So cc_comm_init_timeout at nranks 8 (the id
    carried over torch.distributed), cc_pool_scan_dev's all-gather of every
    rank's partials into [rank][n] and the device XOR fold over 8 ranks,
    cc_comm_wait and the teardown all run as at the driver's N = 8, and the
    exchanged digests must equal torch.distributed's and the CPU chain's.
    RCCL's own transport is the one part not exercised."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    stub = os.path.join(root, "build", "stub", "libcurvecrc_stubrccl.so")
    main_lib = os.path.join(root, "curve_amd", "libcurvecrc.so")
    if not os.path.exists(stub) or os.path.getmtime(stub) < os.path.getmtime(main_lib) - 1:
        # missing or older than the library: build it now (make stubrccl; a test
        # build kept out of the product's default target)
        import subprocess
        r = subprocess.run(["make", "-s", "-C", os.path.join(root, "curve_amd", "csrc"), "stubrccl"],
                           capture_output=True, text=True)
        if r.returncode or not os.path.exists(stub):
            pytest.skip("stub-RCCL test build unavailable: " + (r.stderr or r.stdout)[-500:])
    import glob
    before = set(glob.glob("/dev/shm/ccrcclstub-*"))
    try:
        d = _bench_world8(tmp_path, "bench_world8_stubrccl.log", {"CURVE_AMD_LIB": stub})
    finally:  # a rank that died before its destroy leaves its segment behind: remove it
        for f in set(glob.glob("/dev/shm/ccrcclstub-*")) - before:
            try:
                os.unlink(f)
            except FileNotFoundError:
                pass
    ex = d["digest_exchange"]
    assert ex["path"].startswith("native RCCL"), ex
    assert ex["matches_torch_distributed"] is True and ex["matches_cpu_chain"] is True, ex
