#!/usr/bin/env python3
"""bench.py -- device-resident CRC32C over 4 KiB pages (Curve chunk-integrity path).

Workload (BASELINE.json configs[1]): per GPU, 1024 chunk files resident in HBM
(16 MiB data + 4 KiB metapage each, synthetic uniform-random bytes).  One
*step* is one pass of the scan hasher over that batch:
    page CRCs of every 4 KiB data page      (the hot kernel)
  + metapage CRCs, 4 MiB slice CRCs (ScanMap.crc), chunk data/file CRCs
  + per-copyset digest partials (XOR of shifted file CRCs)
  + at N>1: all_gather of the per-copyset partials over RCCL (the only exchange)
Multi-GPU: one process per GPU (torchrun), chunk ranges sharded by rank
(weak scaling: every rank holds its own 1024 chunks).

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
GiB = float(1 << 30)
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md
ALG_BYTES_PER_PAGE = 4100  # 4096 read + 4 written
N_COPYSETS = 64


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=10, help="untimed steps: the first ~7 launches after idle run slow while clocks ramp")
    p.add_argument("--clock-warm-ms", type=float, default=1000.0,
                   help="untimed warm-up floor in ms of estimated work (extra steps beyond --warmup; 0 = none)")
    p.add_argument("--chunks", type=int, default=1024, help="chunks per GPU")
    p.add_argument("--page-bytes", type=int, default=4096)
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline time budget (rank 0, N=1)")
    p.add_argument("--cpu-sample-chunks", type=int, default=256, help="CPU baseline sample: 16 MiB chunks (256 = 4 GiB)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-e2e", action="store_true")
    p.add_argument("--no-pmc", action="store_true", help="skip the live rocprofv3 traffic passes (use profiles/)")
    p.add_argument("--e2e-gib", type=float, default=1.0, help="pinned host buffer for the e2e leg")
    p.add_argument("--updates", type=int, default=65536, help="config-3 updates per batch")
    p.add_argument("--update-batches", type=int, default=10)
    p.add_argument("--reads", type=int, default=65536, help="verify-on-read leg: reads per batch (0 = skip)")
    p.add_argument("--stream-chunks", type=int, default=10000, help="config-4 stream leg (0 = skip)")
    p.add_argument("--stream-chunks-per-rank", type=int, default=2000, help="N>1: streamed chunks per rank")
    p.add_argument("--stream-distinct", type=int, default=10000,
                   help="N=1 stream leg: distinct pinned 16 MiB data chunks (10000 = every chunk distinct, 156 GiB of "
                        "pinned host memory; fewer if the host cannot spare that, see _host_chunk_budget)")
    p.add_argument("--file-chunks", type=int, default=128, help="datastore read-path leg (0 = skip)")
    p.add_argument("--file-passes", type=int, default=5, help="datastore read-path leg: passes per io-thread count")
    p.add_argument("--scan-op-threads", type=int, default=10,
                   help="scan-op leg: apply threads (wconcurrentapply.size, conf/chunkserver.conf:183; 0 = skip)")
    p.add_argument("--scan-op-calls", type=int, default=500, help="scan-op leg: ops per thread")
    p.add_argument("--wal-entries", type=int, default=65536, help="WAL replay leg: entries per batch (0 = skip)")
    p.add_argument("--no-numa-bind", action="store_true",
                   help="leave the CPU affinity alone (default: bind to the GPU's NUMA node, see bind_to_gpu_numa)")
    p.add_argument("--comm-timeout-ms", type=int, default=60000, help="N>1: bound on the native RCCL init")
    p.add_argument("--exchange-timeout-ms", type=int, default=120000,
                   help="N>1: bound on waiting for the steps' digest exchanges (a peer lost after init)")
    p.add_argument("--traffic-json", default=None, help="PMC traffic summary (default: newest profiles/traffic_*.json)")
    return p.parse_args()


def log(rank, *a):
    if rank == 0:
        print("[bench]", *a, flush=True)


def host_cores():
    """Threads this process may run on (the cpuset, not the machine: a GPU box
    hands each GPU a share of a larger host) and the cgroup CPU quota if any."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    return aff, quota


def _cpulist(text):
    cpus = set()
    for part in text.strip().split(","):
        if part:
            lo, _, hi = part.partition("-")
            cpus.update(range(int(lo), int(hi or lo) + 1))
    return cpus


def bind_to_gpu_numa(dev):
    """Run this rank's threads on the CPUs of the NUMA node its GPU hangs off
    (sysfs local_cpulist of the GPU's PCI function, within the CPUs this
    process may use), before any pinned buffer exists, so the rank's pinned
    staging and stream-leg chunks are placed, its chunk files' page cache is
    written, its reader threads run and its host-side CRC checks run next to
    its PCIe link.  N > 1: eight ranks' H2D streams otherwise cross the socket
    interconnect at random.  N = 1 too: unbound, the files leg (page cache ->
    pinned staging by the reader threads) measured 47.0 / 32.5 / 41.8 GiB/s in
    three processes on one box, bound 46.7 / 45.9 / 48.4; the pinned H2D legs
    are the same either way (profiles/numa_files_ab_r05.jsonl).  Every thread
    the process has at that point (the HIP runtime's included) is bound, and
    threads made afterwards inherit the mask.  Never fatal: reports what it did ("bound" false
    and why otherwise)."""
    try:
        p = torch.cuda.get_device_properties(dev)
        path = f"/sys/bus/pci/devices/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        node = int(open(path + "/numa_node").read())
        local = _cpulist(open(path + "/local_cpulist").read())
        allowed = os.sched_getaffinity(0)
        use = local & allowed
        if node < 0 or not use or use == allowed:
            return {"numa_node": node, "bound": False,
                    "why": "no NUMA node" if node < 0 else "no local CPU allowed" if not use else "already local"}
        # every thread of the process, not only this one: the HIP runtime's
        # threads already exist (started by the device query above) and keep
        # their own masks otherwise; threads made later inherit the mask
        tids = [int(t) for t in os.listdir("/proc/self/task")]
        bound = 0
        for tid in tids:
            try:
                os.sched_setaffinity(tid, use)
                bound += 1
            except OSError:
                pass  # a thread that exited meanwhile
        return {"numa_node": node, "bound": True, "cpus": len(use), "of_allowed": len(allowed),
                "threads_bound": bound, "threads_seen": len(tids)}
    except Exception as e:  # report, never fail the run on it
        return {"bound": False, "why": repr(e)}


def cpu_baseline(pool, args, rank):
    """Reference CPU path restated (oracle, single-stream SSE4.2 crc32q as butil
    builds it, one CRC32(page, 4096) call per page) timed on this host over a
    DRAM-resident sample of the same workload: `--cpu-sample-chunks` 16 MiB
    chunks (default 256 = 4 GiB, far above the L3) copied from HBM.  Timed at
    1 thread and at every core this process may use (page-partitioned), plus a
    cache-resident microbench of libcurvecrc's own CPU primitive (VPCLMULQDQ
    fold where the CPU has it, else 3-way crc32q; `libcurvecrc_path` says which)
    against the single-stream oracle at 4 KiB and 64 KiB per call."""
    import ctypes
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    sample_chunks = min(args.cpu_sample_chunks, pool.n)
    host = pool.data[:sample_chunks].cpu().numpy()
    pages_per_chunk = pool.chunk_size // args.page_bytes
    dev_crcs = pool.page_crcs[: sample_chunks * pages_per_chunk].cpu().numpy().view(np.uint32)
    aff, quota = host_cores()
    threads_all = max(1, aff if quota is None else min(aff, int(quota)))
    res = {}
    for threads, budget in ((1, args.cpu_seconds), (threads_all, max(2.0, args.cpu_seconds / 2))):
        nbytes, t0 = 0, time.perf_counter()
        while True:
            want = O.page_crcs(host, args.page_bytes, threads=threads)
            nbytes += host.nbytes
            el = time.perf_counter() - t0
            if el >= budget:
                break
        res[threads] = (nbytes / GiB / el, nbytes, el)
    parity = bool((want == dev_crcs).all())
    # cache-resident per-call rate: the product's crc32c_extend vs the oracle's
    # single stream, both driven by the same C loop (no Python per call)
    from curve_amd import _lib
    L, P = O.lib(), _lib.lib()
    L.oc_time_calls.restype = ctypes.c_double
    L.oc_time_calls.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_void_p]
    buf = host[0, : 1 << 16]
    micro = {}
    for n in (4096, 65536):
        for name, fn in (("oracle_single_stream", L.oc_crc32c_sse42), ("libcurvecrc", P.crc32c_extend)):
            it = max(1, (2 << 30) // n)  # 2 GiB per measurement
            t = L.oc_time_calls(ctypes.cast(fn, ctypes.c_void_p).value, buf.ctypes.data, n, it, None)
            micro[f"{name}_{n // 1024}KiB_GiBps"] = round(it * n / GiB / t, 2)
    micro["libcurvecrc_path"] = cpu_primitive_path()
    v1, nb1, el1 = res[1]
    vN, nbN, elN = res[threads_all]
    return {
        "value": round(v1, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
        "sample": f"{sample_chunks} x 16 MiB chunks ({sample_chunks * pool.chunk_size / GiB:.1f} GiB, DRAM-resident) "
                  f"copied from HBM, CRC32(page, {args.page_bytes}) per page, {nb1 / GiB:.1f} GiB hashed in {el1:.1f} s "
                  "(oracle/crc32c_oracle.c oc_crc32c_sse42, single-stream crc32q as butil builds it)",
        "all_cores": {"value": round(vN, 3), "cores": threads_all, "seconds": round(elN, 2),
                      "hashed_GiB": round(nbN / GiB, 1), "affinity_cpus": aff, "cgroup_cpu_quota": quota,
                      "machine_cpus": os.cpu_count()},
        "parity_vs_device": parity,
        "cpu_model": cpu_model(),
        "per_call_cache_resident": micro,
    }


def cpu_primitive_path():
    """Which loop crc32c_cpu.cpp's raw_update runs here: its run-time checks
    (avx512f + vpclmulqdq, CURVE_CRC_NO_FOLD unset; the split on AMD unless
    CURVE_CRC_FOLD_SPLIT says otherwise) restated from /proc/cpuinfo."""
    flags, vendor = set(), ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("vendor_id") and not vendor:
                    vendor = line.split(":", 1)[1].strip()
                if line.startswith("flags"):
                    flags = set(line.split(":", 1)[1].split())
                    break
    except OSError:
        pass
    off = os.environ.get("CURVE_CRC_NO_FOLD", "")
    if not ({"avx512f", "vpclmulqdq", "pclmulqdq"} <= flags) or (off and off != "0"):
        return "3-way crc32q"
    sp = os.environ.get("CURVE_CRC_FOLD_SPLIT", "")
    split = sp != "0" if sp else vendor == "AuthenticAMD"
    return ("vpclmulqdq fold (>= 256 B) + crc32q split (>= 6016 B)" if split
            else "vpclmulqdq fold (>= 256 B)")


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def e2e_leg(args, dev):
    """Host-resident input (pinned, as chunk files pread into pinned buffers):
    cc_page_crc_host = pinned H2D + kernel + D2H of CRCs, 2-slot overlap."""
    from curve_amd import crc as C
    nb = int(args.e2e_gib * GiB) // args.page_bytes * args.page_bytes
    h = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    h.random_(0, 256)
    a = h.numpy()
    C.page_crc_host(a, args.page_bytes)  # warm (staging alloc)
    t0, reps = time.perf_counter(), 0
    while time.perf_counter() - t0 < 2.0:
        C.page_crc_host(a, args.page_bytes)
        reps += 1
    el = time.perf_counter() - t0
    return round(reps * nb / GiB / el, 2)


def _scan_op_lib():
    import ctypes
    L = ctypes.CDLL(os.path.join(ROOT, "curve_amd", "host", "libscanop_bench.so"))
    L.sob_run.restype = ctypes.c_int
    L.sob_run.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                          ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    return L


SCAN_OP_MODES = {"cpu": 0, "gpu": 1, "routed": 2}


def run_scan_ops(bufs, offs, lens, calls, mode):
    """curve_amd/host/scan_op_bench.cpp sob_run: thread t (one per buffer) runs
    `calls` ops over bufs[t], op i = (offs[i % n], lens[i % n]); mode "cpu"
    (crc32c_value), "gpu" (cc_page_crc_host + cc_fold_host) or "routed"
    (cchost::ScanOpCrc).  Returns (rc, latency us [t, i], crcs [t, i], wall s,
    summed calling-thread CPU s); run_scan_ops.last_process_cpu_s = the whole
    process's CPU s over the run (HIP runtime threads included, and the
    launching thread's spin while it waits for the start)."""
    import ctypes
    L = _scan_op_lib()
    t = len(bufs)
    ptrs = (ctypes.c_void_p * t)(*[b.ctypes.data for b in bufs])
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    lat = np.zeros(t * calls, dtype=np.float64)
    crcs = np.zeros(t * calls, dtype=np.uint32)
    out = np.zeros(3, dtype=np.float64)
    rc = L.sob_run(t, ptrs, offs.ctypes.data, lens.ctypes.data, len(offs), calls, SCAN_OP_MODES[mode],
                   lat.ctypes.data, crcs.ctypes.data, out.ctypes.data)
    run_scan_ops.last_process_cpu_s = float(out[2])
    return rc, lat.reshape(t, calls), crcs.reshape(t, calls), float(out[0]), float(out[1])


def scan_op_leg(args):
    """Row f1 at the reference's own call shape: ScanChunkRequest::OnApply hashes
    ONE scan op per raft-applied request -- the 4 KiB metapage or one 4 MiB data
    slice, `crc = CRC32(readBuffer, size)` (op_request.cpp:776-794, :847) -- on
    the write apply pool, wconcurrentapply.size = 10 threads
    (conf/chunkserver.conf:183, op_request.cpp:179-187); a 16 MiB chunk is 5 ops
    (scan_manager_test.cpp:107-142).  Here 1 and 10 native threads (no
    interpreter between calls) each run a chunk file's 5 ops in turn over a
    pinned chunk file of their own, per call: the CPU primitive crc32c_value
    (the drop-in for CRC32), cc_page_crc_host + cc_fold_host,
    and the routed call cchost::ScanOpCrc (metapage on the CPU, slices on the
    GPU).  Every op's CRC is checked against the CPU primitive's.  Then one
    thread's per-call latency by op size, CPU vs GPU, for the size cutoff."""
    T = args.scan_op_threads
    calls = args.scan_op_calls
    file_bytes = 4096 + (16 << 20)
    hs = [torch.empty(file_bytes, dtype=torch.uint8, pin_memory=True).random_(0, 256) for _ in range(T)]
    bufs = [h.numpy() for h in hs]
    offs = [0] + [4096 + k * (4 << 20) for k in range(4)]
    lens = [4096] + [4 << 20] * 4
    op_bytes = np.array(lens * (calls // len(lens) + 1))[:calls]
    # the CPU primitive's CRC of every op of every thread's file: the check
    rc, _, c0, _, _ = run_scan_ops(bufs, offs, lens, len(offs), "cpu")
    assert rc == 0
    want = c0
    res = {"threads": {}, "ops_per_thread": calls,
           "op_mix": "per chunk file: 4 KiB metapage + 4 x 4 MiB slices (5 ScanChunkRequests)"}
    for nt in sorted({1, T}):
        per = {}
        for mode in ("cpu", "gpu", "routed"):
            run_scan_ops(bufs[:nt], offs, lens, 2 * len(offs), mode)  # warm: lanes, staging, pages
            rc, lat, crcs, wall, cpu_s = run_scan_ops(bufs[:nt], offs, lens, calls, mode)
            ok = rc == 0 and bool(all((crcs[t][: calls] == np.resize(want[t], calls)).all() for t in range(nt)))
            total = float(op_bytes.sum()) * nt
            sl = lat[:, op_bytes == (4 << 20)].ravel()
            mp = lat[:, op_bytes == 4096].ravel()
            per[mode] = {"agg_GiBps": round(total / GiB / wall, 2),
                         "slice_us_p50": round(float(np.percentile(sl, 50)), 1),
                         "slice_us_p99": round(float(np.percentile(sl, 99)), 1),
                         "metapage_us_p50": round(float(np.percentile(mp, 50)), 2),
                         "metapage_us_p99": round(float(np.percentile(mp, 99)), 2),
                         "cpu_s_per_GiB": round(cpu_s / (total / GiB), 4),
                         "process_cpu_s_per_GiB": round(run_scan_ops.last_process_cpu_s / (total / GiB), 4),
                         "crc_ok": ok, "rc": rc}
        res["threads"][str(nt)] = per
    # one thread's per-call latency by size (the cutoff): median of `n` calls
    sweep = {}
    for size in (4096, 16384, 65536, 262144, 512 << 10, 1 << 20, 2 << 20, 4 << 20, 16 << 20):
        row = {}
        for mode in ("cpu", "gpu"):
            n = 64 if size >= (4 << 20) else 200
            run_scan_ops(bufs[:1], [4096], [size], 4, mode)
            rc, lat, crcs, _, cpu_s = run_scan_ops(bufs[:1], [4096], [size], n, mode)
            row[mode + "_us_p50"] = round(float(np.median(lat)), 2) if rc == 0 else None
            row[mode + "_thread_cpu_us_per_call"] = round(cpu_s / n * 1e6, 2)
            row[mode + "_process_cpu_us_per_call"] = round(run_scan_ops.last_process_cpu_s / n * 1e6, 2)
            row[mode + "_crc"] = int(crcs[0, 0])
        row["crc_ok"] = row.pop("cpu_crc") == row.pop("gpu_crc")
        sweep[str(size)] = row
    res["latency_by_size_1thread"] = sweep
    faster = [int(k) for k, r in sweep.items() if r["gpu_us_p50"] and r["gpu_us_p50"] < r["cpu_us_p50"]]
    res["gpu_faster_per_call_from_bytes"] = min(faster) if faster else None
    cheaper = [int(k) for k, r in sweep.items()
               if r["gpu_process_cpu_us_per_call"] < r["cpu_process_cpu_us_per_call"]]
    res["gpu_cheaper_in_process_cpu_from_bytes"] = min(cheaper) if cheaper else None
    # the reference's own buffer kind: `new char[size]` (pageable), 10 threads
    pg = [np.random.default_rng(t).integers(0, 256, file_bytes, dtype=np.uint8) for t in range(T)]
    run_scan_ops(pg, offs, lens, 2 * len(offs), "gpu")
    rc, lat, _, wall, cpu_s = run_scan_ops(pg, offs, lens, calls, "gpu")
    total = float(op_bytes.sum()) * T
    res["pageable_gpu"] = {"threads": T, "agg_GiBps": round(total / GiB / wall, 2),
                           "slice_us_p50": round(float(np.percentile(lat[:, op_bytes == (4 << 20)], 50)), 1),
                           "cpu_s_per_GiB": round(cpu_s / (total / GiB), 4),
                           "process_cpu_s_per_GiB": round(run_scan_ops.last_process_cpu_s / (total / GiB), 4),
                           "rc": rc}
    res["path"] = ("curve_amd/host/scan_op_bench.cpp sob_run: native threads; gpu = cc_page_crc_host (a lane of its "
                   "own per concurrent caller: engine.hip page_crc_lane) + cc_fold_host")
    return res


def _host_chunk_budget(want, margin=32 << 30):
    """How many 16 MiB chunks of pinned host memory this process can take: `want`,
    or fewer when MemAvailable or the cgroup's memory limit (less its current
    use) minus `margin` is smaller -- never below min(64, want)."""
    from curve_amd import crc as C
    free = None
    try:
        for line in open("/proc/meminfo"):
            if line.startswith("MemAvailable:"):
                free = int(line.split()[1]) * 1024
    except OSError:
        pass
    for lim_f, cur_f in (("/sys/fs/cgroup/memory.max", "/sys/fs/cgroup/memory.current"),
                         ("/sys/fs/cgroup/memory/memory.limit_in_bytes", "/sys/fs/cgroup/memory/memory.usage_in_bytes")):
        try:
            lim = open(lim_f).read().strip()
            if lim != "max" and int(lim) < (1 << 60):
                room = int(lim) - int(open(cur_f).read().strip())
                free = room if free is None else min(free, room)
            break
        except (OSError, ValueError):
            continue
    if free is None:
        return want
    return max(min(64, want), min(want, (free - margin) // C.CHUNK_SIZE))


def _stream_sources(n, pool_n, rank=0, dev=None):
    """`pool_n` distinct pinned 16 MiB data chunks (re-referenced round robin
    when fewer than n: 10,000 distinct chunks take 156 GiB of host RAM) and `n`
    DISTINCT pinned metapages (sn = global chunk index), so every chunk FILE --
    metapage || data -- and its file CRC differ.  The data are random bytes
    made on the device (`dev`) 1 GiB at a time and copied down (a CPU random
    fill of 16 GiB takes tens of seconds)."""
    from curve_amd import crc as C
    from curve_amd.chunkfile import ChunkFileMetaPage
    data = torch.empty((pool_n, C.CHUNK_SIZE), dtype=torch.uint8, pin_memory=True)
    if dev is None:
        data.random_(0, 256)
    else:
        step = 64
        tmp = torch.empty((min(step, pool_n), C.CHUNK_SIZE), dtype=torch.uint8, device=dev)
        for k in range(0, pool_n, step):
            m = min(step, pool_n - k)
            tmp[:m].random_(0, 256)
            data[k:k + m].copy_(tmp[:m])
        torch.cuda.synchronize(dev)
        del tmp
    meta = torch.zeros((n, C.META_PAGE_SIZE), dtype=torch.uint8, pin_memory=True)
    mn = meta.numpy()
    for i in range(n):
        mn[i] = np.frombuffer(ChunkFileMetaPage(sn=rank * n + i + 1).encode(), dtype=np.uint8)
    dn = data.numpy()
    return dn, mn, [(mn[i], dn[i % pool_n]) for i in range(n)]


def _stream_expected(dn, mn, n, pool_n, lay, lo):
    """Expected CRCs of the stream from libcurvecrc's CPU primitive (not the
    oracle): slice CRCs of the distinct data chunks, every metapage CRC, file
    CRC = combine(metapage, data, 16 MiB), digest = XOR of shifted file CRCs."""
    from curve_amd import crc as C
    S = C.CHUNK_SIZE // C.SCAN_SIZE
    sl = np.array([[C.CRC32(dn[k][j * C.SCAN_SIZE:(j + 1) * C.SCAN_SIZE]) for j in range(S)] for k in range(pool_n)],
                  dtype=np.uint32)
    dc = np.empty(pool_n, dtype=np.uint32)
    for k in range(pool_n):  # chunk data CRC = the slices chained
        c = int(sl[k][0])
        for j in range(1, S):
            c = C.combine(c, int(sl[k][j]), C.SCAN_SIZE)
        dc[k] = c
    mc = np.array([C.CRC32(mn[i]) for i in range(n)], dtype=np.uint32)
    fc = np.array([C.combine(int(mc[i]), int(dc[i % pool_n]), C.CHUNK_SIZE) for i in range(n)], dtype=np.uint32)
    dig = np.zeros(lay.n_groups, dtype=np.uint32)
    for i in range(n):
        dig[lay.group[lo + i]] ^= C.shift(int(fc[i]), lay.after_bytes[lo + i])
    return mc, sl, fc, dig


def cpu_digest_check(pool, lay, lo, n, digest, dist_, dev, sample=(0, 37)):
    """Copysets `sample` of the pool's digests, recomputed on the host: every
    rank hashes its own chunk files of those copysets with libcurvecrc's CPU
    primitive (file CRC = combine(metapage CRC, data CRC, 16 MiB), shifted by
    the bytes after the file in its copyset's sorted-name chain) and the partials
    are XOR-reduced over the ranks.  Returns {"copysets", "ok"} (same on every rank)."""
    from curve_amd import crc as C
    from curve_amd.pool import reduce_digests
    part = np.zeros(lay.n_groups, dtype=np.uint32)
    files = 0
    for i in range(n):
        gi = lo + i
        if lay.group[gi] not in sample:
            continue
        m = pool.meta[i].cpu().numpy()
        d = pool.data[i].cpu().numpy()
        fc = C.combine(C.CRC32(m), C.CRC32(d), C.CHUNK_SIZE)
        part[lay.group[gi]] ^= C.shift(fc, lay.after_bytes[gi])
        files += 1
    t = torch.from_numpy(part.view(np.int32)).to(dev)
    full = reduce_digests(t, dist_) if dist_ is not None else t
    got = digest.cpu().numpy().view(np.uint32)
    want = full.cpu().numpy().view(np.uint32)
    ok = bool(all(got[g] == want[g] for g in sample))
    return {"copysets": list(sample), "files_hashed_on_this_rank": files, "ok": ok,
            "by": "libcurvecrc CPU primitive over the chunk files' bytes, partials XOR-reduced over the ranks"}


def stream_leg(args):
    """BASELINE config 4: scan-service stream of `--stream-chunks` x 16 MiB chunk
    files from pinned host memory (as pread into pinned buffers would leave
    them): pipelined H2D + page kernel + fused epilogue per batch, ScanMap
    slice CRCs, file CRCs AND the per-copyset digests (100 chunks per copyset)
    computed on the device -- ONE cc_scan_host_digest call.  Every output is
    checked afterwards against libcurvecrc's CPU primitive."""
    from curve_amd import crc as C
    from curve_amd.pool import copyset_layout
    n, per = args.stream_chunks, 100
    pool_n = _host_chunk_budget(max(1, min(args.stream_distinct, n)))
    dn, mn, chunks = _stream_sources(n, pool_n, dev=torch.device("cuda", 0))
    lay = copyset_layout(list(range(n)), [i // per for i in range(n)], [C.CHUNK_SIZE + C.META_PAGE_SIZE] * n)
    C.scan_host(chunks[:8])  # warm (staging)
    t0 = time.perf_counter()
    mc, sc, fc, dig = C.scan_host(chunks, after_bytes=lay.after_bytes, group=lay.group, n_groups=lay.n_groups)
    el = time.perf_counter() - t0
    w_mc, w_sl, w_fc, w_dig = _stream_expected(dn, mn, n, pool_n, lay, 0)
    bad = {"meta": int((mc != w_mc).sum()), "slices": int((sc != w_sl[np.arange(n) % pool_n]).sum()),
           "files": int((fc != w_fc).sum()), "digests": int((dig != w_dig).sum())}
    out = {"chunks": n, "GiBps_e2e": round(n * (C.CHUNK_SIZE + C.META_PAGE_SIZE) / GiB / el, 2),
           "seconds": round(el, 3), "copysets": lay.n_groups, "scan_maps": int(sc.size + mc.size),
           "digest": "device (fused epilogue, cc_scan_host_digest)",
           "crc_check": {"vs": "libcurvecrc CPU primitive", "mismatches": bad, "ok": not any(bad.values())},
           "source": f"{n} distinct pinned metapages + {pool_n} distinct pinned 16 MiB data chunks "
                     f"({pool_n * C.CHUNK_SIZE / GiB:.0f} GiB" + (", re-referenced round robin)" if pool_n < n else ")")}
    assert out["crc_check"]["ok"], f"stream leg CRC mismatch: {bad}"
    return out


def stream_all_ranks_leg(args, rank, world, dev):
    """Config 5 end to end: each rank streams `--stream-chunks-per-rank` chunk
    files from pinned host memory through cc_scan_host_digest on its own GPU
    (file CRCs + per-copyset digest partials on the device), then joins the
    digest exchange; aggregate = all ranks' bytes / the slowest rank's time
    (barrier on both sides).  Rank 0 checks the exchanged digests against the
    CPU primitive over every rank's chunks."""
    from curve_amd import crc as C
    from curve_amd.pool import copyset_layout, reduce_digests
    n, per = args.stream_chunks_per_rank, 100
    pool_n = min(64, n)  # distinct pinned 16 MiB chunks per rank (1 GiB at most)
    total = n * world
    lay = copyset_layout(list(range(total)), [i // per for i in range(total)],
                         [C.CHUNK_SIZE + C.META_PAGE_SIZE] * total)
    dn, mn, chunks = _stream_sources(n, pool_n, rank)
    lo = rank * n
    C.scan_host(chunks[:4])  # warm
    dist.barrier()
    t0 = time.perf_counter()
    *_, part = C.scan_host(chunks, after_bytes=lay.after_bytes[lo:lo + n], group=lay.group[lo:lo + n],
                           n_groups=lay.n_groups)
    dig = reduce_digests(torch.from_numpy(part.view(np.int32)).to(dev), dist)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64,
                     device="cpu" if dist.get_backend() == "gloo" else dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    # untimed check: every rank's expected partial, XORed, == the exchanged digests
    *_, w_part = _stream_expected(dn, mn, n, pool_n, lay, lo)
    want = reduce_digests(torch.from_numpy(w_part.view(np.int32)).to(dev), dist)
    ok = bool((dig.cpu().numpy().view(np.uint32) == want.cpu().numpy().view(np.uint32)).all())
    return {"chunks_per_rank": n, "ranks": world, "seconds_max_rank": round(el, 3),
            "GiBps_e2e_aggregate": round(total * (C.CHUNK_SIZE + C.META_PAGE_SIZE) / GiB / el, 2),
            "copysets": lay.n_groups, "digests": int(dig.numel()), "digest_check_ok": ok,
            "source": "pinned host chunk files per rank; cc_scan_host_digest per rank + digest exchange"}


def files_leg(args):
    """The datastore read path: `--file-chunks` real chunk files (metapage ||
    16 MiB data) in a temp directory (page-cache / tmpfs resident, as a hot
    copyset would be), read AND scanned by the engine itself (cc_scan_files:
    native pread by io threads into pinned staging, overlapped with H2D +
    kernels).  Reports whole-file GiB/s per io-thread count."""
    import shutil
    import tempfile
    from curve_amd import crc as C
    from curve_amd.chunkfile import ChunkFileMetaPage
    n = args.file_chunks
    d = tempfile.mkdtemp(prefix="cc_files_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        rng = np.random.default_rng(3)
        body = rng.integers(0, 256, C.CHUNK_SIZE + C.META_PAGE_SIZE, dtype=np.uint8)
        paths = []
        for i in range(n):
            # a valid metapage (sn = i + 1: every file distinct), random data
            body[:C.META_PAGE_SIZE] = np.frombuffer(ChunkFileMetaPage(sn=i + 1).encode(C.META_PAGE_SIZE), dtype=np.uint8)
            p = os.path.join(d, f"chunk_{i}")
            body.tofile(p)
            paths.append(p)
        out = {"files": n, "file_bytes": C.CHUNK_SIZE + C.META_PAGE_SIZE, "source": "tmp dir, page-cache resident"}
        C.scan_files(paths[:4])  # warm
        fb = n * (C.CHUNK_SIZE + C.META_PAGE_SIZE) / GiB
        # median of --file-passes passes per io-thread count, the counts
        # interleaved pass by pass (a slow stretch of the box hits every count);
        # io_threads=0 is the engine's default (from the affinity and cgroup quota)
        counts = (0, 4, 8, 16)
        runs = {t: [] for t in counts}
        for _ in range(args.file_passes):
            for t in counts:
                t0 = time.perf_counter()
                st, _, _, _ = C.scan_files(paths, io_threads=t)
                el = time.perf_counter() - t0
                assert (st == 0).all()
                runs[t].append(fb / el)
        for t in counts:
            key = "GiBps_default" if t == 0 else f"GiBps_io{t}"
            out[key] = round(float(np.median(runs[t])), 2)
            out[key + "_each"] = [round(x, 2) for x in runs[t]]
        out["default_io_threads"] = C.default_io_threads()
        out["passes"] = args.file_passes
        # an integrity job's check of the same files against
        # their per-page CRC tables (cc_integrity_check: the reads as above, page
        # CRCs on the device, compared with the sidecar tables; the first pass
        # creates the tables, untimed)
        from curve_amd import integrity as I
        tables = [q + ".pcrc" for q in paths]
        first = I.check_files(paths, tables)
        assert all(r.status == 0 and r.table == "created" for r in first), first[:2]
        ic = []
        for _ in range(3):
            t0 = time.perf_counter()
            res = I.check_files(paths, tables)
            ic.append(fb / (time.perf_counter() - t0))
            assert all(r.status == 0 and r.bad_pages == 0 and r.table == "ok" for r in res), res[:2]
        out["integrity_check"] = {"GiBps": round(float(np.median(ic)), 2), "GiBps_each": [round(x, 2) for x in ic],
                                  "path": "cc_integrity_check: the files read by the engine's readers, page CRCs on "
                                          "the device, compared with their stored per-page CRC tables (0 bad pages)"}
        return out
    finally:
        shutil.rmtree(d, ignore_errors=True)


def warm_clock(fn, ms=1000.0):
    """Run `fn` back to back for about `ms` of wall time, untimed: after host-side
    setup the GPU has idled and its clock ramps back over ~10-30 ms of work (a
    kernel trace shows the first launches of a leg 5-25 % slow), and a fresh box
    needs about a second of sustained load to reach its steady rate -- every
    leg gets the main leg's floor (--clock-warm-ms).  It returns with two more
    calls enqueued and NOT waited for: the timed calls that follow then queue
    behind work, so the first one's begin event is not recorded on an idle GPU
    that then waits for the host to submit its kernels (round 3: the first
    timed call of each leg ran 2-5 % long, 0.7072 vs 0.6644-0.6781 ms for WAL
    replay)."""
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
    fn()
    fn()


def partial_write_leg(pool, args):
    """BASELINE config 3: client partial writes into the resident 1024-chunk pool.
    Per batch a write LOG of U random updates (size uniform in [512, 4096] B,
    offset uniform and unaligned; ~54 % straddle two pages -- ~101,000 touched
    pages a batch, ~1 % of them with more than one piece; overlapping entries
    apply in log order) and its data, both resident in HBM as the pool is: one
    cc_apply_log_dev call groups the pieces by page on the device (a hash
    table, no sort), applies them and rehashes every touched page in place.  Timed with HIP events on the
    launch stream; `wall_ms_incl_log_upload` adds the host->device copy of the
    log records (C.apply_updates, the host-log entry point)."""
    from curve_amd import crc as C
    dev = pool.data.device
    U = args.updates
    rng = np.random.default_rng(0xC3)
    pool_bytes = pool.data.numel()
    src = torch.empty(U * 4096, dtype=torch.uint8, device=dev).random_(0, 256)
    flat = pool.data.view(-1)
    stream = torch.cuda.current_stream()
    logs, upd_bytes, touched = [], 0, 0
    for it in range(args.update_batches + 1):
        lens = rng.integers(512, 4097, U)
        dst = rng.integers(0, pool_bytes - 4096, U)
        src_off = rng.integers(0, U * 4096 - 4096, U)
        rec = C.log_records(dst, src_off, lens)
        logs.append((torch.from_numpy(rec.view(np.uint8)).to(dev), (dst, src_off, lens)))
        if it:
            p0, p1 = dst // 4096, (dst + lens - 1) // 4096
            touched += len(np.unique(np.concatenate([p0, p1])))
            upd_bytes += int(lens.sum())
    # warm: work buffer, and the clock ramp after the host-side setup
    warm_clock(lambda: C.apply_log(flat, pool.page_crcs, src, logs[0][0], U, 4096, 4096), args.clock_warm_ms)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in logs[1:]]
    for (d_log, _), (e0, e1) in zip(logs[1:], ev):
        e0.record(stream)
        C.apply_log(flat, pool.page_crcs, src, d_log, U, 4096, 4096)
        e1.record(stream)
    torch.cuda.synchronize()
    dev_ms = [a.elapsed_time(b) for a, b in ev]
    # the same batches as ONE queue (cc_apply_logs_dev: each page kernel also
    # groups the next batch in its tail, so only the queue's first batch pays the
    # grouping launch): re-applying the logs in order leaves the pool as it is.
    # Five queue calls enqueued back to back (each behind the previous one's
    # work), HIP events around each, ms per batch
    qb = [(src, d_log, U) for d_log, _ in logs[1:]]
    C.apply_logs(flat, pool.page_crcs, qb, 4096, 4096)  # warm (work buffer, table pair), not waited for
    ev_q = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
    for e0, e1 in ev_q:
        e0.record(stream)
        C.apply_logs(flat, pool.page_crcs, qb, 4096, 4096)
        e1.record(stream)
    torch.cuda.synchronize()
    q_each = [a.elapsed_time(b) / len(qb) for a, b in ev_q]
    q_ms = float(np.mean(q_each))
    # host-log entry point: the records cross PCIe first
    walls = []
    for _, (dst, src_off, lens) in logs[1:]:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        C.apply_updates(flat, pool.page_crcs, src, dst, src_off, lens, 4096)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
    # delta mode (cc_apply_log_delta_dev): the same logs again (re-applying a
    # log is idempotent), the stored CRCs updated by linearity from the touched
    # rows; afterwards every page must still verify against its bytes
    ev_d = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in logs[1:]]
    for _ in range(2):  # untimed, not waited for: the first timed call queues behind work (warm_clock)
        C.apply_log(flat, pool.page_crcs, src, logs[0][0], U, 4096, 4096, delta=True)
    for (d_log, _), (e0, e1) in zip(logs[1:], ev_d):
        e0.record(stream)
        C.apply_log(flat, pool.page_crcs, src, d_log, U, 4096, 4096, delta=True)
        e1.record(stream)
    # and the delta queue (cc_apply_logs_dev, delta = 1): three calls back to back
    ev_dq = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
    for e0, e1 in ev_dq:
        e0.record(stream)
        C.apply_logs(flat, pool.page_crcs, qb, 4096, 4096, delta=True)
        e1.record(stream)
    torch.cuda.synchronize()
    delta_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_d]))
    delta_q_ms = float(np.mean([a.elapsed_time(b) / len(qb) for a, b in ev_dq]))
    # the write log's access pattern alone (cc_apply_log_probe_dev): per log,
    # the log re-applied (untimed), then the same touched pages read -- covered
    # rows from the source -- and their dirty rows stored back, no table, no
    # CRC (idempotent right after the apply); HIP events around the probe only
    descs = [C.log_probe_descs(dst, so, ln) for _, (dst, so, ln) in logs[1:]]
    d_descs = [torch.from_numpy(d.view(np.uint8)).to(dev) for d in descs]
    pout = torch.empty(max(d.size for d in descs), dtype=torch.int32, device=dev)
    C.log_probe(flat, src, d_descs[-1], descs[-1].size, pout)  # the last log applied: idempotent warm call
    ev_p = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in descs]
    for (d_log, _), dd, d, (e0, e1) in zip(logs[1:], d_descs, descs, ev_p):
        C.apply_log(flat, pool.page_crcs, src, d_log, U, 4096, 4096)
        e0.record(stream)
        C.log_probe(flat, src, dd, d.size, pout)
        e1.record(stream)
    torch.cuda.synchronize()
    probe_each = [a.elapsed_time(b) for a, b in ev_p]
    probe_ms = float(np.mean(probe_each))
    # bytes the probe moves: 4 KiB read a page (rows from the page or the
    # source) + its dirty rows written
    probe_moved = float(np.mean([d.size * 4096 + 256 * int(np.unpackbits(np.ascontiguousarray(d["dirty"]).view(np.uint8)).sum())
                                 for d in descs]))
    cnt = C.page_verify(flat, pool.page_crcs, 4096)
    torch.cuda.synchronize()
    delta_ok = int(cnt[0]) == 0
    nb = len(dev_ms)
    ms = float(np.mean(dev_ms))
    # update bytes read + 4096 read and 4 written per touched page
    # (covered rows come from the source, not the page, so an update byte is
    # read once).  moved_2u: the round-5 figure, every update byte counted twice
    alg = (upd_bytes + touched * (4096 + 4)) / nb
    moved_2u = (2 * upd_bytes + touched * (4096 + 4)) / nb

    def frac(b, t_ms):
        return round(b / (t_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    return {"updates_per_batch": U, "batches": nb,
            "device_ms_per_batch": round(ms, 4),
            "ms_median": round(float(np.median(dev_ms)), 4),
            "ms_each": [round(x, 4) for x in dev_ms],
            "updates_per_s": round(U / (ms * 1e-3), 1),
            "touched_pages_per_batch": touched // nb,
            "alg_GBps": round(alg / (ms * 1e-3) / 1e9, 1),
            "alg_frac_of_hbm_peak": frac(alg, ms),
            "moved_frac_2u": frac(moved_2u, ms),
            "alg_bytes_per_batch": int(alg),
            "wall_ms_incl_log_upload": round(float(np.mean(walls)) * 1e3, 3),
            "frac_of_random_probe": round(probe_ms / ms, 4),
            "delta": {"device_ms_per_batch": round(delta_ms, 4),
                      "updates_per_s": round(U / (delta_ms * 1e-3), 1),
                      "alg_frac_of_hbm_peak": frac(alg, delta_ms),
                      "moved_frac_2u": frac(moved_2u, delta_ms),
                      "frac_of_random_probe": round(probe_ms / delta_ms, 4),
                      "queue_device_ms_per_batch": round(delta_q_ms, 4),
                      "queue_frac_of_random_probe": round(probe_ms / delta_q_ms, 4),
                      "all_pages_verify_after": delta_ok,
                      "path": "cc_apply_log_delta_dev: stored CRCs updated by linearity, touched rows read only"},
            "queue": {"batches_per_call": len(qb), "device_ms_per_batch": round(q_ms, 4),
                      "ms_each": [round(x, 4) for x in q_each],
                      "updates_per_s": round(U / (q_ms * 1e-3), 1),
                      "alg_frac_of_hbm_peak": frac(alg, q_ms),
                      "moved_frac_2u": frac(moved_2u, q_ms),
                      "frac_of_random_probe": round(probe_ms / q_ms, 4),
                      "path": "cc_apply_logs_dev: the batches as one queue; each batch's page kernel also groups "
                              "the next batch in its tail (one grouping launch a queue instead of one a batch)"},
            "random_probe": {"ms_per_batch": round(probe_ms, 4), "ms_median": round(float(np.median(probe_each)), 4),
                             "ms_each": [round(x, 4) for x in probe_each],
                             "pages_per_batch": int(np.mean([d.size for d in descs])),
                             "alg_frac_of_hbm_peak": frac(alg, probe_ms),
                             "moved_frac_2u": frac(moved_2u, probe_ms),
                             "moved_GBps": round(probe_moved / (probe_ms * 1e-3) / 1e9, 1),
                             "path": "cc_apply_log_probe_dev: the same touched pages read (covered rows from the "
                                     "source) and their dirty rows stored nt, write-log page-pass grid, no table, "
                                     "no CRC -- the ceiling of this access pattern"},
            "path": "cc_apply_log_dev: pieces grouped by page in a device hash table (one CAS per piece, no sort) + one wave per touched page",
            "note": "alg bytes (SURVEY 8d) = update bytes + 4100 x touched pages; moved_frac_2u = (2 x update "
                    "bytes + 4100 x touched pages) / t / 8 TB/s, the round-5 accounting; log + data resident in HBM"}


def read_verify_leg(pool, args):
    """Verify-on-read (the datastore read path, CSChunkFile::Read): batches of
    `--reads` random client reads of 4 KiB-128 KiB at page-aligned offsets
    (CheckRequestOffsetAndLength) over the resident pool; every touched page is
    rehashed and compared with its stored CRC (cc_verify_reads_dev).  Reads and
    CRC table resident in HBM; HIP events on the launch stream."""
    from curve_amd import crc as C
    dev = pool.data.device
    n, pb = args.reads, args.page_bytes
    flat = pool.data.view(-1)
    n_pages = flat.numel() // pb
    rng = np.random.default_rng(0xEAD)
    stream = torch.cuda.current_stream()
    pages, walls = 0, []
    bad = torch.zeros(n, dtype=torch.int32, device=dev)
    total = torch.zeros(1, dtype=torch.int64, device=dev)
    batches = []
    for it in range(11):
        npg = rng.integers(1, 33, n)
        first = rng.integers(0, n_pages - 32, n)
        # the batches of reads are resident before the timed calls, as the pool is
        d_reads = torch.from_numpy(np.stack([first * pb, npg * pb], axis=1).reshape(-1).astype(np.int64)).to(dev)
        batches.append((d_reads, first, npg))
        if it:
            pages += int(npg.sum())
    # untimed: work buffer, and the clock ramp after the host-side setup
    warm_clock(lambda: C.verify_read_records(flat, pool.page_crcs, batches[0][0], n, bad, total, pb),
               args.clock_warm_ms)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in batches[1:]]
    for (d_reads, _, _), (e0, e1) in zip(batches[1:], ev):
        e0.record(stream)
        C.verify_read_records(flat, pool.page_crcs, d_reads, n, bad, total, pb)
        e1.record(stream)
    torch.cuda.synchronize()
    assert int(total.item()) == 0, "clean pool flagged"
    ms = [a.elapsed_time(b) for a, b in ev]
    for _, first, npg in batches[1:6]:
        # host-record entry point (records cross PCIe inside the call)
        t0 = time.perf_counter()
        C.verify_reads(flat, pool.page_crcs, first * pb, npg * pb, pb)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
    t = float(np.mean(ms))
    per = pages / len(ms)
    # the access pattern's ceiling (cc_page_list_probe_dev): the same batches'
    # pages read in read order with everything else removed, verify-on-read's
    # grid and occupancy; events around each probe call, enqueued back to back
    lists = [torch.from_numpy(C.read_pages_list(first * pb, npg * pb, pb)).to(dev) for _, first, npg in batches[1:]]
    pout = torch.empty(max(x.numel() for x in lists), dtype=torch.int32, device=dev)
    C.page_list_probe(flat, lists[0], lists[0].numel(), pout)  # warm, not waited for
    ev_p = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in lists]
    for lst, (e0, e1) in zip(lists, ev_p):
        e0.record(stream)
        C.page_list_probe(flat, lst, lst.numel(), pout)
        e1.record(stream)
    torch.cuda.synchronize()
    probe_each = [a.elapsed_time(b) for a, b in ev_p]
    probe_ms = float(np.mean(probe_each))
    return {"reads_per_batch": n, "pages_per_batch": int(per), "ms_per_batch": round(t, 4),
            "ms_median": round(float(np.median(ms)), 4),
            "alg_frac_of_hbm_peak_at_median": round(per * (pb + 4) / (float(np.median(ms)) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "ms_each": [round(x, 4) for x in ms],
            "GiBps_verified": round(per * pb / GiB / (t * 1e-3), 1),
            "alg_frac_of_hbm_peak": round(per * (pb + 4) / (t * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "wall_ms_incl_host_records": round(float(np.mean(walls)) * 1e3, 3),
            "frac_of_run_probe": round(probe_ms / t, 4),
            "run_probe": {"ms_per_batch": round(probe_ms, 4), "ms_each": [round(x, 4) for x in probe_each],
                          "read_GBps": round(per * pb / (probe_ms * 1e-3) / 1e9, 1),
                          "path": "cc_page_list_probe_dev: the batch's pages read in read order, verify-on-read's "
                                  "grid and occupancy, no CRC, no stored CRCs -- the ceiling of this access pattern"},
            "note": "reads + pool + CRC table resident in HBM; one cc_verify_reads_dev call per batch "
                    "(count, scan, verify); alg bytes = 4100 per touched page"}


def wal_replay_leg(pool, args):
    """SURVEY §8f row 3, the raft WAL's data checksums on replay
    (CurveSegment::_load_entry, raftlog/curve_segment.cpp:307-371): entries laid
    out as CurveSegment::append writes them (28-byte header + data, padded to
    4 KiB, walAlignSize) back to back in HBM; data_real_len uniform in
    [1 KiB, 128 KiB] (client writes).  One cc_crc_ranges_dev call verifies the
    data CRC of every entry; the header walk stays on the host (curve_amd/wal.py).
    The synthetic segments are the resident pool's bytes (random), so the
    ranges are arbitrary-alignment views of HBM, as the WAL's are."""
    from curve_amd import crc as C
    dev = pool.data.device
    flat = pool.data.view(-1)
    n = args.wal_entries
    rng = np.random.default_rng(0x3A1)
    real = rng.integers(1024, (128 << 10) + 1, n).astype(np.uint64)
    slot = (28 + real + 4095) // 4096 * 4096          # header + data, padded to walAlignSize
    start = np.concatenate([[0], np.cumsum(slot)[:-1]]).astype(np.uint64) + 4096  # after the meta page
    if int(start[-1] + slot[-1]) > flat.numel():
        return {"skipped": "pool too small for the WAL batch"}
    offs = start + 28
    rec = np.empty((n, 2), dtype=np.uint64)
    rec[:, 0], rec[:, 1] = offs, real
    d_rec = torch.from_numpy(rec.view(np.uint8).reshape(-1)).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()
    L = C.lib()
    def call():
        C.check(L.cc_crc_ranges_dev(flat.data_ptr(), d_rec.data_ptr(), n, out.data_ptr(),
                                    C._stream_handle(stream)), "cc_crc_ranges_dev")

    warm_clock(call, args.clock_warm_ms)  # untimed: the clock ramp after the host-side setup (the main leg's floor)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
    for e0, e1 in ev:  # back to back, as a replay issues its segments
        e0.record(stream)
        call()
        e1.record(stream)
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) for a, b in ev]
    # spot check against the CPU primitive (crc32c_value, the product's own)
    got = C.as_u32(out)
    host = {int(i): flat[int(offs[i]):int(offs[i] + real[i])].cpu().numpy().tobytes() for i in (0, n // 2, n - 1)}
    spot = all(int(got[i]) == C.CRC32(b) for i, b in host.items())
    t = float(np.mean(ms))
    data = float(real.sum())
    return {"entries_per_batch": n, "data_bytes_per_batch": int(data), "ms_per_batch": round(t, 4),
            "ms_median": round(float(np.median(ms)), 4),
            "alg_frac_of_hbm_peak_at_median": round((data + 4 * n) / (float(np.median(ms)) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "ms_each": [round(x, 4) for x in ms],
            "entries_per_s": round(n / (t * 1e-3), 1), "GBps": round(data / (t * 1e-3) / 1e9, 1),
            "alg_frac_of_hbm_peak": round((data + 4 * n) / (t * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "spot_check_vs_cpu_primitive": spot,
            "note": "entry records resident in HBM; alg bytes = data bytes read + 4 B CRC written per entry"}


def live_traffic(gib):
    """HBM bytes per page-kernel launch measured in THIS run: two rocprofv3 PMC
    passes (FETCH_SIZE, then WRITE_SIZE: one counter group each, never combined
    with tracing), each over scripts/prof_page.py as a child process on the same
    pool geometry, under a KILL timeout.  gfx950 correction as
    MI355X_MICROARCH.md prescribes: bytes = FETCH_SIZE x 1024 x 2 + WRITE_SIZE x
    1024 (calibrated on this access pattern: profiles/probe_r01.jsonl).
    Returns (bytes or None, note)."""
    import csv
    import shutil
    import subprocess
    import tempfile
    if any(k.startswith("ROCPROF") for k in os.environ) or "rocprof" in os.environ.get("LD_PRELOAD", ""):
        return None, "this run is itself under a profiler (no PMC pass may nest inside a trace)"
    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(exe):
        return None, "rocprofv3 not found"
    tmp = tempfile.mkdtemp(prefix="cc_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    med = {}
    try:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, ctr)
            cmd = ["timeout", "-s", "KILL", "120", exe, "--pmc", ctr, "-d", d, "-o", "run", "--output-format", "csv",
                   "--", sys.executable, os.path.join(ROOT, "scripts", "prof_page.py"), "--n", "2", "--gib", str(gib)]
            r = subprocess.run(cmd, cwd=tmp, capture_output=True, text=True, timeout=150,
                               env=dict(os.environ, TMPDIR=tmp))
            if r.returncode != 0:
                return None, f"rocprofv3 --pmc {ctr} exited {r.returncode}"
            vals = []
            for root, _, files in os.walk(d):
                for fn in files:
                    if fn.endswith("counter_collection.csv"):
                        for row in csv.DictReader(open(os.path.join(root, fn))):
                            if "page_crc_kernel<16, 0>" in row["Kernel_Name"] and row["Counter_Name"] == ctr:
                                vals.append(float(row["Counter_Value"]))
            if not vals:
                return None, f"no {ctr} samples for the page kernel"
            med[ctr] = float(np.median(vals))
    except Exception as e:  # report, never lose the line
        return None, f"live PMC failed: {e!r}"
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return med["FETCH_SIZE"] * 1024 * 2 + med["WRITE_SIZE"] * 1024, \
        "live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over scripts/prof_page.py in this run"


def load_traffic(args):
    path = args.traffic_json
    if path is None:
        cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "traffic_*.json")))
        path = cands[-1] if cands else None
    if not path or not os.path.exists(path):
        return None, None
    with open(path) as f:
        t = json.load(f)
    return t.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)


def launch_ranks(args):
    """`--gpus N` is honoured whoever starts the bench: under torchrun (the
    driver's multi-GPU form) WORLD_SIZE must equal N; started plainly with
    N > 1, the bench starts one rank per GPU itself -- torch.distributed.run as
    a CHILD process, before this process touches the GPU -- and exits with its
    status."""
    import subprocess
    import sys
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            print(json.dumps({"error": f"--gpus {args.gpus} but WORLD_SIZE={ws}: refusing to report a "
                                       f"{ws}-rank run as {args.gpus} GPUs"}), flush=True)
            sys.exit(2)
        return
    if args.gpus <= 1:
        return
    import socket
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


TIMED = {}


def timed_steps(args, step, sync, world, rank, n, chunk, dist):
    """W untimed warm-up steps (plus the clock floor), then EXACTLY K timed
    steps bracketed by a barrier and a device sync on both sides.  Results in
    TIMED (el: seconds of this rank, clock_warm: extra untimed steps)."""
    for _ in range(args.warmup):
        step(None)
    # The GPU needs sustained load before it runs at its steady rate: launches
    # ramp 2.77 -> 2.51 ms over the first ~30 ms after idle, and the first
    # process on a fresh box stays ~4 % slow (2.57 ms a step) through 100 ms of
    # warm-up but settles at 2.47 ms after ~2.5 s of it.  The metric is the
    # steady state of a continuous scan, so when the W requested warm-up steps
    # are shorter than --clock-warm-ms of work, extra UNTIMED steps run up to
    # that, reported as "clock_warmup_steps".  The count follows from the
    # per-rank bytes only, so every rank runs the same number of steps (each
    # step holds a collective).  The timed region is still exactly K steps.
    est_ms = n * chunk / 6.5e12 * 1e3  # ~6.5 TB/s
    clock_warm = max(0, int(np.ceil(args.clock_warm_ms / est_ms)) - args.warmup) if args.warmup > 0 else 0
    for _ in range(clock_warm):
        step(None)
    sync()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    sync()
    if world > 1:
        dist.barrier()
    TIMED["el"] = time.perf_counter() - t0
    TIMED["clock_warm"] = clock_warm


def main():
    args = parse()
    launch_ranks(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; BENCH_DIST_BACKEND=gloo + more ranks than GPUs only to
    # rehearse the multi-rank flow on a 1-GPU box (the driver uses nccl = RCCL)
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if world > 1 and backend == "nccl" and ndev < int(os.environ.get("LOCAL_WORLD_SIZE", world)):
        raise SystemExit(f"{world} ranks need {world} GPUs, {ndev} visible (BENCH_DIST_BACKEND=gloo rehearses "
                         "the multi-rank flow on fewer)")
    local = local % max(1, ndev)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    numa = None if args.no_numa_bind else bind_to_gpu_numa(dev)
    if world > 1:
        # collectives outside the native exchange (barriers, timing all-reduces,
        # the torch.distributed digest path) are bounded by the group's timeout
        import datetime
        pg_timeout = datetime.timedelta(seconds=float(os.environ.get("BENCH_DIST_TIMEOUT_S", "600")))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=pg_timeout)
        else:
            dist.init_process_group(backend, timeout=pg_timeout)

    from curve_amd import crc as C
    from curve_amd.pool import agreed_comm, copyset_layout, pool_scan, reduce_digests, shard_range
    from curve_amd.scan import DevicePool

    pb = args.page_bytes
    chunk, meta_sz = C.CHUNK_SIZE, C.META_PAGE_SIZE
    n = args.chunks
    log(rank, f"world={world} chunks/gpu={n} ({n * chunk / GiB:.1f} GiB data per GPU)")
    data = torch.empty((n, chunk), dtype=torch.uint8, device=dev)
    data.random_(0, 256)
    meta = torch.zeros((n, meta_sz), dtype=torch.uint8, device=dev)
    meta[:, 0] = 2  # FORMAT_VERSION_V2 in the metapage's first byte
    meta[:, 1:9].random_(0, 256)
    first_id = rank * n
    ids = list(range(first_id, first_id + n))
    pool = DevicePool(data, meta, ids, page_bytes=pb)

    # copyset geometry over the WHOLE pool (all ranks): chunk id -> copyset id % 64,
    # chunk files named chunk_<id>, chained in std::sort name order per copyset
    total = n * world
    lay = copyset_layout(list(range(total)), [i % N_COPYSETS for i in range(total)],
                         [chunk + meta_sz] * total)
    lo, hi = shard_range(total, rank, world)
    assert (lo, hi) == (first_id, first_id + n)
    after = torch.tensor(lay.after_bytes[lo:hi], dtype=torch.int64, device=dev)
    group = torch.tensor(lay.group[lo:hi], dtype=torch.int32, device=dev)
    digest = torch.zeros(lay.n_groups, dtype=torch.int32, device=dev)
    after_mult = C.xpow8(after)  # static layout: shift multipliers computed once
    full_digest = [digest]

    stream = torch.cuda.current_stream()
    # the digest exchange at N>1: libcurvecrc's own RCCL communicator (what a
    # C++ chunkserver binds); torch.distributed only carries its 128-byte id.
    # Init is bounded (--comm-timeout-ms) and the ranks agree on ONE path: if
    # any rank's native init failed, every rank uses torch.distributed (a mix
    # would pair ncclAllGather with all_gather_into_tensor and hang).
    comm, comm_note = None, None
    if world > 1:
        comm, comm_note = agreed_comm(dist, device=dev, timeout_ms=args.comm_timeout_ms)
    # per timed step: one event pair around the page kernel, recorded inside the
    # native call on `stream` (created up front: the call re-records them)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for a, b in ev:
        a.record(stream)
        b.record(stream)
    # and one around each timed step's digest exchange at N > 1: HIP events
    # recorded inside the native call around the all-gather + XOR fold, or the
    # host wall of the torch.distributed exchange (reduce_digests; the step's
    # kernels drained first, so only the exchange is inside it)
    xev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)] if world > 1 else []
    for a, b in xev:
        a.record(stream)
        b.record(stream)
    x_host_ms = [0.0] * args.steps

    # failure injection (the reference's libfiu failpoints play this role): the
    # rank named here stops participating in the digest exchange after init, as
    # a rank whose peer link died would; its peers must give up at the bound
    # (--exchange-timeout-ms for the native exchange, the group timeout for
    # torch.distributed) and the run must end with an error line, not a hang
    skip_exchange = world > 1 and os.environ.get("CC_INJECT_SKIP_EXCHANGE_RANK", "") == str(rank)

    def step(k):
        # ONE C call: page CRCs + metapage CRCs + fused epilogue (slice CRCs,
        # file CRCs, digest partials) + the RCCL digest exchange (cc_pool_scan_dev)
        pool_scan(pool, after_mult, group, digest, comm=None if skip_exchange else comm, stream=stream,
                  events=ev[k] if k is not None else None,
                  exchange_events=xev[k] if (k is not None and xev) else None)
        if world > 1 and comm is None and not skip_exchange:
            if k is not None:
                stream.synchronize()
                t0 = time.perf_counter()
            full_digest[0] = reduce_digests(digest, dist)
            if k is not None:
                stream.synchronize()
                x_host_ms[k] = (time.perf_counter() - t0) * 1e3

    def sync():
        # the steps' exchanges complete, or the run ends: cc_comm_wait polls the
        # stream and the communicator against a deadline and aborts it when a
        # peer is gone (a plain synchronize would wait forever)
        if comm is not None:
            comm.wait(stream, args.exchange_timeout_ms)
        torch.cuda.synchronize()

    def fail(e):
        # one JSON error line -- rank 0's on stdout (the line the driver reads),
        # every other rank's on stderr (ranks share the launcher's stdout: two
        # lines written at once could interleave into one unparsable line) --
        # then leave at once: no barrier, no teardown that could wait for the
        # lost peer
        line = json.dumps({"error": f"rank {rank}: digest exchange failed: {e}", "n_gpus": world,
                           "metric": "GiB/s CRC32C over 4KiB pages (device-resident) + % HBM roofline, 1/2/4/8 GPU",
                           "value": None})
        print(line, file=sys.stdout if rank == 0 else sys.stderr, flush=True)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(3)

    try:
        timed_steps(args, step, sync, world, rank, n, chunk, dist)
    except (C.CurveCrcError, RuntimeError) as e:
        if world == 1:
            raise
        fail(e)
    el = TIMED["el"]
    clock_warm = TIMED["clock_warm"]
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    digest_check = None
    if world > 1 and comm is not None:
        # untimed cross-check: the native RCCL digests == torch.distributed's
        native = digest.clone()
        local = torch.zeros_like(digest)
        pool_scan(pool, after_mult, group, local, comm=None, stream=stream)
        digest_check = bool(torch.equal(native, reduce_digests(local, dist)))
    final_digest = full_digest[0] if (world > 1 and comm is None) else digest
    kern_each = [a.elapsed_time(b) for a, b in ev]
    kern_ms = float(np.mean(kern_each))
    # every rank's mean page-kernel time: the aggregate roofline is set by the slowest
    rank_kern = [kern_ms]
    if world > 1:
        kt = torch.tensor([kern_ms], dtype=torch.float64, device="cpu" if backend == "gloo" else dev)
        ga = torch.empty(world, dtype=torch.float64, device=kt.device)
        dist.all_gather_into_tensor(ga, kt)
        rank_kern = [float(x) for x in ga.cpu().tolist()]

    # verify pass (after the timed region, before any host-side work that idles
    # the GPU): every page must match.  The clock floor first (the gather above
    # and the host sync leave the GPU idle; round 4 timed the verify pass right
    # after a host CRC check and read the clock ramp: 5,104 vs ~6,400 GiB/s),
    # then 5 calls back to back, each between its own event pair.
    cnt = torch.tensor([0, -1], dtype=torch.int64, device=dev)
    warm_clock(lambda: C.page_verify(pool.data, pool.page_crcs, pb, counters=cnt), min(args.clock_warm_ms, 500.0))
    vev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
    for ve0, ve1 in vev:
        ve0.record(stream)
        C.page_verify(pool.data, pool.page_crcs, pb, counters=cnt)
        ve1.record(stream)
    torch.cuda.synchronize()
    verify_each = [a.elapsed_time(b) for a, b in vev]
    verify_ms = float(np.mean(verify_each))
    bad = int(cnt[0].item())

    # measured read ceiling of THIS device: pure nt read of the same 16 GiB, same stream
    sink = torch.empty(2 * 1024 * 16, dtype=torch.int32, device=dev)
    probe_ms = []
    for r in range(6):
        pe0, pe1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        pe0.record(stream)
        C.hbm_read_probe(pool.data, sink)
        pe1.record(stream)
        torch.cuda.synchronize()
        if r:
            probe_ms.append(pe0.elapsed_time(pe1))
    probe_gbs = pool.data.numel() / (float(np.mean(probe_ms)) * 1e-3) / 1e9
    # the page kernel itself with its CRC arithmetic removed (same tiles, prefetch
    # ring, dynamic tail, loads and CRC-sized stores): the ceiling for THIS schedule
    lo_out = torch.empty(pool.data.numel() // 4096, dtype=torch.int32, device=dev)
    lo_ms = []
    for r in range(6):
        pe0, pe1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        pe0.record(stream)
        C.page_load_probe(pool.data, lo_out, stream=stream)
        pe1.record(stream)
        torch.cuda.synchronize()
        if r:
            lo_ms.append(pe0.elapsed_time(pe1))
    del lo_out
    load_only_gbs = pool.data.numel() // 4096 * ALG_BYTES_PER_PAGE / (float(np.mean(lo_ms)) * 1e-3) / 1e9

    # untimed, every N, after the device timings above (it idles the GPU for tens
    # of ms): the exchanged digests of two copysets == the sorted-name chain of
    # those copysets' files over the WHOLE pool, from the bytes by libcurvecrc's
    # CPU primitive (each rank hashes its own files on the host; partials
    # XOR-reduced over torch.distributed): the exchange checked against an
    # independent computation, not only against another transport
    cpu_digest = cpu_digest_check(pool, lay, lo, n, final_digest, dist if world > 1 else None, dev)
    shard_ranges = [[lo, hi]]
    if world > 1:
        st = torch.tensor([lo, hi], dtype=torch.int64, device="cpu" if backend == "gloo" else dev)
        sg = torch.empty(2 * world, dtype=torch.int64, device=st.device)
        dist.all_gather_into_tensor(sg, st)
        shard_ranges = sg.view(world, 2).cpu().tolist()

    n_pages = n * chunk // pb
    # the timed launch: with a metapage the size of a page and a batch big enough
    # for the page kernel's dynamic tail, cc_pool_scan_dev hashes the n metapages
    # inside the data launch (engine.hip pool_page_launches / plan_tail: >= 8
    # 64-page tiles per wave of a one-workgroup-per-CU grid), so they are its bytes too
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    fused_meta = meta_sz == pb and pb == 4096 and n_pages // 64 >= cus * 8 * 8
    launch_pages = n_pages + (n if fused_meta else 0)
    per_step_bytes = n * chunk * world
    value = per_step_bytes * args.steps / GiB / el
    achieved = launch_pages * ALG_BYTES_PER_PAGE / (kern_ms * 1e-3) / 1e9
    traffic, traffic_src = None, None
    if rank == 0 and world == 1 and not args.no_pmc and pb == 4096:
        traffic, traffic_src = live_traffic(n * chunk / GiB)
    if traffic is None:  # the committed PMC summary of the same geometry
        why = traffic_src
        traffic, traffic_src = load_traffic(args)
        if traffic and abs(traffic / (launch_pages * ALG_BYTES_PER_PAGE) - 1.0) > 0.05:
            traffic, traffic_src = None, f"{traffic_src} profiles a different pool size"  # not this workload
        if why:
            traffic_src = f"{traffic_src} (live measurement unavailable: {why})"

    out = {
        "metric": "GiB/s CRC32C over 4KiB pages (device-resident) + % HBM roofline, 1/2/4/8 GPU",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "clock_warmup_steps": clock_warm,
        "ms_per_step": round(el / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (uniform random bytes generated in HBM)",
        "config": {"workload": f"{n} x 16 MiB chunk files per GPU (+4 KiB metapages), 4 KiB pages: "
                               "page CRC + fused epilogue (4 MiB slice CRCs, file CRC, per-copyset digest)"
                               + (" + digest all_gather inside the one cc_pool_scan_dev call (native RCCL comm)" if comm is not None else
                                  " (one cc_pool_scan_dev call) + digest all_gather via torch.distributed"
                                  if world > 1 else " (one cc_pool_scan_dev call)"),
                   "chunks_per_gpu": n, "page_bytes": pb, "copysets": N_COPYSETS,
                   "parallelism": f"chunk-range shard x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": "page_crc_kernel<16,0>", "kernel_ms_avg": round(kern_ms, 4),
                     "kernel_ms_each": [round(x, 4) for x in kern_each],
                     "kernel_ms_median": round(float(np.median(kern_each)), 4),
                     "kernel_spread_pct": round((max(kern_each) - min(kern_each)) / min(kern_each) * 100, 2),
                     "alg_bytes_per_launch": launch_pages * ALG_BYTES_PER_PAGE,
                     "pages_per_launch": launch_pages,
                     "metapages_in_launch": n if fused_meta else 0,
                     "traffic_source": traffic_src,
                     "read_probe_GBps": round(probe_gbs, 1),
                     "frac_of_read_probe": round(achieved / probe_gbs, 4),
                     "load_only_probe_GBps": round(load_only_gbs, 1),
                     "frac_of_load_only_probe": round(achieved / load_only_gbs, 4)},
        "verify": {"GiBps": round(n * chunk / GiB / (verify_ms * 1e-3), 2), "bad_pages": bad,
                   "ms_avg": round(verify_ms, 4), "ms_each": [round(x, 4) for x in verify_each],
                   "spread_pct": round((max(verify_each) - min(verify_each)) / min(verify_each) * 100, 2),
                   "alg_frac_of_hbm_peak": round(n_pages * (pb + 4) / (verify_ms * 1e-3) / 1e9
                                                 / HBM_PEAK_GBS, 4),
                   "note": "cc_page_verify_dev over the pool after a clock floor; alg bytes = 4096 read + "
                           "4 expected CRC read per page"},
        "shard_ranges": shard_ranges,
    }
    out["digest_check_cpu"] = cpu_digest
    out["numa_binding_rank0"] = numa
    if world > 1:
        if comm is not None:
            x_each = [a.elapsed_time(b) for a, b in xev]
            x_how = "HIP events on the step stream around the all-gather + XOR fold inside cc_pool_scan_dev"
        else:
            x_each = x_host_ms
            x_how = ("host wall of reduce_digests (torch.distributed all_gather + device XOR fold), the step's "
                     "kernels drained before it")
        x_ms = float(np.mean(x_each))
        # every rank's mean exchange time (the slowest rank's sets the step)
        xt = torch.tensor([x_ms], dtype=torch.float64, device="cpu" if backend == "gloo" else dev)
        xg = torch.empty(world, dtype=torch.float64, device=xt.device)
        dist.all_gather_into_tensor(xg, xt)
        rank_x = [float(v) for v in xg.cpu().tolist()]
        step_ms = el / args.steps * 1e3
        out["digest_exchange"] = {"path": comm_note, "matches_torch_distributed": digest_check,
                                  "matches_cpu_chain": cpu_digest["ok"],
                                  "ms_each": [round(x, 4) for x in x_each], "ms_avg": round(x_ms, 4),
                                  "share_of_step": round(x_ms / step_ms, 4),
                                  "rank_ms_avg": [round(x, 4) for x in rank_x],
                                  "share_of_step_max_rank": round(max(rank_x) / step_ms, 4),
                                  "timing": x_how}
        # aggregate roofline over the node: every rank's algorithmic bytes over the
        # slowest rank's page-kernel time, against N x the per-GPU peak
        agg = world * launch_pages * ALG_BYTES_PER_PAGE / (max(rank_kern) * 1e-3) / 1e9
        out["roofline"].update({"aggregate_achieved": round(agg, 1), "aggregate_peak": HBM_PEAK_GBS * world,
                                "aggregate_frac": round(agg / (HBM_PEAK_GBS * world), 4),
                                "rank_kernel_ms": [round(x, 4) for x in rank_kern],
                                "rank_kernel_ms_min": round(min(rank_kern), 4),
                                "rank_kernel_ms_max": round(max(rank_kern), 4),
                                "note": "frac/achieved/kernel_ms_* are rank 0's; aggregate_* use every rank"})
    if rank == 0 and world == 1 and args.updates:
        out["partial_write"] = partial_write_leg(pool, args)
    if rank == 0 and world == 1 and args.reads:
        out["read_verify"] = read_verify_leg(pool, args)
    if rank == 0 and world == 1 and args.wal_entries:
        out["wal_replay"] = wal_replay_leg(pool, args)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(pool, args, rank)
    if world > 1 and not args.no_e2e and args.stream_chunks:
        # BASELINE config 5 streamed end to end: every rank scans its own chunk
        # files from pinned host memory through its own PCIe link
        try:
            out["stream_all_ranks"] = stream_all_ranks_leg(args, rank, world, dev)
        except Exception as e:  # report, never lose the main line
            out["stream_all_ranks"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_e2e:
        out["e2e_pinned_GiBps"] = e2e_leg(args, dev)
        if args.stream_chunks:
            try:
                out["stream"] = stream_leg(args)
            except Exception as e:  # a CRC mismatch is reported in the line, never hidden
                out["stream"] = {"error": repr(e)}
        if args.file_chunks:
            out["files"] = files_leg(args)
        if args.scan_op_threads:
            try:
                out["scan_op"] = scan_op_leg(args)
            except Exception as e:  # report, never lose the main line
                out["scan_op"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
