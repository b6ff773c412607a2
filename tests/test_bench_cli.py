"""bench.py honours --gpus (a plain `--gpus 8` used to run one rank
and report n_gpus 1).  Under a launcher WORLD_SIZE must equal --gpus; the check
runs before anything touches a GPU, so it is testable here."""
import json
import os
import subprocess
import sys

from conftest import ROOT


def test_world_size_mismatch_refused():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2, p.stderr[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert "WORLD_SIZE=2" in line["error"]


def test_numa_binding_helpers_never_fail():
    """bench.bind_to_gpu_numa parses sysfs cpulists and never fails the run: with
    no GPU (here) it reports why it did not bind and leaves the affinity alone."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench._cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert bench._cpulist("5") == {5}
    assert bench._cpulist("\n") == set()
    before = os.sched_getaffinity(0)
    r = bench.bind_to_gpu_numa(0)
    assert r["bound"] is False and r["why"]
    assert os.sched_getaffinity(0) == before


def test_stream_distinct_bounded_by_free_host_memory():
    """The C3 stream leg pins up to --stream-distinct 16 MiB chunks (156 GiB for
    all 10,000 distinct): _host_chunk_budget keeps that under MemAvailable /
    the cgroup limit less a margin, never below 64 chunks, never above the ask."""
    sys.path.insert(0, ROOT)
    import bench
    want = 10000
    got = bench._host_chunk_budget(want)
    assert 64 <= got <= want
    free = None
    for line in open("/proc/meminfo"):
        if line.startswith("MemAvailable:"):
            free = int(line.split()[1]) * 1024
    if free is not None:
        assert got == want or got == 64 or got * (16 << 20) <= free
    assert bench._host_chunk_budget(10) == 10
    assert bench._host_chunk_budget(want, margin=1 << 62) == 64  # nothing to spare: the floor
