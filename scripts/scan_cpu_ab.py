"""Scan op on the CPU primitive at the reference's call shape (bench.py scan_op_leg's "cpu"
mode: T native threads, each a 16 MiB chunk file's 5 ops in turn), under each CPU-path mode
of crc32c_cpu.cpp, each mode in a process of its own (the mode is read once), modes
alternated over rounds.  usage: python scripts/scan_cpu_ab.py [threads] [rounds]"""
import json
import os
import subprocess
import sys

CHILD = r"""
import sys, time, numpy as np
sys.path.insert(0, %r)
import bench
T, calls = %d, 500
file_bytes = 4096 + (16 << 20)
bufs = [np.random.default_rng(t).integers(0, 256, file_bytes, dtype=np.uint8) for t in range(T)]
offs = [0] + [4096 + k * (4 << 20) for k in range(4)]
lens = [4096] + [4 << 20] * 4
op_bytes = np.array(lens * (calls // len(lens) + 1))[:calls]
bench.run_scan_ops(bufs, offs, lens, 2 * len(offs), "cpu")
out = []
for r in range(3):
    rc, lat, crcs, wall, cpu_s = bench.run_scan_ops(bufs, offs, lens, calls, "cpu")
    total = float(op_bytes.sum()) * T
    out.append(round(total / 2**30 / wall, 1))
print(out)
"""


def main():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    modes = {"split": {"CURVE_CRC_FOLD_SPLIT": "1"}, "fold": {"CURVE_CRC_FOLD_SPLIT": "0"},
             "3way": {"CURVE_CRC_NO_FOLD": "1"}}
    res = {m: [] for m in modes}
    for _ in range(rounds):
        for m, env in modes.items():
            r = subprocess.run([sys.executable, "-c", CHILD % (root, threads)], env=dict(os.environ, **env),
                               capture_output=True, text=True, timeout=300)
            if r.returncode:
                print(r.stderr[-2000:])
                sys.exit(1)
            res[m] += json.loads(r.stdout.strip().splitlines()[-1])
            print(m, res[m], flush=True)
    print(json.dumps({"threads": threads, "agg_GiBps": res}))


if __name__ == "__main__":
    main()
