#!/usr/bin/env python3
"""Per-build kernel durations from ONE interleaved A/B run under rocprofv3
--kernel-trace: builds loaded side by side get distinct Kernel_Ids for the same
kernel name, so each build's launches are told apart; the last N launches of
each (the interleaved timed rounds, after any one-build warm-up) are compared.
usage: kid_ab.py RUN_DIR KERNEL_SUBSTRING [N]
e.g.   rocprofv3 --kernel-trace -d gpurun_out/x -o run --output-format csv -- \\
           python3 scripts/wal_ab.py A.so B.so
       kid_ab.py gpurun_out/x range_flat_kernel 150
(Kernel_Ids are in load order: the first build passed to the harness has the lowest.)"""
import csv
import glob
import statistics
import sys

run, kn = sys.argv[1], sys.argv[2]
last = int(sys.argv[3]) if len(sys.argv) > 3 else 0
f = glob.glob(f"{run}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted((r for r in csv.DictReader(open(f)) if kn in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
by = {}
for r in rows:
    by.setdefault(int(r["Kernel_Id"]), []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k in sorted(by):
    v = by[k][-last:] if last else by[k]
    print(f"kernel_id {k}: n {len(v)} median {statistics.median(v) / 1000:.2f} us mean {statistics.mean(v) / 1000:.2f} us "
          f"min {min(v) / 1000:.2f} max {max(v) / 1000:.2f}")
