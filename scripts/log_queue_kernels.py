#!/usr/bin/env python3
"""Page-kernel durations of a write-log queue run under rocprofv3 --kernel-trace,
by what precedes each kernel, counting only full kernels (> MIN_US, so a timing
ablation whose every other kernel is empty can be compared).
usage: log_queue_kernels.py RUN_DIR [MIN_US]"""
import csv
import glob
import statistics
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
lo = float(sys.argv[2]) if len(sys.argv) > 2 else 50.0
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
a, b = [], []
for prev, cur in zip(rows, rows[1:]):
    if "log_pages_kernel<16, false>" not in cur["Kernel_Name"]:
        continue
    d = (int(cur["End_Timestamp"]) - int(cur["Start_Timestamp"])) / 1000
    if d < lo:
        continue
    (a if "log_insert_kernel" in prev["Kernel_Name"] else b).append(d)
print(f"page kernels after an insert kernel: n {len(a)} median {statistics.median(a):.2f} us")
if b:
    print(f"page kernels after a page kernel (queue): n {len(b)} median {statistics.median(b):.2f} us")
