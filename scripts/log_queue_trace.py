#!/usr/bin/env python3
"""Kernel-trace summary of scripts/log_queue_ab.py under rocprofv3 --kernel-trace:
per page kernel, its duration and the idle gap before it, split by what ran
just before it (the insert kernel: one call per batch; another page kernel: the
queue, whose page kernels also group the next batch).
usage: log_queue_trace.py RUN_DIR"""
import csv
import glob
import statistics
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
by = {"after insert (one call a batch)": ([], [], []), "after a page kernel (queue)": ([], [], [])}
for prev, cur in zip(rows, rows[1:]):
    if "log_pages_kernel<16, false>" not in cur["Kernel_Name"]:
        continue
    d = (int(cur["End_Timestamp"]) - int(cur["Start_Timestamp"])) / 1000
    g = (int(cur["Start_Timestamp"]) - int(prev["End_Timestamp"])) / 1000
    if "log_insert_kernel" in prev["Kernel_Name"]:
        ins = (int(prev["End_Timestamp"]) - int(prev["Start_Timestamp"])) / 1000
        by["after insert (one call a batch)"][0].append(d)
        by["after insert (one call a batch)"][1].append(g)
        by["after insert (one call a batch)"][2].append(ins)
    elif "log_pages_kernel" in prev["Kernel_Name"]:
        by["after a page kernel (queue)"][0].append(d)
        by["after a page kernel (queue)"][1].append(g)
for k, (d, g, ins) in by.items():
    if d:
        print(f"{k}: n {len(d)} page kernel median {statistics.median(d):.2f} us, gap before it median "
              f"{statistics.median(g):.2f} us" + (f", insert kernel median {statistics.median(ins):.2f} us" if ins else ""))

# the timeline of the last queue call: from the last standalone insert kernel
# followed by a page kernel that is followed by page kernels
names = [r["Kernel_Name"] for r in rows]
last_q = None
for i in range(len(rows) - 2):
    if "log_insert_kernel" in names[i] and "log_pages_kernel" in names[i + 1] and "log_pages_kernel" in names[i + 2]:
        last_q = i
if last_q is not None:
    t0 = int(rows[last_q - 1]["End_Timestamp"])
    print("last queue call (us from the end of the kernel before it):")
    for r in rows[last_q - 1:last_q + 12]:
        s, e = (int(r["Start_Timestamp"]) - t0) / 1000, (int(r["End_Timestamp"]) - t0) / 1000
        print(f"  {s:9.2f} {e:9.2f} {e - s:8.2f}  {r['Kernel_Name'][:60]}")
