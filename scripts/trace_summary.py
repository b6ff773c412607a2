#!/usr/bin/env python3
"""Per-(kernel, grid) duration summary from a rocprofv3 --kernel-trace CSV, so the
page kernel's 16 GiB launches are not averaged with its tiny metapage launches
(same instantiation, different grid).  usage: trace_summary.py run_kernel_trace.csv out.json"""
import csv
import json
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
groups = {}
for r in rows:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    short = name.split("(")[0]
    grid = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
    wg = int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or 0)
    key = (short, grid, wg)
    dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    groups.setdefault(key, []).append(dur)
out = []
for (k, g, w), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
    out.append({"kernel": k, "grid_threads": g, "workgroup": w, "calls": len(d),
                "avg_ns": round(statistics.mean(d), 1), "median_ns": statistics.median(d),
                "min_ns": min(d), "max_ns": max(d)})
json.dump(out, open(sys.argv[2], "w"), indent=1)
for o in out[:8]:
    print(o)
