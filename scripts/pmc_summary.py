#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes of the page kernels into profiles/traffic_<tag>.json.

HBM bytes per launch = FETCH_SIZE * 1024 * 2 + WRITE_SIZE * 1024
  - FETCH_SIZE/WRITE_SIZE are in KiB;
  - gfx950: FETCH_SIZE reads exactly 1/2 of the bytes of a wide coalesced streaming
    read (MI355X_MICROARCH.md §HBM).  Calibrated on THIS access pattern with
    scripts/hbm_probe.hip: a known 16 GiB read gives FETCH_SIZE*1024 = 0.5000 x bytes
    for dword, dwordx2 and dwordx4 loads (profiles/probe_r01.jsonl).
  - WRITE_SIZE is exact for our 256-B tile stores (16 MiB of CRCs per launch).
usage: scripts/pmc_summary.py gpurun_out/pmc_<tag> profiles/traffic_<tag>.json
"""
import csv
import json
import os
import statistics
import sys

src, dst = sys.argv[1], sys.argv[2]
vals = {}
for sub in sorted(os.listdir(src)):
    f = os.path.join(src, sub, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "page_crc_kernel" not in name:
            continue
        kind = "verify" if ", 1>" in name else "compute"
        vals.setdefault(kind, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
out = {"source": src, "formula": "FETCH_SIZE*1024*2 + WRITE_SIZE*1024 (gfx950 1/2 read correction)"}
for kind, cs in vals.items():
    med = {k: statistics.median(v) for k, v in cs.items()}
    fetch = med.get("FETCH_SIZE", 0.0) * 1024 * 2
    write = med.get("WRITE_SIZE", 0.0) * 1024
    out[kind] = {"counters_median": med, "read_bytes": fetch, "write_bytes": write,
                 "hbm_bytes_per_launch": fetch + write,
                 "lds_insts_per_page": med.get("SQ_INSTS_LDS", 0) / (16 << 30 >> 12),
                 "valu_insts_per_page": med.get("SQ_INSTS_VALU", 0) / (16 << 30 >> 12)}
out["hbm_bytes_per_launch"] = out.get("compute", {}).get("hbm_bytes_per_launch")
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps({k: (v if not isinstance(v, dict) else v.get("hbm_bytes_per_launch")) for k, v in out.items()}))
