#!/usr/bin/env python3
"""Summarise the write-log PMC passes (scripts/gpu_pmc_log.sh) into one JSON:
per mode and kernel the mean counter value per dispatch, HBM bytes (FETCH_SIZE x
1024 x 2 per MI355X_MICROARCH.md's gfx950 correction, WRITE_SIZE x 1024) and the
SQ mix per touched page.  usage: pmc_log_summary.py TAG OUT.json [touched_pages]
(reads gpurun_out/pmc_log_<PASS>_<TAG> and gpurun_out/pmc_log_<PASS>_<TAG>_delta)"""
import csv
import json
import os
import statistics
import sys

tag, dst = sys.argv[1], sys.argv[2]
pages = int(sys.argv[3]) if len(sys.argv) > 3 else 101161
out = {"source": f"rocprofv3 --pmc passes over scripts/prof_log.py --reps 2 (65,536 random 512 B-4 KiB writes over a "
                 f"16 GiB pool), scripts/gpu_pmc_log.sh; one counter group per pass; tag {tag}",
       "correction": "HBM read bytes = FETCH_SIZE x 1024 x 2 (gfx950, MI355X_MICROARCH.md), write bytes = WRITE_SIZE x "
                     "1024; the x2 is calibrated for streaming reads, these are random 256-byte rows",
       "touched_pages_per_batch_approx": pages, "modes": {}}
for mode, suf in (("full", ""), ("delta", "_delta")):
    per = {}
    for p in ("FETCH_SIZE", "WRITE_SIZE", "SQ_WAVES"):
        d = f"gpurun_out/pmc_log_{p}_{tag}{suf}"
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        acc = {}
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            k = k.replace("cc::", "")
            if "log_" not in k:
                continue
            acc.setdefault(k, {}).setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            acc[k][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for k, cs in acc.items():
            for c, v in cs.items():
                per.setdefault(k, {})[c] = statistics.mean(v.values())
    for k, c in per.items():
        if "FETCH_SIZE" in c:
            c["hbm_read_bytes"] = c["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in c:
            c["hbm_write_bytes"] = c["WRITE_SIZE"] * 1024
        if ("pages" in k or "quad" in k) and "SQ_INSTS_VALU" in c:
            for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
                c[n + "_per_page"] = round(c[n] / pages, 1)
            c["wait_inst_frac_of_wave_cycles"] = round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 3)
    out["modes"][mode] = per
json.dump(out, open(dst, "w"), indent=1)
for m, per in out["modes"].items():
    for k, c in per.items():
        print(m, k, {x: round(y) if isinstance(y, float) and y > 100 else y for x, y in c.items()
                     if x in ("hbm_read_bytes", "hbm_write_bytes", "SQ_INSTS_VALU_per_page", "SQ_INSTS_SALU_per_page",
                              "wait_inst_frac_of_wave_cycles")})
