#!/usr/bin/env python3
"""HBM traffic per launch of one kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs.

Correction per /opt/skills/guides/MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE counts
half the bytes of wide (16 B/lane) reads, so traffic = 2 * FETCH_SIZE + WRITE_SIZE (both
reported in KiB).  Writes/updates profiles/hbm_traffic.json under `key`.

usage: python tools/hbm_traffic.py <prof_dir with pmc_FETCH_SIZE/ pmc_WRITE_SIZE/> <key> <kernel-substring>
"""
import csv
import glob
import json
import os
import sys

prof, key, kname = sys.argv[1], sys.argv[2], sys.argv[3]
vals = {}
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    xs = []
    for f in glob.glob(os.path.join(prof, f"pmc_{ctr}", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kname in r["Kernel_Name"] and r["Counter_Name"] == ctr:
                xs.append(float(r["Counter_Value"]) * 1024.0)
    if not xs:
        sys.exit(f"no {ctr} samples for {kname!r} under {prof}")
    vals[ctr] = (sum(xs) / len(xs), len(xs))
traffic = 2.0 * vals["FETCH_SIZE"][0] + vals["WRITE_SIZE"][0]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = os.path.join(root, "profiles", "hbm_traffic.json")
db = json.load(open(out)) if os.path.exists(out) else {}
db[key] = {"bytes_per_launch": round(traffic), "fetch_size_bytes_avg": round(vals["FETCH_SIZE"][0]),
           "write_size_bytes_avg": round(vals["WRITE_SIZE"][0]), "dispatches": vals["FETCH_SIZE"][1],
           "formula": "2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md §HBM)",
           "kernel": kname,
           "source": os.path.relpath(prof, root)}
json.dump(db, open(out, "w"), indent=1, sort_keys=True)
print(key, db[key])
