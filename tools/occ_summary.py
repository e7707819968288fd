#!/usr/bin/env python3
"""Mean resident waves per SIMD per kernel from ONE rocprofv3 --pmc pass that holds
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE (tools/cl/occ_calib.sh).

waves/SIMD = 4 * SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8) / 1024: rocprofv3 sums both counters
over the 8 XCDs, SQ_WAVE_CYCLES counts quad-cycles (MI355X_MICROARCH.md) and the chip has 1024
SIMDs.  Every counter comes from the same dispatches, so the ratio is per kernel span.
usage: python tools/occ_summary.py <run_counter_collection.csv> [--per-dispatch]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    k = r["Kernel_Name"] + (f" #{r['Dispatch_Id']}" if "--per-dispatch" in sys.argv else "")
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
print(f"{'kernel':72s} {'disp':>5s} {'waves/SIMD':>10s} {'SQ_WAVES/disp':>13s} {'cycles/disp':>12s}")
for k, c in agg.items():
    cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8
    if not cyc:
        continue
    n = len(disp[k])
    print(f"{k[:72]:72s} {n:5d} {4 * c['SQ_WAVE_CYCLES'] / cyc / 1024:10.2f} {c['SQ_WAVES'] / n:13.0f} {cyc / n:12.0f}")
