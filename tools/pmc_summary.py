"""Aggregate rocprofv3 --pmc CSVs per kernel name (sum over dispatches, plus dispatch count).

usage: python tools/pmc_summary.py <dir with g*/run_counter_collection.csv> [kernel-substring ...]
"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
keys = sys.argv[2:] or ["trace_queue", "winit", "wfinal", "wmcpt", "gbuffer"]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(f"{root}/g*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        k = next((k for k in keys if k in name), None)
        if k is None:
            continue
        kk = name if "step" in name or "start" in name else k
        agg[kk][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[kk].add((f, r["Dispatch_Id"]))
for k, c in agg.items():
    n = len({d for d in disp[k] if "g1/" in d[0]}) or 1
    print(f"== {k}  ({n} dispatches in g1)")
    wc = c.get("SQ_WAVE_CYCLES", 0)
    if wc:
        for m in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM"):
            print(f"   {m:24s} {c.get(m, 0) / wc:6.3f} of wave cycles")
    if c.get("SQ_INSTS_VALU"):
        print(f"   VALU lane util          {c['SQ_THREAD_CYCLES_VALU'] / (64 * c['SQ_INSTS_VALU']) if c.get('SQ_THREAD_CYCLES_VALU') else 0:6.3f}")
        tot = sum(c.get(x, 0) for x in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH"))
        for x in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH"):
            print(f"   {x:24s} {c.get(x, 0) / tot:6.3f} of insts")
    if c.get("TCC_HIT_sum") is not None and (c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0)):
        print(f"   L2 hit                  {c['TCC_HIT_sum'] / (c['TCC_HIT_sum'] + c['TCC_MISS_sum']):6.3f}")
    if c.get("TCP_TOTAL_CACHE_ACCESSES_sum"):
        print(f"   L1->L2 req / L1 access  {c['TCP_TCC_READ_REQ_sum'] / c['TCP_TOTAL_CACHE_ACCESSES_sum']:6.3f}")
