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

# Chip-level limiter figures per dispatch (rocprofv3 sums the SQ / GRBM counters over the
# 8 XCDs; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles, MI355X_MICROARCH.md):
#   cycles            = GRBM_GUI_ACTIVE / 8 (per XCD; the kernel's span in shader clocks)
#   resident waves    = 4 * SQ_WAVE_CYCLES / cycles / 1024 SIMDs  (mean waves per SIMD)
#   VALU issue share  = 4 * SQ_ACTIVE_INST_VALU / (1024 * cycles)  (SIMD cycles issuing VALU)
#   VALU instr/query  = SQ_INSTS_VALU / queries (when the query count is given)
SIMDS = 1024
print("\n== chip-level, per dispatch of group 1's dispatch count")
for k, c in agg.items():
    n = len({d for d in disp[k] if "g1/" in d[0]}) or 1
    cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8 / n
    if not cyc or not c.get("SQ_WAVE_CYCLES"):
        continue
    res = 4 * c["SQ_WAVE_CYCLES"] / n / cyc / SIMDS
    valu = 4 * c.get("SQ_ACTIVE_INST_VALU", 0) / n / (SIMDS * cyc)
    l2 = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]) if c.get("TCC_HIT_sum") else float("nan")
    l1 = 1 - c["TCP_TCC_READ_REQ_sum"] / c["TCP_TOTAL_CACHE_ACCESSES_sum"] if c.get("TCP_TOTAL_CACHE_ACCESSES_sum") else float("nan")
    print(f"   {k[:48]:48s} cycles {cyc:9.0f}  waves/SIMD {res:5.2f}  VALU issue {valu:5.3f}  "
          f"VALU insts {c.get('SQ_INSTS_VALU', 0) / n:10.4g}  SALU {c.get('SQ_INSTS_SALU', 0) / n:10.4g}  "
          f"L1 hit {l1:5.3f}  L2 hit {l2:5.3f}")
