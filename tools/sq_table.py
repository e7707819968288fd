"""Per-kernel SQ wave-cycle breakdown of one `tools/gpu.sh sq` pass (rocprofv3 --pmc CSV):
parked (SQ_WAIT_ANY: s_waitcnt / barrier), issue-stalled (SQ_WAIT_INST_ANY), issuing
(SQ_ACTIVE_INST_ANY) as fractions of SQ_WAVE_CYCLES, and instructions per wave.

    python tools/sq_table.py gpurun_out/r6/<case>/pmc_sq/run_counter_collection.csv
"""
import collections
import csv
import sys


def main(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0][:48]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    print(f"{'kernel':48s} {'disp':>5s} {'waves':>9s} {'cyc/wave':>9s} {'parked':>7s} {'stall':>7s} {'issue':>7s} "
          f"{'valu/w':>7s} {'vmrd/w':>7s} {'vmwr/w':>7s}")
    for k, c in sorted(agg.items(), key=lambda t: -t[1].get("SQ_WAVE_CYCLES", 0)):
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        nw = c.get("SQ_WAVES", 0) or 1
        print(f"{k:48s} {len(disp[k]):5d} {nw:9.0f} {wc / nw:9.0f} {c.get('SQ_WAIT_ANY', 0) / wc:7.3f} "
              f"{c.get('SQ_WAIT_INST_ANY', 0) / wc:7.3f} {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:7.3f} "
              f"{c.get('SQ_INSTS_VALU', 0) / nw:7.0f} {c.get('SQ_INSTS_VMEM_RD', 0) / nw:7.1f} "
              f"{c.get('SQ_INSTS_VMEM_WR', 0) / nw:7.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
