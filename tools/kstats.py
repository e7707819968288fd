"""Per-kernel calls / average / total of a rocprofv3 --stats CSV (tools/gpu.sh kstats).

    python tools/kstats.py gpurun_out/.../trace/run_kernel_stats.csv [more.csv ...]
"""
import csv
import sys


def main(paths):
    for path in paths:
        rows = list(csv.DictReader(open(path)))
        tot = sum(float(r["TotalDurationNs"]) for r in rows) or 1.0
        print(path)
        for r in rows[:16]:
            name = r["Name"].split("(")[0][:60]
            print(f"  {name:60s} calls={int(r['Calls']):5d} avg={float(r['AverageNs']) / 1e3:8.1f} us "
                  f"share={float(r['TotalDurationNs']) / tot:6.3f}")


if __name__ == "__main__":
    main(sys.argv[1:])
