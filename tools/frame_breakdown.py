"""Per-launch durations of the last complete frame in a rocprofv3 kernel trace.

usage: python tools/frame_breakdown.py <run_kernel_trace.csv> [first-kernel-substring]
"""
import csv
import sys

path = sys.argv[1]
first = sys.argv[2] if len(sys.argv) > 2 else "gbuffer"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
lo, hi = idx[-2], idx[-1]
tot = 0.0
for r in rows[lo:hi]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    print(f"{d:9.1f} us  {r['Kernel_Name'].split('(')[0][:50]:50s} vgpr={r['VGPR_Count']}")
span = (int(rows[hi]["Start_Timestamp"]) - int(rows[lo]["Start_Timestamp"])) / 1e3
print(f"sum {tot:.1f} us, frame span {span:.1f} us")
