"""Concurrency timeline of one frame of a multi-stream kernel trace (rocprofv3 --kernel-trace).

usage: python tools/timeline.py <run_kernel_trace.csv> [first-kernel-substring] [frame-from-end]
Prints, per stream (queue), the launch sequence of the chosen frame with start offsets and
durations, and the share of the frame span during which 0 / 1 / 2 / 3+ kernels ran."""
import csv
import sys

path = sys.argv[1]
first = sys.argv[2] if len(sys.argv) > 2 else "wgbuffer"
back = int(sys.argv[3]) if len(sys.argv) > 3 else 2
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
# frame starts: a `first` launch that follows a launch of another kernel on every stream
starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"] and
          (i == 0 or first not in rows[i - 1]["Kernel_Name"])]
lo, hi = starts[-back - 1], starts[-back]
fr = rows[lo:hi]
t0 = int(fr[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in fr)
ev = []
for r in fr:
    ev.append((int(r["Start_Timestamp"]), 1))
    ev.append((int(r["End_Timestamp"]), -1))
ev.sort()
occ = {}
cur, last = 0, t0
for t, d in ev:
    occ[min(cur, 3)] = occ.get(min(cur, 3), 0) + (t - last)
    cur += d
    last = t
span = t1 - t0
qs = sorted({r["Queue_Id"] for r in fr})
for q in qs:
    print(f"queue {q}:")
    for r in fr:
        if r["Queue_Id"] != q:
            continue
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        print(f"  {s:8.1f} +{d:7.1f} us  {r['Kernel_Name'].split('(')[0][:48]}  grid={int(r['Grid_Size_X'])//int(r['Workgroup_Size_X'])}")
print(f"frame span {span/1e3:.1f} us; kernels running: " +
      ", ".join(f"{k}{'+' if k == 3 else ''}: {100*v/span:.1f}%" for k, v in sorted(occ.items())))
