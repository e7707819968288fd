#!/usr/bin/env python3
"""Print the kernel timeline of the last N wgbuffer-started frames of a rocprofv3 kernel trace
(one line per dispatch: start offset, duration, stream, name).  usage: timeline.py trace.csv [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "wgbuffer" in r["Kernel_Name"]]
i0 = starts[-n - 1] if len(starts) > n else 0
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("ptx::", "").split("(")[0][:48]
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} q{r['Queue_Id']:>2} {name}")
