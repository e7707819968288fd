#!/usr/bin/env python3
"""Markdown roofline table of DESIGN.md §4.2 from the committed bench lines and rocprof stats
(profiles/<round>/<workload>/bench_line.json, kernel_stats.csv).
usage: python tools/roofline_table.py [round]"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rnd = sys.argv[1] if len(sys.argv) > 1 else "r1"
cols = [("reuse", "**reuse, C3** (headline, configs[2])"), ("gi", "ReSTIR GI, C3 (configs[4])"),
        ("restir", "ReSTIR, C1"), ("mcpt", "TEST_MCPT, C1 (configs[1])")]
lines, stats = {}, {}
for wl, _ in cols:
    d = os.path.join(ROOT, "profiles", rnd, wl)
    lines[wl] = json.loads(open(os.path.join(d, "bench_line.json")).read())
    calls = total = 0
    for r in csv.DictReader(open(os.path.join(d, "kernel_stats.csv"))):
        if r["Name"].startswith("void ptx::trace_queue<false, "):  # every timed instance (GI: + occlusion)
            calls += int(r["Calls"])
            total += float(r["TotalDurationNs"])
    if calls:
        stats[wl] = (calls, total / calls / 1e6)
rows = [
    ("frame (bench `ms_per_step`)", lambda d, w: f"{d['ms_per_step']:.2f} ms → **{d['value']:.0f} Msamples/s**"),
    ("`trace_queue` launches per frame", lambda d, w: f"{d['roofline']['launches_per_frame']:.0f}"),
    ("`trace_queue` avg launch (events / rocprof)",
     lambda d, w: f"{d['roofline']['avg_launch_ms']:.3f} / {stats[w][1]:.3f} ms" if w in stats else "–"),
    ("algorithmic bytes per launch", lambda d, w: f"{d['roofline']['alg_bytes_per_launch'] / 1e9:.2f} GB"),
    ("roofline frac (`trace_queue`)", lambda d, w: f"**{d['roofline']['frac']:.3f}**"),
    ("the same bytes over the rocprof average",
     lambda d, w: f"{d['roofline']['alg_bytes_per_launch'] / (stats[w][1] * 1e-3) / 8e12:.3f}" if w in stats else "–"),
    ("L2 request bytes per launch (frac of ≈34.5 TB/s; hit rate)",
     lambda d, w: (f"{lim['l2_bytes_per_launch'] / 1e6:.0f} MB ({lim['l2_frac']:.3f}; {lim['l2_hit_rate']:.2f})"
                   if (lim := d['roofline'].get('limiters') or {}).get('l2_bytes_per_launch') else "–")),
    ("node-loop lane use (SIMD-utilisation build)",
     lambda d, w: f"{(d['roofline'].get('limiters') or {}).get('node_loop_lane_util'):.3f}"
     if (d['roofline'].get('limiters') or {}).get('node_loop_lane_util') is not None else "–"),
    ("frame-level frac (§8d)", lambda d, w: f"{d['roofline']['frame']['frac']:.3f}"),
    ("HBM traffic per trace launch (PMC)",
     lambda d, w: f"{d['roofline']['traffic'] / 1e6:.0f} MB" if d['roofline'].get('traffic') else "–"),
    ("CPU baseline (C oracle; threads)",
     lambda d, w: f"{d['cpu_baseline']['value']:.2f} Msamples/s ({d['cpu_baseline']['cores']})"),
    ("JS CPU baseline (reference pipeline, Node workers)",
     lambda d, w: f"{d['ts_cpu_baseline']['value']:.2f} Msamples/s" if d.get("ts_cpu_baseline") else "–"),
]
print(f"| 1×MI355X, 1920×1080, 1 spp (`profiles/{rnd}/`) | " + " | ".join(c for _, c in cols) + " |")
print("|---|" + "---|" * len(cols))
for name, fn in rows:
    print(f"| {name} | " + " | ".join(fn(lines[w], w) for w, _ in cols) + " |")
