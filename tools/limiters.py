#!/usr/bin/env python3
"""What bounds the roofline kernel, from one `tools/gpu.sh profile` directory (+ a simd_util report):
writes profiles/hbm_traffic.json[key] (HBM bytes per launch: 2*FETCH_SIZE + WRITE_SIZE, the gfx950
FETCH_SIZE halving of MI355X_MICROARCH.md §HBM) and profiles/limiters.json[key]:
  * l2_bytes_per_launch: TCC_REQ per launch x bytes per request, the request size calibrated by the
    same counter pass over a streaming copy of known bytes (tools/l2_calib.py); l2_hit_rate;
  * node_loop_lane_util (and every region's): lanes active per wave-execution / 64 of the traversal's
    regions over every traced pass of the frame, weighted by wave-executions (tools/simd_util.py).
bench.py puts the entry into its line's roofline.limiters (with the L2 fraction of ~34.5 TB/s).

usage: python tools/limiters.py <profile dir> <key> <kernel substring> [simd_util report]
"""
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counter_rows(d):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        yield from csv.DictReader(open(f))


def per_dispatch(d, ctr, match):
    """{dispatch id: value} of counter `ctr` for kernels whose name satisfies match()."""
    out = {}
    for r in counter_rows(d):
        if r["Counter_Name"] == ctr and match(r["Kernel_Name"]):
            k = r.get("Dispatch_Id") or r.get("Correlation_Id") or str(len(out))
            out[k] = out.get(k, 0.0) + float(r["Counter_Value"])
    return out


def mean(xs):
    xs = list(xs)
    return sum(xs) / len(xs) if xs else None


def lane_util(report):
    """Weighted lane utilisation per region over the passes of a simd_util report."""
    tot = {}
    for m in re.finditer(r"^\s+(\w+)\s+wave-execs\s+(\d+)\s+lanes/exec\s+([\d.]+)", open(report).read(), re.M):
        reg, n, lanes = m.group(1), int(m.group(2)), float(m.group(3))
        a = tot.setdefault(reg, [0, 0.0])
        a[0] += n
        a[1] += n * lanes
    return {reg: round(s / n / 64.0, 4) for reg, (n, s) in tot.items() if n}


def main():
    prof, key, kname = sys.argv[1], sys.argv[2], sys.argv[3]
    simd = sys.argv[4] if len(sys.argv) > 4 else None
    match = lambda n: kname in n  # noqa: E731
    # HBM traffic (two separate passes)
    fetch = per_dispatch(os.path.join(prof, "pmc_FETCH_SIZE"), "FETCH_SIZE", match)
    write = per_dispatch(os.path.join(prof, "pmc_WRITE_SIZE"), "WRITE_SIZE", match)
    if not fetch or not write:
        sys.exit(f"no FETCH_SIZE / WRITE_SIZE samples for {kname!r} under {prof}")
    f_b, w_b = mean(fetch.values()) * 1024.0, mean(write.values()) * 1024.0
    hbm = {"bytes_per_launch": round(2.0 * f_b + w_b), "fetch_size_bytes_avg": round(f_b),
           "write_size_bytes_avg": round(w_b), "dispatches": len(fetch),
           "formula": "2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md §HBM)",
           "kernel": kname, "source": os.path.relpath(prof, ROOT)}
    # L2 requests, calibrated on the copy kernel of tools/l2_calib.py (5 x 512 MiB moved)
    tcc = os.path.join(prof, "pmc_TCC_REQ_sum")
    req = per_dispatch(tcc, "TCC_REQ_sum", match)
    hit = per_dispatch(tcc, "TCC_HIT_sum", match)
    miss = per_dispatch(tcc, "TCC_MISS_sum", match)
    cal = per_dispatch(os.path.join(prof, "pmc_calib"), "TCC_REQ_sum", lambda n: "copy" in n.lower())
    lim = {"kernel": kname, "source": os.path.relpath(prof, ROOT)}
    if req and cal:
        big = sorted(cal.values())[-5:]  # the five 256 MiB copies
        bpr = (2 * (1 << 28)) / mean(big)
        lim["l2_requests_per_launch"] = round(mean(req.values()))
        lim["l2_bytes_per_request"] = round(bpr, 2)
        lim["l2_bytes_per_launch"] = round(mean(req.values()) * bpr)
        lim["l2_calibration"] = ("TCC_REQ_sum of a device copy of 256 MiB read + 256 MiB written (tools/l2_calib.py, "
                                 "same pass): bytes per request for 16-B-per-lane streaming accesses")
    if hit and miss:
        h, m = mean(hit.values()), mean(miss.values())
        lim["l2_hit_rate"] = round(h / (h + m), 4) if h + m else None
    if simd:
        u = lane_util(simd)
        lim["lane_util_by_region"] = u
        lim["node_loop_lane_util"] = u.get("node")
        lim["lane_util_source"] = os.path.relpath(simd, ROOT) + " (tools/simd_util.py, measurement build)"
    for name, entry in (("hbm_traffic.json", hbm), ("limiters.json", lim)):
        out = os.path.join(ROOT, "profiles", name)
        db = json.load(open(out)) if os.path.exists(out) else {}
        db[key] = entry
        json.dump(db, open(out, "w"), indent=1, sort_keys=True)
        print(name, key, json.dumps(entry))


if __name__ == "__main__":
    main()
