#!/usr/bin/env python3
"""Per-band frame time of a strong-scaled frame, one band per PROCESS (as a rank sees it:
one handle, its own streams), each timed alone on the idle GPU with bench.calibrate_band
(the band path a rank runs, pipelined, without the exchange: PTX_FLAG_HALO_SKIP).
`tools/band_timing.py` times all bands from one process, where 9 handles' streams share the
process's hardware queues.  usage: python tools/band_alone.py [--world 8] [--bands census|calibrated]
prints one JSON line: bands, per-band ms, max/mean, implied speedup over the one-GPU frame.
(The exchange proxy, PTX_AB=HALO_PROXY_US=<us>, is an A/B switch: run it with
PTX_LIB_PATH=$PWD/pathtracerdemo_amd/libptx_ab.so, the measurement build.)"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_band(W, H, b0, b1, scene, overlap=False):
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench; "
            f"from pathtracerdemo_amd.scene.world import compile_scene; "
            f"cs = compile_scene({scene!r}); "
            f"print(bench.calibrate_band(cs, {W}, {H}, 'reuse', 0, {b0}, {b1}, bench.PASSES['reuse'], frames=6, overlap={overlap}))")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    if out.returncode != 0:
        sys.exit(f"band {b0}-{b1} failed: {out.stderr[-2000:]}")
    return float(out.stdout.strip().splitlines()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frame", default="3840x2160")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--scene", default="c3_interior_32")
    ap.add_argument("--bands", default=None, help="JSON list of [b0, b1]; default: equal bands")
    ap.add_argument("--recut", type=int, default=0, help="re-cut rounds from the measured times")
    ap.add_argument("--overlap", action="store_true", help="bands with PTX_FLAG_HALO_OVERLAP")
    args = ap.parse_args()
    sys.path.insert(0, ROOT)
    import numpy as np
    from pathtracerdemo_amd import bands as B
    W, H = (int(v) for v in args.frame.split("x"))
    bands = json.loads(args.bands) if args.bands else [list(B.band(H, args.world, r)) for r in range(args.world)]
    costs = np.ones(H)
    rounds = []
    for it in range(args.recut + 1):
        ms = [run_band(W, H, b0, b1, args.scene, args.overlap) for b0, b1 in bands]
        rounds.append({"bands": bands, "band_ms": [round(v, 4) for v in ms],
                       "max_over_mean": round(max(ms) / (sum(ms) / len(ms)), 4), "sum_ms": round(sum(ms), 3)})
        print(json.dumps(rounds[-1]), flush=True)
        if it < args.recut:
            costs = B.recalibrated_costs(costs, bands, ms)
            bands = [list(b) for b in B.balanced_bands(costs, args.world, min_rows=30)]


if __name__ == "__main__":
    main()
