#!/usr/bin/env python3
"""One band of a strong-scaled frame timed alone (bench.calibrate_band, one process per run) under
several PTX_AB settings of the measurement build: which switches shorten a rank's band frame.
usage: PTX_LIB_PATH=.../libptx_ab.so python tools/band_knobs.py --band 898,1064 --ab "" "PIPE_DEPTH=3" ...
prints one JSON line per setting."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("--band", default="898,1064")
ap.add_argument("--frame", default="3840x2160")
ap.add_argument("--frames", type=int, default=20)
ap.add_argument("--overlap", action="store_true")
ap.add_argument("--ab", nargs="*", default=[""])
a = ap.parse_args()
W, H = (int(v) for v in a.frame.split("x"))
b0, b1 = (int(v) for v in a.band.split(","))
for ab in a.ab:
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench; "
            f"from pathtracerdemo_amd.scene.world import compile_scene; cs = compile_scene('c3_interior_32'); "
            f"print(bench.calibrate_band(cs, {W}, {H}, 'reuse', 0, {b0}, {b1}, bench.PASSES['reuse'], "
            f"frames={a.frames}, overlap={a.overlap}))")
    env = dict(os.environ, PTX_AB=ab)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env)
    if out.returncode != 0:
        sys.exit(f"{ab}: {out.stderr[-1500:]}")
    print(json.dumps({"band": [b0, b1], "ab": ab, "overlap": a.overlap,
                      "ms": round(float(out.stdout.strip().splitlines()[-1]), 4)}), flush=True)
