#!/usr/bin/env python3
"""SIMD utilisation of the wavefront trace kernel by traversal region (diagnostic build).

Runs each pass of one 1080p frame with PTX_FLAG_COUNT_WORK and PTX_AB=TRACE_PROF and prints,
per region (instance transform, root test, node loop, leaf block, triangle loop), the
wave-level executions, the mean active lanes per execution (of 64) and per-query averages.
On scenes the production walk flattens (>= 3 instances, tables in LDS) the profiled kernel is
that walk with the instance cull applied (its AABB / triangle counts are the tests executed);
otherwise the counting walk (every instance visited, the reference's counts).
usage: python tools/simd_util.py [--workload restir|mcpt]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["PTX_AB"] = ",".join(v for v in (os.environ.get("PTX_AB", ""), "TRACE_PROF") if v)
# (TRACE_PROF is an A/B switch: only the measurement build reads it -- make -C pathtracerdemo_amd/csrc ab)
os.environ.setdefault("PTX_LIB_PATH", os.path.join(ROOT, "pathtracerdemo_amd", "libptx_ab.so"))
if not os.path.exists(os.environ["PTX_LIB_PATH"]):
    sys.exit(f"{os.environ['PTX_LIB_PATH']} missing: make -C pathtracerdemo_amd/csrc ab")

from pathtracerdemo_amd import _native as N  # noqa: E402
from pathtracerdemo_amd.renderer import Renderer  # noqa: E402
from pathtracerdemo_amd.scene.world import compile_scene  # noqa: E402

REGIONS = ["inst", "root", "node", "leaf", "tri"]
ORDER = {"root": 0, "node": 1, "leaf": 2, "tri": 3, "inst": 4}

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="restir", choices=["restir", "mcpt", "reuse"])
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--scene", default=None, help="default: c3_interior_32 (reuse), dummy_scene_1 (others)")
args = ap.parse_args()
cs = compile_scene(args.scene or ("c3_interior_32" if args.workload == "reuse" else "dummy_scene_1"))
r = Renderer(args.width, args.height, device=0, pipeline=args.workload, count_work=True)
r.Initialize(cs)
r.Update()
passes = {"restir": [("gbuffer", N.PTX_PASS_GBUFFER), ("init", N.PTX_PASS_INIT), ("final", N.PTX_PASS_FINAL)],
          "reuse": [("gbuffer", N.PTX_PASS_GBUFFER), ("init", N.PTX_PASS_INIT), ("temporal", N.PTX_PASS_TEMPORAL),
                    ("spatial", N.PTX_PASS_SPATIAL), ("final", N.PTX_PASS_FINAL)],
          "mcpt": [("mcpt", N.PTX_PASS_MCPT)]}[args.workload]
for name, pid in passes:
    r.reset_stats()
    r.run_pass(pid)
    r.synchronize()
    c = np.zeros(32, dtype=np.uint64)
    r._call("ptx_read_buffer", r._h, N.PTX_BUF_COUNTERS, c.ctypes.data, c.nbytes)
    rays = int(c[0])
    if name == "gbuffer":
        print(f"{name}: rays {rays} (profile regions are recorded by the wavefront trace kernel only)")
        continue
    print(f"== {name}: {rays} queries, {int(c[2]) / max(rays, 1):.2f} AABB + {int(c[3]) / max(rays, 1):.2f} tri tests/query")
    for reg in REGIONS:
        k = ORDER[reg]
        waves, lanes = int(c[8 + 2 * k]), int(c[9 + 2 * k])
        util = lanes / max(64 * waves, 1)
        print(f"   {reg:5s} wave-execs {waves:>12d}  lanes/exec {lanes / max(waves, 1):6.2f}  util {util:6.3f}"
              f"  wave-execs/query {64 * waves / max(rays, 1):7.2f}")
