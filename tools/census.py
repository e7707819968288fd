"""Per-pass work census (rays, slab tests, triangle tests) of one frame via the counting build.
usage: python tools/census.py [workload] [scene] [W] [H] [frames]"""
import sys

sys.path.insert(0, ".")
from pathtracerdemo_amd import _native as N  # noqa: E402
from pathtracerdemo_amd.renderer import Renderer  # noqa: E402
from pathtracerdemo_amd.scene.world import compile_scene  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "reuse"
scene = sys.argv[2] if len(sys.argv) > 2 else "c3_interior_32"
W, H = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (1920, 1080)
frames = int(sys.argv[5]) if len(sys.argv) > 5 else 2
passes = {"reuse": ["GBUFFER", "INIT", "TEMPORAL", "SPATIAL", "FINAL"], "restir": ["GBUFFER", "INIT", "FINAL"],
          "mcpt": ["MCPT"]}[wl]
r = Renderer(W, H, device=0, pipeline=wl, count_work=True)
r.Initialize(compile_scene(scene))
for f in range(frames):
    r.Update()
    for p in passes:
        r.reset_stats()
        r.run_pass(getattr(N, "PTX_PASS_" + p))
        r.synchronize()
        c = r.read_counters()
        if f == frames - 1:
            px = W * H
            print(f"{p:9s} rays/px {c['rays'] / px:6.2f}  aabb/ray {c['aabb_tests'] / max(1, c['rays']):7.1f}  "
                  f"tri/ray {c['tri_tests'] / max(1, c['rays']):6.1f}  rays {c['rays']}")
