"""Child process of tests/test_gpu_debug_fill.py: runs with PTX_AB=DEBUG_FILL=<byte> set, so
every device buffer the library allocates starts filled with that byte instead of whatever
the allocator hands back.  An uninitialised read in any kernel then changes the output (or
faults) instead of passing by luck.  Renders C3 reuse frames (whole pipeline, pipelined
frames, the spatial combine's folded last job step) and TEST_MCPT frames, each checked bit
for bit against the oracle; prints "ok" on success."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from helpers import uniform_for  # noqa: E402
from oracle import oracle as O  # noqa: E402
from pathtracerdemo_amd.renderer import Renderer  # noqa: E402
from pathtracerdemo_amd.scene.world import compile_scene  # noqa: E402


def same(got, want, what):
    got, want = np.asarray(got).view(np.uint32), np.asarray(want).view(np.uint32)
    bad = np.any(got != want, axis=-1)
    if bad.any():
        sys.exit(f"{what}: {int(bad.sum())} pixels differ, first at {np.argwhere(bad)[:4].tolist()}")


def main():
    assert os.environ.get("PTX_AB", "").startswith("DEBUG_FILL="), "run through test_gpu_debug_fill.py"
    O.build()
    cs = compile_scene("c3_interior_32")
    W, H = 96, 64
    fr = O.Frame(uniform_for(cs, W, H, 1), cs.scene, cs.geometry, cs.accel)
    fr.reuse = (30, 3, 20)
    r = Renderer(W, H, device=0, pipeline="reuse", reuse_radius=30, reuse_neighbors=3, temporal_cap=20)
    r.Initialize(cs)
    for f in (1, 2, 3):
        fr.set_frame_index(f)
        fr.run_reuse_frame(threads=8)
        r.Update()
        r.Render()
    same(r.read_history(), fr.res_hist, "reuse: spatial output")
    same(r.read_image(), fr.accum, "reuse: radiance")
    r.close()

    cs1 = compile_scene("dummy_scene_1")
    W, H = 64, 48
    fr = O.Frame(uniform_for(cs1, W, H, 1), cs1.scene, cs1.geometry, cs1.accel)
    r = Renderer(W, H, device=0, pipeline="mcpt")
    r.Initialize(cs1)
    for f in (1, 2):
        r.Update()
        r.Render()
        fr.set_frame_index(f)
        fr.run(O.PASS_MCPT, 8)
    same(r.read_image(), fr.accum, "mcpt: radiance")
    r.close()
    print("ok")


if __name__ == "__main__":
    main()
