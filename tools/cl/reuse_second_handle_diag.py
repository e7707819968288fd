"""smoke()'s reuse scenario with a prior ReSTIR handle; per-frame comparison (reads sync)."""
import os
import sys
import numpy as np
sys.path.insert(0, os.getcwd())
from oracle import oracle as O
from pathtracerdemo_amd.renderer import Renderer
from pathtracerdemo_amd.scene.world import compile_scene

if os.environ.get("PRIOR", "1") == "1":
    cs = compile_scene("dummy_scene_1")
    r = Renderer(64, 64, device=0)
    r.Initialize(cs)
    r.Update()
    r.Render()
    r.read_image()
c3 = compile_scene("c3_interior_32")
per_frame = os.environ.get("PER_FRAME", "0") == "1"
ru = Renderer(48, 32, device=0, pipeline="reuse")
ru.Initialize(c3)
fo = None
out = []
for f in (1, 2, 3):
    ru.Update()
    ru.Render()
    if fo is None:
        fo = O.Frame(ru.uniform, c3.scene, c3.geometry, c3.accel)
    fo.set_frame_index(f)
    fo.run_reuse_frame(threads=8)
    if per_frame or f == 3:
        t = np.any(ru.read_reservoir().view(np.uint32) != fo.reservoir.view(np.uint32), axis=-1)
        s = np.any(ru.read_history().view(np.uint32) != fo.res_hist.view(np.uint32), axis=-1)
        out.append(f"f{f}: temporal {int(t.sum())} spatial {int(s.sum())}")
print(f"tag={os.environ.get('DIAG_TAG', '')}: " + "; ".join(out), flush=True)
