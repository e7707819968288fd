"""smoke()'s reuse scenario, reads only after the last frame; optional prior ReSTIR renderer."""
import os
import sys
import numpy as np
sys.path.insert(0, os.getcwd())
from oracle import oracle as O
from pathtracerdemo_amd.renderer import Renderer
from pathtracerdemo_amd.scene.world import compile_scene

prior = os.environ.get("PRIOR", "1") == "1"
if prior:
    cs = compile_scene("dummy_scene_1")
    r = Renderer(64, 64, device=0)
    r.Initialize(cs)
    r.Update()
    r.Render()
    img = r.read_image()
c3 = compile_scene("c3_interior_32")
for frames in ((1, 2), (1, 2, 3)):
    ru = Renderer(48, 32, device=0, pipeline="reuse")
    ru.Initialize(c3)
    fo = None
    for f in frames:
        ru.Update()
        ru.Render()
        if fo is None:
            fo = O.Frame(ru.uniform, c3.scene, c3.geometry, c3.accel)
        fo.set_frame_index(f)
        fo.run_reuse_frame(threads=8)
    t = np.any(ru.read_reservoir().view(np.uint32) != fo.reservoir.view(np.uint32), axis=-1)
    s = np.any(ru.read_history().view(np.uint32) != fo.res_hist.view(np.uint32), axis=-1)
    a = np.any(ru.read_image().view(np.uint32) != fo.accum.view(np.uint32), axis=-1)
    print(f"prior={prior} frames={len(frames)} tag={os.environ.get('DIAG_TAG', '')}: temporal {int(t.sum())} "
          f"spatial {int(s.sum())} image {int(a.sum())}", flush=True)
    ru.close()
