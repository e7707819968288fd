"""Diagnose smoke()'s C3 reuse mismatch: sizes x env knobs, which buffer differs first."""
import os
import sys
import numpy as np
sys.path.insert(0, os.getcwd())
from oracle import oracle as O
from pathtracerdemo_amd.renderer import Renderer
from pathtracerdemo_amd.scene.world import compile_scene

c3 = compile_scene(sys.argv[1] if len(sys.argv) > 1 else "c3_interior_32")
for (W, H) in [(48, 32), (48, 40), (96, 64), (64, 32), (48, 48)]:
    ru = Renderer(W, H, device=0, pipeline="reuse")
    ru.Initialize(c3)
    fo = None
    res = []
    for f in (1, 2):
        ru.Update()
        ru.Render()
        if fo is None:
            fo = O.Frame(ru.uniform, c3.scene, c3.geometry, c3.accel)
        fo.set_frame_index(f)
        fo.run_reuse_frame(threads=8)
        t = np.any(ru.read_reservoir().view(np.uint32) != fo.reservoir.view(np.uint32), axis=-1)
        s = np.any(ru.read_history().view(np.uint32) != fo.res_hist.view(np.uint32), axis=-1)
        a = np.any(ru.read_image().view(np.uint32) != fo.accum.view(np.uint32), axis=-1)
        res.append(f"f{f}: temporal {int(t.sum())} spatial {int(s.sum())} image {int(a.sum())}"
                   + (f" first spatial {np.argwhere(s)[:3].tolist()}" if s.any() else ""))
    print(f"{W}x{H} env={os.environ.get('DIAG_TAG', '')}: " + "; ".join(res), flush=True)
    ru.close()
