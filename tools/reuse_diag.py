"""Frame-by-frame GPU vs oracle diff of the reuse pipeline (debug aid).
usage: python tools/reuse_diag.py <scene> W H frames"""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from helpers import uniform_for  # noqa: E402
from oracle import oracle as O  # noqa: E402
from pathtracerdemo_amd import _native as N  # noqa: E402
from pathtracerdemo_amd.renderer import Renderer  # noqa: E402
from pathtracerdemo_amd.scene.world import compile_scene  # noqa: E402

scene, W, H, frames = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
cs = compile_scene(scene)
fr = O.Frame(uniform_for(cs, W, H, 1), cs.scene, cs.geometry, cs.accel)
r = Renderer(W, H, device=0, pipeline="reuse")
r.Initialize(cs)


def cmp(name, a, b):
    bad = np.argwhere(np.any(a.view(np.uint32) != b.view(np.uint32), axis=-1))
    print(f"  {name}: {len(bad)} differ", bad[:3].tolist())
    return bad


for f in range(1, frames + 1):
    fr.set_frame_index(f)
    r.Update()
    # GPU pass by pass, oracle pass by pass, compare after each
    for gp, op, nm in ((N.PTX_PASS_GBUFFER, O.PASS_GBUFFER, "gbuffer"), (N.PTX_PASS_INIT, O.PASS_INIT_REUSE, "init"),
                       (N.PTX_PASS_TEMPORAL, O.PASS_TEMPORAL, "temporal"), (N.PTX_PASS_SPATIAL, O.PASS_SPATIAL, "spatial")):
        r.run_pass(gp)
        fr.run(op, threads=8)
        got = r.read_gbuffer() if nm == "gbuffer" else (r.read_history() if nm == "spatial" else r.read_reservoir())
        want = fr.gbuffer if nm == "gbuffer" else (fr.res_hist if nm == "spatial" else fr.reservoir)
        print(f"frame {f}")
        bad = cmp(nm, got, want)
        if len(bad):
            y, x = bad[0]
            g, w = got[y, x], want[y, x]
            words = np.nonzero(g != w)[0]
            print("   words", words.tolist())
            print("   gpu   ", g.tolist())
            print("   oracle", w.tolist())
            print("   gpu f ", g.view(np.float32)[24:30].tolist(), "oracle f", w.view(np.float32)[24:30].tolist())
            if nm == "spatial":  # resync the GPU with the oracle's state to localise further diffs
                r.write_buffer(N.PTX_BUF_RESERVOIR_HIST, fr.res_hist)
            elif nm != "gbuffer":
                r.write_buffer(N.PTX_BUF_RESERVOIR, fr.reservoir)
    r.run_pass(N.PTX_PASS_FINAL)
    fr.run(O.PASS_FINAL_REUSE, threads=8, reservoir=fr.res_hist)
    fr.hist_valid = True
