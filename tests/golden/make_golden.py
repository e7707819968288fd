#!/usr/bin/env python3
"""Generate the committed golden fixtures (tests/golden/*) from the CPU oracle.

The reference has no runnable WGSL runtime, tests or golden images (SURVEY.md §4,
§8c), so these fixtures pin the oracle restatement itself: any later change to the
oracle, the scene compiler or the HIP path that alters them is a regression.
Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from helpers import uniform_for  # noqa: E402
from oracle import oracle as O  # noqa: E402
from pathtracerdemo_amd.scene.world import compile_scene  # noqa: E402

W, H = 24, 24
REUSE_FRAMES = 3


# (scene, frames) -> fixture file; C3 is the build-defined many-light interior (scenes/make_c3.py)
FIXTURES = {"c1_24x24_4frames.npz": ("dummy_scene_1", 4), "c3_24x24_2frames.npz": ("c3_interior_32", 2)}


def scene_digest(cs) -> np.ndarray:
    """sha256 of the three device arrays: pins the scene compiler's output too."""
    import hashlib
    h = hashlib.sha256()
    for a in (cs.scene, cs.geometry, cs.accel):
        h.update(np.ascontiguousarray(a, dtype="<u4").tobytes())
    return np.frombuffer(h.digest(), dtype=np.uint8)


def frame_fixture(cs, frames):
    fr = O.Frame(uniform_for(cs, W, H, 1), cs.scene, cs.geometry, cs.accel)
    for f in range(1, frames + 1):
        fr.set_frame_index(f)
        fr.run(O.PASS_RESTIR, threads=1)
    mc = O.Frame(uniform_for(cs, W, H, 1), cs.scene, cs.geometry, cs.accel)
    mc.run(O.PASS_MCPT, threads=1)
    # the build-defined reuse pipeline, default parameters, 3 frames
    ru = O.Frame(uniform_for(cs, W, H, 1), cs.scene, cs.geometry, cs.accel)
    for f in range(1, REUSE_FRAMES + 1):
        ru.set_frame_index(f)
        ru.run_reuse_frame(threads=1)
    # the build-defined ReSTIR GI pipeline, default parameters, 3 frames
    gi = O.Frame(uniform_for(cs, W, H, 1), cs.scene, cs.geometry, cs.accel)
    for f in range(1, REUSE_FRAMES + 1):
        gi.set_frame_index(f)
        gi.run_gi_frame(threads=1)
    return dict(uniform=fr.uniform, gbuffer=fr.gbuffer, reservoir=fr.reservoir, accum_restir=fr.accum,
                accum_mcpt=mc.accum, frames=np.int32(frames), scene_sha256=scene_digest(cs),
                accum_reuse=ru.accum, hist_reuse=ru.res_hist, reuse_frames=np.int32(REUSE_FRAMES),
                reuse_params=np.array(ru.reuse, dtype=np.int32),
                accum_gi=gi.accum, hist_gi=gi.gi_hist, direct_gi=gi.direct)


def kat_table():
    rows = {"pcg": {str(s): O.pcg(s) for s in [0, 1, 2, 3, 1973, 9277, 26699, 2 ** 31, 2 ** 32 - 1]}}
    n = [0.0, 0.0, 1.0]
    mats = {"diffuse": [0.8, 0.8, 0.8, 0.0, 1.0, 0.0, 1.5], "metal": [0.9, 0.6, 0.3, 1.0, 0.25, 0.0, 1.5],
            "glass": [1.0, 1.0, 0.0, 0.0, 0.01, 1.0, 1.5]}
    v = [0.0, 0.6, 0.8]
    ls = {"same": [0.48, 0.0, 0.8775], "across": [0.1, -0.5, -0.86]}
    rows["bsdf"] = {f"{m}/{l}": [float(x) for x in O.bsdf(n, mats[m], v, ls[l])] for m in mats for l in ls}
    rows["pdf_bsdf"] = {f"{m}/{l}": O.pdf_bsdf(n, mats[m], v, ls[l]) for m in mats for l in ls}
    rows["sample_bsdf"] = {}
    for m in mats:
        for seed in (1, 77, 4096):
            d, lobe, s2 = O.sample_bsdf(n, mats[m], v, seed)
            rows["sample_bsdf"][f"{m}/{seed}"] = [[float(x) for x in d], lobe, s2]
    return rows


def main():
    O.build()
    for fname, (scene, frames) in FIXTURES.items():
        np.savez_compressed(os.path.join(HERE, fname), **frame_fixture(compile_scene(scene), frames))
    with open(os.path.join(HERE, "kat.json"), "w") as fh:
        json.dump(kat_table(), fh, indent=1, sort_keys=True)
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
