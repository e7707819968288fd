"""Scenes with many instances.  The root / instance tables are staged in LDS sized to the scene
(32 B per sub-mesh root, 144 B per instance, up to kLdsTableMax = 24 KB, ptx_device.h):
the furnished C3 (13 instances, scenes/c3_furnished.json) and C1 with ten windows take the
LDS fast path (round 1 capped it at 8 instances); C1 with 170 windows (30 KB of tables) takes
the fallback kernels (global-memory tables, the pass-by-pass G-buffer).  Every pipeline
matches the oracle bit for bit either way, and a furnished frame splits into bands."""
import copy
import json
import os

import numpy as np
import pytest

from helpers import uniform_for

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def many_instances():
    """DUMMY_SCENE_1 with ten PureWindow instances (11 instances > the 8 staged in LDS)."""
    from pathtracerdemo_amd.scene.world import compile_scene
    d = json.load(open(os.path.join(ROOT, "scenes", "dummy_scene_1.json")))
    win = next(a for a in d["assets"] if a.get("meshName") == "PureWindow")
    extra = []
    for k in range(1, 10):
        w = copy.deepcopy(win)
        w["id"] = f"window_instance_{k}"
        w["transform"]["position"] = [-3.0 + 0.6 * k, 0.1 * k, -2.0 - 0.3 * k]
        extra.append(w)
    d["assets"] = d["assets"][:2] + extra + d["assets"][2:]
    cs = compile_scene(d)
    assert cs.instance_count == 11
    return cs


def windows_scene(n):
    from pathtracerdemo_amd.scene.world import compile_scene
    d = json.load(open(os.path.join(ROOT, "scenes", "dummy_scene_1.json")))
    win = next(a for a in d["assets"] if a.get("meshName") == "PureWindow")
    extra = []
    for k in range(1, n):
        w = copy.deepcopy(win)
        w["id"] = f"window_instance_{k}"
        w["transform"]["position"] = [-3.0 + 0.035 * k, 0.006 * k, -2.0 - 0.02 * k]
        extra.append(w)
    d["assets"] = d["assets"][:2] + extra + d["assets"][2:]
    return compile_scene(d)


def table_bytes(cs):
    n_subs = sum(int(cs.scene[cs.offsets["mesh_descriptor"] + 6 * int(cs.scene[33 * i + 32]) + 5])
                 for i in range(cs.instance_count))
    return ((32 * n_subs + 15) & ~15) + 144 * cs.instance_count


@pytest.fixture(scope="module")
def furnished():
    from pathtracerdemo_amd.scene.world import compile_scene
    return compile_scene("c3_furnished")


@pytest.fixture(scope="module")
def huge_tables():
    cs = windows_scene(170)
    assert table_bytes(cs) > 24576  # past kLdsTableMax: the global-table kernels
    return cs


@pytest.mark.parametrize("which", ["many_instances", "furnished", "huge_tables"])
@pytest.mark.parametrize("pipeline", ["restir", "mcpt", "reuse", "gi"])
def test_many_instances_bit_exact(request, which, oracle_mod, pipeline):
    from pathtracerdemo_amd.renderer import Renderer
    cs, O, W, H = request.getfixturevalue(which), oracle_mod, 40, 32
    r = Renderer(W, H, device=0, pipeline=pipeline)
    r.Initialize(cs)
    fr = O.Frame(uniform_for(cs, W, H, 1), cs.scene, cs.geometry, cs.accel)
    for f in (1, 2):
        r.Update()
        r.Render()
        fr.set_frame_index(f)
        if pipeline == "reuse":
            fr.run_reuse_frame(threads=8)
        elif pipeline == "gi":
            fr.run_gi_frame(threads=8)
        else:
            fr.run(O.PASS_RESTIR if pipeline == "restir" else O.PASS_MCPT, threads=8)
    np.testing.assert_array_equal(r.read_image().view(np.uint32), fr.accum.view(np.uint32))
    r.close()


def test_furnished_bands_bit_identical(furnished):
    """A furnished C3 frame (13 instances: LDS tables) as 3 band handles with the halo carried
    by peer copies equals one whole-image handle (ptx_render_bands)."""
    from pathtracerdemo_amd.renderer import Renderer
    W, H = 96, 120
    whole = Renderer(W, H, device=0, pipeline="reuse")
    whole.Initialize(furnished)
    cuts = [0, 40, 78, H]
    bands = [Renderer(W, H, device=0, pipeline="reuse", row_begin=a, row_end=b) for a, b in zip(cuts, cuts[1:])]
    for b in bands:
        b.Initialize(furnished)
    for _ in range(2):
        whole.Update()
        whole.Render()
        for b in bands:
            b.Update()
        Renderer.render_bands(bands)
    ref = whole.read_image()
    got = np.concatenate([b.read_image() for b in bands], axis=0)
    np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
    for r in bands + [whole]:
        r.close()
