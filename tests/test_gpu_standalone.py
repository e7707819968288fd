"""The product path without torch in the process (PTX_STANDALONE_RUNTIME=1): libptx.so binds
the HIP runtime it was built against (/opt/rocm), as a Node host does.  A child process
renders 3 reuse frames of the C1 scene at 48x40 and compares every buffer bit for bit with
the oracle; it also reports which libamdhip64 it mapped and that torch was never imported
(_native.share_torch_runtime is skipped)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys
import numpy as np
sys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})
from pathtracerdemo_amd import _native
from pathtracerdemo_amd.renderer import Renderer
from pathtracerdemo_amd.scene.world import compile_scene
from oracle import oracle as O
from helpers import uniform_for
_native.load()
cs = compile_scene("dummy_scene_1")
W, H = 48, 40
O.build()
fr = O.Frame(uniform_for(cs, W, H, 1), cs.scene, cs.geometry, cs.accel)
fr.reuse = (30, 3, 20)
r = Renderer(W, H, device=0, pipeline="reuse", reuse_radius=30, reuse_neighbors=3, temporal_cap=20)
r.Initialize(cs)
for f in range(1, 4):
    fr.set_frame_index(f)
    fr.run_reuse_frame(threads=4)
    r.Update()
    r.Render()
def same(a, b):
    return int(np.any(np.asarray(a).view(np.uint32) != np.asarray(b).view(np.uint32), axis=-1).sum())
bad = dict(temporal=same(r.read_reservoir(), fr.reservoir), spatial=same(r.read_history(), fr.res_hist),
           image=same(r.read_image(), fr.accum))
r.close()
maps = open("/proc/self/maps").read()
hip = sorted({{l.split()[-1] for l in maps.splitlines() if "libamdhip64" in l}})
print("RESULT " + json.dumps(dict(bad=bad, hip=hip, torch="torch" in sys.modules)))
"""


def test_standalone_runtime_reuse_frames_bit_exact():
    env = dict(os.environ, PTX_STANDALONE_RUNTIME="1")
    code = CHILD.format(root=ROOT, tests=os.path.join(ROOT, "tests"))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")][-1]
    res = json.loads(line[len("RESULT "):])
    assert not res["torch"], "torch was imported on the standalone path"
    assert res["hip"] and all("torch" not in h for h in res["hip"]), res["hip"]
    assert res["bad"] == {"temporal": 0, "spatial": 0, "image": 0}, res["bad"]
