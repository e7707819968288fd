"""The JS CPU baseline (pathtracerdemo_amd/js/cpu/pt_cpu.js): the reference's
live pipeline restated in the reference's host language, run on Node worker_threads.  Its
G-buffer, reservoirs and radiance must equal the C oracle's bit for bit, so the baseline the
bench times is the same computation as the GPU path's."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from helpers import uniform_for

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node")
BENCH = os.path.join(ROOT, "pathtracerdemo_amd", "js", "cpu", "bench_cpu.js")
pytestmark = pytest.mark.skipif(NODE is None, reason="node is not installed")


@pytest.mark.parametrize("scene,W,H,rows", [("dummy_scene_1", 32, 24, (0, 24)), ("c3_interior_32", 40, 28, (5, 21))])
def test_js_frame_bit_exact_vs_oracle(tmp_path, oracle_mod, scene, W, H, rows):
    from pathtracerdemo_amd.scene.export import export_compiled
    from pathtracerdemo_amd.scene.world import compile_scene
    cs = compile_scene(scene)
    d = export_compiled(cs, str(tmp_path / "scene"), scene)
    u = uniform_for(cs, W, H, 3)
    ufile = str(tmp_path / "u.bin")
    u.astype("<u4").tofile(ufile)
    prefix = str(tmp_path / "out")
    out = subprocess.run([NODE, BENCH, d, ufile, "3", str(rows[0]), str(rows[1]), prefix], capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    fr = oracle_mod.Frame(u, cs.scene, cs.geometry, cs.accel)
    fr.run(oracle_mod.PASS_RESTIR, threads=4, rect=(0, rows[0], W, rows[1]))
    y0, y1 = rows
    gb = np.fromfile(prefix + ".gbuffer.bin", np.uint32).reshape(H, W, 4)
    res = np.fromfile(prefix + ".reservoir.bin", np.uint32).reshape(H, W, 32)
    acc = np.fromfile(prefix + ".accum.bin", np.float32).reshape(H, W, 4)
    np.testing.assert_array_equal(gb[y0:y1], fr.gbuffer[y0:y1])
    np.testing.assert_array_equal(res[y0:y1], fr.reservoir[y0:y1])
    np.testing.assert_array_equal(acc[y0:y1].view(np.uint32), fr.accum[y0:y1].view(np.uint32))
