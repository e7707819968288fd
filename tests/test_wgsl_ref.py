"""The C oracle pinned by an independent per-pixel restatement of the WGSL.

tests/wgsl_ref.py restates PT_01, PT_1, PT_4 and TEST_MCPT straight from the shader sources
(SH/PT_01_GBufferPass.wgsl:628-659, SH/PT_1_InitPass.wgsl:1361-1486,
SH/PT_4_FinalShadingPass.wgsl:1357-1428, SH/TEST_MCPT.wgsl:1315-1372) -- reading the reference
buffers as the shaders do, tracing with the literal WGSL stack walk over the 8-word BlasNode
records and the full [1e-4, 1e10] range -- not from oracle/pt_oracle.c.  On random pixels of
whole frames (two frames: the accumulation mix included) of the C1 Cornell room, the C3
32-light interior and the furnished C3 (13 instances), the oracle's G-buffer texels, all 32
words of every PT_1 reservoir and the radiance must equal the restatement's bit for bit.

The one documented difference: for a G-buffer miss the reference's PT_1 still shades the
garbage surface the zero texel decodes to, while the oracle (and the HIP kernels) write a
zero reservoir there; PT_4 never reads that reservoir (SH/PT_4_FinalShadingPass.wgsl:1404-1408),
and the radiance of those pixels is compared like every other.

CPU only (no GPU): the HIP kernels are compared with the oracle bit for bit by the -m gpu
suite, so this closes the chain reference WGSL -> restatement -> oracle -> HIP.
"""
import numpy as np
import pytest

import wgsl_ref as R
from helpers import uniform_for

CASES = [("dummy_scene_1", 256, 256, 160), ("c3_interior_32", 1920, 1080, 160), ("c3_furnished", 640, 360, 96)]


def _pixels(W, H, n, seed):
    rng = np.random.default_rng(seed)
    return [(int(x), int(y)) for x, y in zip(rng.integers(0, W, n), rng.integers(0, H, n))]


def test_fixed_sincos_restatement_is_the_oracles(oracle_mod):
    """The fixed f32 sin / cos as restated in wgsl_ref equals the oracle's on
    the whole sampling range [0, 2 PI]."""
    xs = np.linspace(0.0, 6.283184, 4001, dtype=np.float32)
    for x in xs:
        s, c = R.sincos(np.float32(x))
        assert np.float32(s).view(np.uint32) == np.float32(oracle_mod.fixed_sin(float(x))).view(np.uint32)
        assert np.float32(c).view(np.uint32) == np.float32(oracle_mod.fixed_cos(float(x))).view(np.uint32)


@pytest.mark.parametrize("name,W,H,npx", CASES)
def test_reference_pipeline_pixels_match_the_wgsl_restatement(oracle_mod, name, W, H, npx):
    """PT_01 -> PT_1 -> PT_4 (Renderer_TEST's live pipeline), frames 1 and 2."""
    from pathtracerdemo_amd.scene.world import compile_scene
    O = oracle_mod
    cs = compile_scene(name)
    fr = O.Frame(uniform_for(cs, W, H, 1), cs.scene, cs.geometry, cs.accel)
    pix = _pixels(W, H, npx, 11)
    acc = {p: np.zeros(4, np.float32) for p in pix}
    R.STATS.clear()
    hits = 0
    for f in (1, 2):
        fr.set_frame_index(f)
        fr.run(O.PASS_RESTIR, threads=8)
        sc = R.Scene(fr.uniform, cs.scene, cs.geometry, cs.accel)
        for x, y in pix:
            gw, ok, gcs = R.gbuffer_pixel(sc, x, y)
            np.testing.assert_array_equal(gw, fr.gbuffer[y, x], f"G-buffer texel ({x},{y}) frame {f}")
            rw = R.init_pixel(sc, x, y, gcs)
            if ok:
                hits += 1
                bad = np.nonzero(rw != fr.reservoir[y, x])[0]
                assert len(bad) == 0, (f"reservoir ({x},{y}) frame {f}: words {bad.tolist()} restated "
                                       f"{rw[bad].tolist()} oracle {fr.reservoir[y, x][bad].tolist()}")
            acc[(x, y)] = R.final_pixel(sc, x, y, gw, gcs, rw, acc[(x, y)])
            np.testing.assert_array_equal(acc[(x, y)].view(np.uint32), fr.accum[y, x].view(np.uint32),
                                          f"radiance ({x},{y}) after frame {f}")
    assert hits >= 64, f"only {hits} pixel-frames with a G-buffer hit"
    # the comparison went through the branches that matter
    for k in ("reconnection_light", "unshiftable_path", "russian_roulette_end", "pt4_replay_length_3"):
        assert R.STATS[k] > 0, f"{name}: no pixel exercised {k} ({dict(R.STATS)})"
    if name != "c3_furnished":
        assert R.STATS["btdf_sample"] > 0 and R.STATS["env_path"] > 0, dict(R.STATS)


@pytest.mark.parametrize("name,W,H,npx", [("dummy_scene_1", 256, 256, 128), ("c3_interior_32", 480, 270, 64)])
def test_test_mcpt_pixels_match_the_wgsl_restatement(oracle_mod, name, W, H, npx):
    """TEST_MCPT (the legacy brute-force pass, configs[1]'s workload), frames 1 and 2."""
    from pathtracerdemo_amd.scene.world import compile_scene
    O = oracle_mod
    cs = compile_scene(name)
    fr = O.Frame(uniform_for(cs, W, H, 1), cs.scene, cs.geometry, cs.accel)
    pix = _pixels(W, H, npx, 12)
    acc = {p: np.zeros(4, np.float32) for p in pix}
    for f in (1, 2):
        fr.set_frame_index(f)
        fr.run(O.PASS_MCPT, threads=8)
        sc = R.Scene(fr.uniform, cs.scene, cs.geometry, cs.accel)
        for x, y in pix:
            acc[(x, y)] = R.mcpt_pixel(sc, x, y, acc[(x, y)])
            np.testing.assert_array_equal(acc[(x, y)].view(np.uint32), fr.accum[y, x].view(np.uint32),
                                          f"TEST_MCPT radiance ({x},{y}) after frame {f}")
