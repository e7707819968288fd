"""ReSTIR GI pipeline (BASELINE configs[4]) on the GPU vs the CPU oracle,
through the C ABI.  Reservoirs, direct light and radiance are compared BIT FOR BIT: each
pass alone on the oracle's inputs first (a mismatch is pinned to one kernel), then whole
frames (history included) on odd sizes, both scenes, a band pair with the halo exchange
and a 1080p frame checked on the row window the oracle can afford.
"""
import numpy as np
import pytest

from helpers import uniform_for

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from pathtracerdemo_amd import _native
    return _native


def gi_renderer(cs, W, H, prm=(30, 3, 20), **kw):
    from pathtracerdemo_amd.renderer import Renderer
    r = Renderer(W, H, device=0, pipeline="gi", reuse_radius=prm[0], reuse_neighbors=prm[1],
                 temporal_cap=prm[2], **kw)
    r.Initialize(cs)
    return r


def oracle_frame(O, cs, W, H, prm=(30, 3, 20)):
    fr = O.Frame(uniform_for(cs, W, H, 1), cs.scene, cs.geometry, cs.accel)
    fr.reuse = prm
    return fr


def assert_same(got, want, what):
    got, want = np.asarray(got), np.asarray(want)
    if got.dtype != np.uint32:
        got, want = got.view(np.uint32), want.view(np.uint32)
    bad = np.any(got != want, axis=-1)
    assert bad.sum() == 0, f"{what}: {bad.sum()} pixels differ, first at {np.argwhere(bad)[:4].tolist()}"


@pytest.mark.parametrize("scene", ["scene1", "scene3"])
def test_gi_passes_bit_exact(request, oracle_mod, native, scene):
    """init, temporal (with a history), spatial and final, each on the oracle's inputs."""
    cs = request.getfixturevalue(scene)
    O, W, H = oracle_mod, 64, 48
    fr = oracle_frame(O, cs, W, H)
    fr.set_frame_index(1)
    fr.run_gi_frame(threads=8)
    fr.set_frame_index(2)
    fr.run(O.PASS_GBUFFER)
    r = gi_renderer(cs, W, H)
    r.set_uniform(fr.uniform)
    r.write_buffer(native.PTX_BUF_GBUFFER, fr.gbuffer)
    r.run_pass(native.PTX_PASS_INIT)
    fr.run_gi(O.GI_PASS_INIT)
    assert_same(r.read_reservoir(), fr.gi_res, "GI init reservoirs")
    assert_same(r.read_direct(), fr.direct, "direct light")
    hist_prev = fr.gi_hist.copy()
    r.run_pass(native.PTX_PASS_SPATIAL)  # makes the handle's history valid for this camera
    r.write_buffer(native.PTX_BUF_RESERVOIR, fr.gi_res)
    r.write_buffer(native.PTX_BUF_RESERVOIR_HIST, hist_prev)
    r.write_buffer(native.PTX_BUF_ACCUM, fr.accum)
    r.run_pass(native.PTX_PASS_TEMPORAL)
    fr.run_gi(O.GI_PASS_TEMPORAL)
    assert (fr.gi_res[..., 11] > 1).any()
    assert_same(r.read_reservoir(), fr.gi_res, "GI temporal output")
    r.run_pass(native.PTX_PASS_SPATIAL)
    fr.run_gi(O.GI_PASS_SPATIAL)
    assert_same(r.read_history(), fr.gi_hist, "GI spatial output")
    r.run_pass(native.PTX_PASS_FINAL)
    fr.run_gi(O.GI_PASS_FINAL)
    assert_same(r.read_image(), fr.accum, "GI radiance")
    r.close()


@pytest.mark.parametrize("W,H,frames,prm", [(48, 40, 4, (30, 3, 20)), (37, 23, 3, (4, 5, 2)), (1, 1, 2, (30, 3, 20)),
                                            (8, 1, 2, (30, 3, 20)), (130, 70, 2, (30, 3, 20))])
def test_gi_frames_bit_exact(scene3, oracle_mod, W, H, frames, prm):
    O = oracle_mod
    fr = oracle_frame(O, scene3, W, H, prm)
    r = gi_renderer(scene3, W, H, prm)
    for f in range(1, frames + 1):
        fr.set_frame_index(f)
        fr.run_gi_frame(threads=8)
        r.Update()
        r.Render()
    assert_same(r.read_reservoir(), fr.gi_res, "temporal output")
    assert_same(r.read_history(), fr.gi_hist, "spatial output")
    assert_same(r.read_image(), fr.accum, "accumulated radiance")
    r.close()


def test_gi_band_pair_with_halo_exchange_bit_exact(scene3, oracle_mod):
    """Two GI band handles, halos (G-buffer + 64-byte GI reservoirs) through device buffers."""
    import torch
    O, W, H, prm = oracle_mod, 72, 64, (12, 3, 20)
    split = 30
    bands = [gi_renderer(scene3, W, H, prm, row_begin=0, row_end=split),
             gi_renderer(scene3, W, H, prm, row_begin=split, row_end=H)]
    rows = [b.halo_rows() for b in bands]
    assert rows[0][:2] == (0, 12) and rows[1][:2] == (12, 0) and rows[0][2] == W * (16 + 64)
    msg = [torch.empty(12 * rows[0][2], dtype=torch.uint8, device="cuda") for _ in range(2)]
    fr = oracle_frame(O, scene3, W, H, prm)
    for f in (1, 2, 3):
        fr.set_frame_index(f)
        fr.run_gi_frame(threads=8)
        for b in bands:
            b.Update()
            b.run_passes([0, 1, 8])
        bands[0].halo_pack(None, msg[0].data_ptr())
        bands[1].halo_pack(msg[1].data_ptr(), None)
        for b in bands:
            b.synchronize()
        bands[0].halo_unpack(None, msg[1].data_ptr())
        bands[1].halo_unpack(msg[0].data_ptr(), None)
        for b in bands:
            b.run_passes([9, 2])
    assert_same(np.concatenate([b.read_history() for b in bands]), fr.gi_hist, "spatial output")
    assert_same(np.concatenate([b.read_image() for b in bands]), fr.accum, "radiance")


def test_full_hd_gi_window_bit_exact(scene3, oracle_mod):
    """1920x1080, 2 GI frames; the oracle evaluates rows [y0 - 2R, y1 + 2R)."""
    O, W, H, R = oracle_mod, 1920, 1080, 30
    y0, y1 = 600, 608
    r = gi_renderer(scene3, W, H)
    fr = oracle_frame(O, scene3, W, H)
    rect = (0, y0 - 2 * R, W, y1 + 2 * R)
    for f in (1, 2):
        r.Update()
        r.Render()
        fr.set_frame_index(f)
        fr.run_gi_frame(threads=16, rect=rect)
    assert_same(r.read_history()[y0:y1], fr.gi_hist[y0:y1], "spatial output (window)")
    assert_same(r.read_image()[y0:y1], fr.accum[y0:y1], "radiance (window)")
    img = r.read_image()
    assert np.isfinite(img).all()


# tests/test_gpu_bands.py's moving-camera path, then a pitch jump past the reuse radius
GI_MOTION_PATH = [((0.0, 0.0, 6.0), 0.0, 0.0), ((0.083, 0.0, 6.0), 0.0, 0.0), ((0.166, 0.0, 5.95), 0.0, 0.0),
                  ((0.25, 0.02, 5.9), 1.5, 0.0), ((0.25, 0.02, 5.9), 3.0, 0.0), ((0.2, 0.02, 5.85), 4.5, 0.0),
                  ((0.2, 0.02, 5.85), 4.5, 0.0), ((0.12, 0.0, 5.8), 3.0, 9.0), ((0.12, 0.0, 5.8), 3.0, 9.0)]


def gi_pose(r, loc, yaw, pitch):
    c = r.GetCamera()
    c.set_location(*loc)
    c.set_yaw(yaw)
    c.set_pitch(pitch)
    r.Update()


@pytest.mark.parametrize("scene,W,H,prm", [("scene3", 64, 48, (30, 3, 20)), ("scene1", 45, 38, (6, 2, 20)),
                                           ("scene3", 80, 64, (8, 3, 5))])
def test_gi_moving_camera_bit_exact(request, oracle_mod, scene, W, H, prm):
    """GI temporal reuse under camera motion (wgim_start / wgim_combine: the history at the
    reprojection of the primary hit, reconnection shifts both ways, pairwise MIS) along a moving
    path with still frames and a pitch jump past the reuse radius: temporal output, spatial output
    and radiance equal the oracle's (gi_temporal_motion_pixel) after every frame, and the
    reprojected history carries most pixels on the moved frames."""
    cs = request.getfixturevalue(scene)
    O = oracle_mod
    r = gi_renderer(cs, W, H, prm)
    fr = oracle_frame(O, cs, W, H, prm)
    used = []
    for f, (loc, yaw, pitch) in enumerate(GI_MOTION_PATH, start=1):
        gi_pose(r, loc, yaw, pitch)
        moved = fr.hist_valid and bool(np.any(np.asarray(r.uniform)[4:23] != fr.prev_uniform[4:23]))
        fr.set_camera(r.uniform)
        fr.set_frame_index(int(r.uniform[23]))
        fr.run_gi_frame(threads=8)
        r.Render()
        assert_same(r.read_reservoir(), fr.gi_res, f"temporal output, frame {f}")
        assert_same(r.read_history(), fr.gi_hist, f"spatial output, frame {f}")
        assert_same(r.read_image(), fr.accum, f"radiance, frame {f}")
        if moved:
            valid = (fr.gbuffer[..., 0] >> 31) == 1
            used.append(float((fr.gi_res[..., 11][valid] > 1).mean()))
    assert len(used) >= 5 and max(used) > 0.6, used
    if (W, prm[0]) == (80, 8):  # the 9-degree pitch moves rows by more than R = 8 at this size
        assert r.read_counters()["motion_clips"] > 0
    r.close()
