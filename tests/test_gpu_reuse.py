"""Reuse pipeline (temporal + spatial) on the GPU vs the CPU oracle,
through the C ABI.  Every reservoir and radiance value is compared BIT FOR BIT.

Each pass is first fed the oracle's inputs (so a mismatch is pinned to one kernel), then
whole frames run end to end (history included), on odd sizes, C3's 32 lights, a band pair
with the halo exchange, camera moves (history reprojected) and a full 1080p frame checked on
a row window the oracle can afford.
"""
import numpy as np
import pytest

from helpers import uniform_for

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from pathtracerdemo_amd import _native
    return _native


def reuse_renderer(cs, W, H, prm=(30, 3, 20), **kw):
    from pathtracerdemo_amd.renderer import Renderer
    r = Renderer(W, H, device=0, pipeline="reuse", reuse_radius=prm[0], reuse_neighbors=prm[1],
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


@pytest.mark.parametrize("prm", [(30, 3, 20), (4, 5, 2)])
def test_temporal_and_spatial_passes_bit_exact(scene1, oracle_mod, native, prm):
    """Each reuse pass alone on the oracle's inputs: temporal (history from the oracle's
    previous frame) then spatial."""
    O, W, H = oracle_mod, 64, 48
    fr = oracle_frame(O, scene1, W, H, prm)
    fr.set_frame_index(1)
    fr.run_reuse_frame(threads=8)
    fr.set_frame_index(2)
    for p in (O.PASS_GBUFFER, O.PASS_INIT_REUSE):
        fr.run(p)
    hist_prev = fr.res_hist.copy()
    r = reuse_renderer(scene1, W, H, prm)
    r.set_uniform(fr.uniform)
    r.write_buffer(native.PTX_BUF_GBUFFER, fr.gbuffer)
    r.write_buffer(native.PTX_BUF_RESERVOIR, fr.reservoir)
    r.write_buffer(native.PTX_BUF_RESERVOIR_HIST, hist_prev)
    r.write_buffer(native.PTX_BUF_ACCUM, fr.accum)  # frame 1's accumulation
    # the handle only trusts a history it wrote itself for this camera: run one spatial
    # pass first so the temporal pass below sees hist_valid, then restore the inputs
    r.run_pass(native.PTX_PASS_SPATIAL)
    r.write_buffer(native.PTX_BUF_RESERVOIR_HIST, hist_prev)
    r.run_pass(native.PTX_PASS_TEMPORAL)
    fr.run(O.PASS_TEMPORAL)
    assert (fr.reservoir[..., 29] > 1).any()
    assert_same(r.read_reservoir(), fr.reservoir, "temporal output")
    r.run_pass(native.PTX_PASS_SPATIAL)
    fr.run(O.PASS_SPATIAL)
    assert_same(r.read_history(), fr.res_hist, "spatial output")
    r.run_pass(native.PTX_PASS_FINAL)
    fr.run(O.PASS_FINAL_REUSE, reservoir=fr.res_hist)
    assert_same(r.read_image(), fr.accum, "PT_4 on the spatial output")
    r.close()


def test_spatial_confidence_past_the_summary_field(scene1, oracle_mod, native):
    """Confidences C >= 2^24 do not fit the spatial pass's 16-byte neighbour summary
    (ptx_reuse.hip wnbr_summary): those neighbours take the escape path (the reservoir itself
    is read) and the pass stays bit-exact.  Spatial pass alone, on the oracle's PT_1 output
    with every third reservoir's C raised past the field."""
    O, W, H = oracle_mod, 64, 48
    fr = oracle_frame(O, scene1, W, H)
    fr.set_frame_index(2)
    for p in (O.PASS_GBUFFER, O.PASS_INIT):
        fr.run(p)
    C = fr.reservoir[..., 29]
    big = (C > 0) & (np.arange(W * H).reshape(H, W) % 3 == 0)
    assert big.sum() > 100
    C[big] += np.uint32(0x00FFFFFF)
    r = reuse_renderer(scene1, W, H)
    r.set_uniform(fr.uniform)
    r.write_buffer(native.PTX_BUF_GBUFFER, fr.gbuffer)
    r.write_buffer(native.PTX_BUF_RESERVOIR, fr.reservoir)
    r.run_pass(native.PTX_PASS_SPATIAL)
    fr.run(O.PASS_SPATIAL)
    assert (fr.res_hist[..., 29] > 0x00FFFFFF).any()
    assert_same(r.read_history(), fr.res_hist, "spatial output with wide confidences")
    r.close()


@pytest.mark.parametrize("W,H,frames", [(48, 40, 4), (37, 23, 3), (1, 1, 2), (8, 1, 2), (130, 70, 2)])
def test_reuse_frames_bit_exact(scene1, oracle_mod, W, H, frames):
    O = oracle_mod
    fr = oracle_frame(O, scene1, W, H)
    r = reuse_renderer(scene1, W, H)
    for f in range(1, frames + 1):
        fr.set_frame_index(f)
        fr.run_reuse_frame(threads=8)
        r.Update()
        r.Render()
        assert r.uniform[23] == f
    assert_same(r.read_reservoir(), fr.reservoir, "temporal output")
    assert_same(r.read_history(), fr.res_hist, "spatial output")
    assert_same(r.read_image(), fr.accum, "accumulated radiance")
    r.close()


def test_reuse_frames_bit_exact_c3(scene3, oracle_mod):
    O, W, H = oracle_mod, 96, 64
    fr = oracle_frame(O, scene3, W, H)
    r = reuse_renderer(scene3, W, H)
    for f in (1, 2, 3):
        fr.set_frame_index(f)
        fr.run_reuse_frame(threads=8)
        r.Update()
        r.Render()
    assert_same(r.read_history(), fr.res_hist, "spatial output")
    assert_same(r.read_image(), fr.accum, "accumulated radiance")
    r.close()


def test_pass_by_pass_equals_render(scene1, native):
    W, H = 64, 40
    a = reuse_renderer(scene1, W, H)
    b = reuse_renderer(scene1, W, H, single_stream=True)
    for f in (1, 2, 3):
        a.Update()
        a.Render()
        b.Update()
        b.run_passes([native.PTX_PASS_GBUFFER, native.PTX_PASS_INIT, native.PTX_PASS_TEMPORAL])
        b.run_pass(native.PTX_PASS_SPATIAL)
        b.run_pass(native.PTX_PASS_FINAL)
    assert_same(a.read_history(), b.read_history(), "history")
    assert_same(a.read_image(), b.read_image(), "radiance")


def test_camera_move_reprojects_history(scene1, oracle_mod):
    """A new camera keeps the temporal history and reprojects it (the motion temporal pass,
    oracle temporal_motion_pixel): frame 3 after the move is bit-identical to the oracle's."""
    O, W, H = oracle_mod, 48, 32
    fr = oracle_frame(O, scene1, W, H)
    r = reuse_renderer(scene1, W, H)
    for f in (1, 2):
        fr.set_frame_index(f)
        fr.run_reuse_frame(threads=8)
        r.Update()
        r.Render()
    r.GetCamera().set_location(0.3, 0.1, 5.5)
    r.Update()
    r.Render()
    fr.set_camera(r.uniform)
    fr.set_frame_index(3)
    fr.run_reuse_frame(threads=8)
    assert_same(r.read_reservoir(), fr.reservoir, "temporal output after the move")
    assert_same(r.read_history(), fr.res_hist, "spatial output after the move")
    assert_same(r.read_image(), fr.accum, "radiance after the move")
    assert (fr.reservoir[..., 29][(fr.gbuffer[..., 0] >> 31) == 1] > 1).mean() > 0.5  # reprojected history used


# an interactive camera path: WebGPUEngine moves the camera by speed * dt per frame (5 units/s at
# 60 Hz, InputController.ts:81-159) and turns it with the mouse
CAMERA_PATH = [((0.0, 0.0, 6.0), 0.0), ((0.083, 0.0, 6.0), 0.0), ((0.166, 0.0, 5.95), 0.0),
               ((0.25, 0.02, 5.9), 1.5), ((0.25, 0.02, 5.9), 3.0), ((0.2, 0.02, 5.85), 4.5),
               ((0.2, 0.02, 5.85), 4.5), ((0.12, 0.0, 5.8), 3.0)]


@pytest.mark.parametrize("scene,W,H,single", [("scene1", 64, 48, False), ("scene3", 96, 64, False),
                                               ("scene3", 96, 64, True)])
def test_moving_camera_path_bit_exact(request, oracle_mod, scene, W, H, single):
    """Eight frames along CAMERA_PATH (translations of 5 units/s at 60 Hz, a yaw turn, two still
    frames) through the reuse pipeline, pipelined (two frames in flight) or one launch sequence:
    every frame's temporal output (motion pass on the moved frames), spatial output and the
    accumulated radiance are bit-identical to the oracle's; the reprojected history is used."""
    O = oracle_mod
    cs = request.getfixturevalue(scene)
    fr = oracle_frame(O, cs, W, H)
    r = reuse_renderer(cs, W, H, single_stream=single, time_launches=single)
    used = 0
    for f, (loc, yaw) in enumerate(CAMERA_PATH, start=1):
        r.GetCamera().set_location(*loc)
        r.GetCamera().set_yaw(yaw)
        r.Update()
        r.Render()
        fr.set_camera(r.uniform)
        fr.set_frame_index(f)
        moved = fr.hist_valid and fr.camera_moved()
        fr.run_reuse_frame(threads=16)
        if moved:
            used += int((fr.reservoir[..., 29] > 1).sum())
        if f in (2, 5, 8):
            assert_same(r.read_reservoir(), fr.reservoir, f"temporal output, frame {f}")
            assert_same(r.read_history(), fr.res_hist, f"spatial output, frame {f}")
            assert_same(r.read_image(), fr.accum, f"radiance, frame {f}")
    assert used > 0
    r.close()


def test_band_pair_with_halo_exchange_bit_exact(scene1, oracle_mod):
    """Two band handles on one GPU, halos swapped through device buffers (what RCCL carries
    between ranks): the bands reproduce the whole-frame oracle."""
    import torch
    O, W, H, prm = oracle_mod, 72, 64, (12, 3, 20)
    split = 30
    bands = [reuse_renderer(scene1, W, H, prm, row_begin=0, row_end=split),
             reuse_renderer(scene1, W, H, prm, row_begin=split, row_end=H)]
    rows = [b.halo_rows() for b in bands]
    assert rows[0][:2] == (0, 12) and rows[1][:2] == (12, 0)
    msg = [torch.empty(12 * rows[0][2], dtype=torch.uint8, device="cuda") for _ in range(2)]
    fr = oracle_frame(O, scene1, W, H, prm)
    for f in (1, 2, 3):
        fr.set_frame_index(f)
        fr.run_reuse_frame(threads=8)
        for b in bands:
            b.Update()
            b.run_passes([0, 1, 8])
        bands[0].halo_pack(None, msg[0].data_ptr())   # band 0's last rows go down
        bands[1].halo_pack(msg[1].data_ptr(), None)   # band 1's first rows go up
        for b in bands:
            b.synchronize()
        bands[0].halo_unpack(None, msg[1].data_ptr())
        bands[1].halo_unpack(msg[0].data_ptr(), None)
        for b in bands:
            b.run_passes([9, 2])
    hist = np.concatenate([b.read_history() for b in bands])
    img = np.concatenate([b.read_image() for b in bands])
    assert_same(hist, fr.res_hist, "spatial output")
    assert_same(img, fr.accum, "radiance")
    with pytest.raises(Exception):
        bands[0].Render()  # a band needs the halo exchange: ptx_render refuses it


def test_full_hd_reuse_window_bit_exact(scene1, oracle_mod):
    """1920x1080, 2 frames on the GPU; the oracle evaluates rows [y0 - 2R, y1 + 2R) (all
    that rows [y0, y1) of frame 2 depend on) and the window must match bit for bit."""
    O, W, H, R = oracle_mod, 1920, 1080, 30
    y0, y1 = 520, 528
    r = reuse_renderer(scene1, W, H)
    fr = oracle_frame(O, scene1, W, H)
    rect = (0, y0 - 2 * R, W, y1 + 2 * R)
    for f in (1, 2):
        r.Update()
        r.Render()
        fr.set_frame_index(f)
        fr.run_reuse_frame(threads=16, rect=rect)
    assert_same(r.read_history()[y0:y1], fr.res_hist[y0:y1], "spatial output (window)")
    assert_same(r.read_image()[y0:y1], fr.accum[y0:y1], "radiance (window)")
    st = r.stats()
    assert st["frames"] == 2 and st["kernel_launches"][7] == 2


def test_c3_full_hd_reuse_windows_bit_exact(scene3, oracle_mod):
    """The headline configuration itself (configs[2]: C3, 32 rect lights, 1920x1080, reuse
    pipeline, 2 frames with history) on the GPU; the oracle evaluates what 3 row windows
    (top edge, middle, bottom edge) of frame 2 depend on, and they must match bit for bit."""
    O, W, H, R = oracle_mod, 1920, 1080, 30
    windows = [(0, 8), (600, 608), (1072, 1080)]
    r = reuse_renderer(scene3, W, H)
    frs = [oracle_frame(O, scene3, W, H) for _ in windows]
    for f in (1, 2):
        r.Update()
        r.Render()
        for (y0, y1), fr in zip(windows, frs):
            fr.set_frame_index(f)
            fr.run_reuse_frame(threads=16, rect=(0, max(0, y0 - 2 * R), W, min(H, y1 + 2 * R)))
    hist, img = r.read_history(), r.read_image()
    for (y0, y1), fr in zip(windows, frs):
        assert_same(hist[y0:y1], fr.res_hist[y0:y1], f"spatial output rows {y0}..{y1}")
        assert_same(img[y0:y1], fr.accum[y0:y1], f"radiance rows {y0}..{y1}")
    assert np.isfinite(img).all()


def test_c3_4k_one_handle_windows_bit_exact(scene3, oracle_mod):
    """configs[3]'s frame on ONE handle -- C3, 3840x2160, reuse pipeline, 2 frames with history --
    under the 4K launch parameters (above 4 Mpx per band: trace at 5 waves per SIMD; frames
    pipelined, two in flight) vs the oracle on 3 row windows: the top edge, rows straddling the cut at row 1081
    of a cost-balanced 8-band split (and the 2-band cut at 1080), and the bottom edge.  The
    8-band tests (test_gpu_bands.py) compare bands with this one handle."""
    O, W, H, R = oracle_mod, 3840, 2160, 30
    windows = [(0, 8), (1076, 1086), (2152, 2160)]
    r = reuse_renderer(scene3, W, H)
    frs = [oracle_frame(O, scene3, W, H) for _ in windows]
    for f in (1, 2):
        r.Update()
        r.Render()
        for (y0, y1), fr in zip(windows, frs):
            fr.set_frame_index(f)
            fr.run_reuse_frame(threads=16, rect=(0, max(0, y0 - 2 * R), W, min(H, y1 + 2 * R)))
    hist, img = r.read_history(), r.read_image()
    for (y0, y1), fr in zip(windows, frs):
        assert_same(hist[y0:y1], fr.res_hist[y0:y1], f"spatial output rows {y0}..{y1}")
        assert_same(img[y0:y1], fr.accum[y0:y1], f"radiance rows {y0}..{y1}")
    assert np.isfinite(img).all()
    st = r.stats()
    assert st["frames"] == 2
    r.close()


@pytest.mark.gpu
def test_pipelined_frames_interleaved_with_host_ops(scene3, oracle_mod, native):
    """Frame pipelining (ptx_render runs frame N's G-buffer + PT_1 beside frame N-1's spatial
    pass, on a second context): host operations between frames -- buffer reads, an
    accumulation reset (which also drops the history), a camera move -- see and act on the
    latest frame exactly as with one frame in flight."""
    O, W, H = oracle_mod, 72, 56
    fr = oracle_frame(O, scene3, W, H)
    r = reuse_renderer(scene3, W, H)
    for f in range(1, 8):
        if f == 5:  # camera move: the handle reprojects the history itself
            r.GetCamera().set_location(0.25, 0.1, 5.5)
        r.Update()
        if f == 5:
            fr.set_camera(r.uniform)
        fr.set_frame_index(r.uniform[23])
        fr.run_reuse_frame(threads=8)
        r.Render()
        if f == 2:
            assert_same(r.read_history(), fr.res_hist, "spatial output, frame 2")
            assert_same(r.read_gbuffer(), fr.gbuffer, "G-buffer, frame 2")
        if f == 3:  # zero the accumulation and drop the history, as ptx_reset_accumulation does
            r.reset_accumulation()
            fr.accum[:] = 0.0
            fr.hist_valid = False
    assert_same(r.read_reservoir(), fr.reservoir, "temporal output")
    assert_same(r.read_history(), fr.res_hist, "spatial output")
    assert_same(r.read_image(), fr.accum, "accumulated radiance")
    r.close()


def test_pipelined_frames_beside_another_handle(scene1, scene3, oracle_mod):
    """A reuse handle created while another handle is alive (smoke()'s order): its one-time
    clears must be done before its non-blocking streams start (a null-stream hipMemset still
    in flight once zeroed part of the first pipelined frame's reservoirs)."""
    from pathtracerdemo_amd.renderer import Renderer
    O = oracle_mod
    other = Renderer(64, 64, device=0)
    other.Initialize(scene1)
    other.Update()
    other.Render()
    other.read_image()
    W, H = 48, 32
    fr = oracle_frame(O, scene3, W, H)
    r = reuse_renderer(scene3, W, H)
    for f in (1, 2, 3):
        fr.set_frame_index(f)
        fr.run_reuse_frame(threads=8)
        r.Update()
        r.Render()
    assert_same(r.read_reservoir(), fr.reservoir, "temporal output")
    assert_same(r.read_history(), fr.res_hist, "spatial output")
    assert_same(r.read_image(), fr.accum, "accumulated radiance")
    r.close()
    other.close()


def test_write_buffer_passes_beside_a_rendering_handle(scene1, scene3, oracle_mod, native):
    """Host copies into a handle's buffers (ptx_write_buffer) and its pass-by-pass launches
    while ANOTHER handle keeps pipelined frames in flight (never synchronised in between): every
    copy runs on the handle's own stream and is waited for there, so each pass reads exactly the
    bytes written (a null-stream copy is ordered before nothing on the handles' non-blocking
    streams).  Both handles match the oracle bit for bit."""
    O = oracle_mod
    Wb, Hb = 96, 64
    frb = oracle_frame(O, scene3, Wb, Hb)
    b = reuse_renderer(scene3, Wb, Hb)
    nb = 0

    def tick():
        nonlocal nb
        nb += 1
        b.Update()
        b.Render()
        frb.set_frame_index(nb)
        frb.run_reuse_frame(threads=8)

    W, H = 64, 48
    fr = oracle_frame(O, scene1, W, H)
    fr.set_frame_index(1)
    fr.run_reuse_frame(threads=8)
    fr.set_frame_index(2)
    for p in (O.PASS_GBUFFER, O.PASS_INIT_REUSE):
        fr.run(p)
    hist_prev = fr.res_hist.copy()
    a = reuse_renderer(scene1, W, H)
    a.set_uniform(fr.uniform)
    tick()
    a.write_buffer(native.PTX_BUF_GBUFFER, fr.gbuffer)
    tick()
    a.write_buffer(native.PTX_BUF_RESERVOIR, fr.reservoir)
    a.write_buffer(native.PTX_BUF_RESERVOIR_HIST, hist_prev)
    tick()
    a.write_buffer(native.PTX_BUF_ACCUM, fr.accum)
    a.run_pass(native.PTX_PASS_SPATIAL)  # (makes the handle trust the history, as in the pass test)
    tick()
    a.write_buffer(native.PTX_BUF_RESERVOIR_HIST, hist_prev)
    a.run_pass(native.PTX_PASS_TEMPORAL)
    tick()
    fr.run(O.PASS_TEMPORAL)
    assert_same(a.read_reservoir(), fr.reservoir, "temporal output")
    a.run_pass(native.PTX_PASS_SPATIAL)
    tick()
    fr.run(O.PASS_SPATIAL)
    assert_same(a.read_history(), fr.res_hist, "spatial output")
    a.run_pass(native.PTX_PASS_FINAL)
    fr.run(O.PASS_FINAL_REUSE, reservoir=fr.res_hist)
    assert_same(a.read_image(), fr.accum, "PT_4 on the spatial output")
    assert_same(b.read_history(), frb.res_hist, "the other handle's spatial output")
    assert_same(b.read_image(), frb.accum, "the other handle's radiance")
    a.close()
    b.close()
