"""Multi-band frames on the GPU (SURVEY.md §8e, configs[3]): the frame split into row bands,
each band a handle with halo rows, the spatial-reuse halo exchanged on the device
(ptx_render_bands: peer copies between the handles of one process, or their RCCL
communicators).  The bar: the bands reproduce the single-handle frame BIT FOR BIT, and the
single handle is itself pinned to the oracle (test_gpu_reuse.py); small splits are checked
against the oracle directly.  Plus the work census the cost-balanced split is cut from.
"""
import os

import numpy as np
import pytest

from helpers import uniform_for

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from pathtracerdemo_amd import _native
    return _native


def make(cs, W, H, pipeline="reuse", radius=30, **kw):
    from pathtracerdemo_amd.renderer import Renderer
    r = Renderer(W, H, device=0, pipeline=pipeline, reuse_radius=radius, **kw)
    r.Initialize(cs)
    return r


def assert_same(got, want, what):
    got, want = np.asarray(got), np.asarray(want)
    if got.dtype != np.uint32:
        got, want = got.view(np.uint32), want.view(np.uint32)
    bad = np.any(got != want, axis=-1)
    assert bad.sum() == 0, f"{what}: {bad.sum()} pixels differ, first at {np.argwhere(bad)[:4].tolist()}"


def render_split(cs, W, H, cuts, frames, pipeline="reuse", radius=30, overlap=False):
    from pathtracerdemo_amd.renderer import Renderer
    bounds = [0] + list(cuts) + [H]
    bands = [make(cs, W, H, pipeline, radius, row_begin=bounds[i], row_end=bounds[i + 1], halo_overlap=overlap)
             for i in range(len(bounds) - 1)]
    img = np.zeros((H, W, 4), np.float32)
    for _ in range(frames):
        for b in bands:
            b.Update()
        Renderer.render_bands(bands, img)
    hist = np.concatenate([b.read_history() for b in bands])
    for b in bands:
        b.close()
    return hist, img


@pytest.mark.parametrize("overlap", [False, True])
def test_bands_small_split_matches_oracle(scene1, oracle_mod, overlap):
    """Three unequal bands (peer-copied halos, radius 12) reproduce the whole-frame oracle."""
    O, W, H, R = oracle_mod, 72, 80, 12
    fr = O.Frame(uniform_for(scene1, W, H, 1), scene1.scene, scene1.geometry, scene1.accel)
    fr.reuse = (R, 3, 20)
    for f in (1, 2, 3):
        fr.set_frame_index(f)
        fr.run_reuse_frame(threads=8)
    hist, img = render_split(scene1, W, H, [17, 50], 3, radius=R, overlap=overlap)
    assert_same(hist, fr.res_hist, "spatial output")
    assert_same(img, fr.accum, "radiance")


@pytest.mark.parametrize("cuts,overlap", [
    ([270 * i for i in range(1, 8)], False),                      # 8 equal bands of 270 rows
    ([270 * i for i in range(1, 8)], True),                       # the same, interior rows overlapped
    ([301, 563, 820, 1081, 1339, 1600, 1861], True),              # cost-balanced style, ragged
])
def test_c4_4k_eight_bands_bit_identical_to_one_handle(scene3, cuts, overlap):
    """configs[3]: the C3 reuse frame at 3840x2160 as 8 band handles (halo carried through
    device buffers) equals one 4K handle bit for bit, 3 frames (history included)."""
    W, H = 3840, 2160
    one = make(scene3, W, H)
    for _ in range(3):
        one.Update()
        one.Render()
    want_hist, want_img = one.read_history(), one.read_image()
    one.close()
    hist, img = render_split(scene3, W, H, cuts, 3, overlap=overlap)
    assert_same(hist, want_hist, "spatial output")
    assert_same(img, want_img, "radiance")
    assert np.isfinite(img).all()


def test_gi_bands_bit_identical(scene3):
    """ReSTIR GI as 3 bands with peer-copied halos equals the single handle."""
    W, H = 256, 160
    one = make(scene3, W, H, "gi")
    for _ in range(2):
        one.Update()
        one.Render()
    hist, img = render_split(scene3, W, H, [40, 100], 2, pipeline="gi", overlap=True)
    assert_same(hist, one.read_history(), "GI spatial output")
    assert_same(img, one.read_image(), "GI radiance")


def test_handle_owned_communicator_world_one(scene3):
    """ptx_comm_init (ncclCommInitRank, world 1): the handle renders through the RCCL band
    path and matches the plain handle."""
    from pathtracerdemo_amd.renderer import Renderer
    W, H = 128, 96
    a, b = make(scene3, W, H), make(scene3, W, H)
    b.comm_init(Renderer.comm_unique_id(), 0, 1)
    for _ in range(2):
        for r in (a, b):
            r.Update()
            r.Render()
    assert_same(b.read_history(), a.read_history(), "spatial output")
    assert_same(b.read_image(), a.read_image(), "radiance")


def test_render_bands_rejects_gaps(scene3):
    from pathtracerdemo_amd.renderer import Renderer
    from pathtracerdemo_amd import _native as N
    W, H = 64, 120
    bands = [make(scene3, W, H, row_begin=0, row_end=40), make(scene3, W, H, row_begin=50, row_end=120)]
    for b in bands:
        b.Update()
    with pytest.raises(N.PtxError):
        Renderer.render_bands(bands)


def test_row_census(scene3, oracle_mod, native):
    """PTX_FLAG_ROW_CENSUS: per tile row, the G-buffer pass's work equals the oracle's for
    those rows exactly; every pass's census sums to the plain counting build's totals; the
    census handle renders the same frame."""
    O, W, H = oracle_mod, 96, 72  # 12 tiles per row: one queue slot per tile row
    cen = make(scene3, W, H, row_census=True)
    cnt = make(scene3, W, H, count_work=True)
    fr = O.Frame(uniform_for(scene3, W, H, 1), scene3.scene, scene3.geometry, scene3.accel)
    keys = ("rays", "instance_xforms", "aabb_tests", "tri_tests", "hits")
    for r in (cen, cnt):
        r.Update()
        r.reset_stats()
        r.run_pass(native.PTX_PASS_GBUFFER)
    g = cen.row_census()
    for t in range(g.shape[0]):
        c = fr.run(O.PASS_GBUFFER, 4, (0, 8 * t, W, min(H, 8 * t + 8)))
        assert [int(v) for v in g[t]] == [c[k] for k in keys], f"tile row {t}"
    for p in (native.PTX_PASS_INIT, native.PTX_PASS_TEMPORAL, native.PTX_PASS_SPATIAL, native.PTX_PASS_FINAL):
        for r in (cen, cnt):
            r.reset_stats()
            r.run_pass(p)
        tot = cen.row_census().sum(axis=0)
        assert [int(v) for v in tot] == [cnt.read_counters()[k] for k in keys], f"pass {p}"
        if p in (native.PTX_PASS_INIT, native.PTX_PASS_SPATIAL):  # (temporal / final may trace nothing)
            assert tot[0] > 0
    assert_same(cen.read_history(), cnt.read_history(), "census handle frame")


def test_halo_skip_band_interior_rows(scene3):
    """PTX_FLAG_HALO_SKIP (a band timed alone, bench.py's calibration): the band renders its
    frames through the rank's band path (pipelined) without the exchange.  Frame f's spatial pass
    reads rows up to R away, whose temporal output carries frame f-1's spatial output there (the
    history): a stale halo reaches f * R rows into the band after f frames, and the rows farther
    than that from both band edges equal the whole frame's."""
    W, H, R, b0, b1, F = 96, 200, 12, 50, 170, 3
    one = make(scene3, W, H, radius=R)
    band = make(scene3, W, H, radius=R, row_begin=b0, row_end=b1, halo_skip=True)
    for _ in range(F):
        for r in (one, band):
            r.Update()
            r.Render()
    lo, hi = F * R, (b1 - b0) - F * R
    assert_same(band.read_history()[lo:hi], one.read_history()[b0 + lo:b0 + hi], "interior spatial output")
    assert_same(band.read_image()[lo:hi], one.read_image()[b0 + lo:b0 + hi], "interior radiance")
    assert band.stats()["frames"] == 3
    one.close()
    band.close()


def test_halo_proxy_band_timed_alone_in_the_shipped_library(tmp_path):
    """PTX_AB=HALO_PROXY_US=n (the exchange's one-GPU stand-in for a band timed alone: its edge
    rows copied into its own halo rows, then an n-microsecond wait on the exchange stream) is
    honoured by the shipped library -- no "not honoured" warning -- and changes no interior row."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = f"""
import sys, time, numpy as np
sys.path.insert(0, {root!r}); sys.path.insert(0, {os.path.join(root, 'tests')!r})
from pathtracerdemo_amd.scene.world import compile_scene
from pathtracerdemo_amd import _native as N
from test_gpu_bands import make
cs = compile_scene('c3_interior_32')
W, H, R, b0, b1, F = 96, 200, 12, 50, 170, 3
one = make(cs, W, H, radius=R)
band = make(cs, W, H, radius=R, row_begin=b0, row_end=b1, halo_skip=True)
t0 = time.perf_counter()
for _ in range(F):
    for r in (one, band):
        r.Update(); r.Render()
band.synchronize(); one.synchronize()
dt = time.perf_counter() - t0
lo, hi = F * R, (b1 - b0) - F * R
assert np.array_equal(band.read_history()[lo:hi].view(np.uint32), one.read_history()[b0 + lo:b0 + hi].view(np.uint32))
assert dt >= F * 0.02, dt
print('ok', N.build_info()['ptx_ab_ignored'])
"""
    env = dict(os.environ, PTX_AB="HALO_PROXY_US=20000")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300, cwd=root)
    assert p.returncode == 0, p.stderr[-3000:]
    assert p.stdout.strip().splitlines()[-1] == "ok []"
    assert "not honoured" not in p.stderr


def test_pipelined_band_frames_with_host_reads(scene3):
    """Band frames run two in flight (the next frame's G-buffer + PT_1 beside this frame's
    exchange, spatial pass and PT_4): host reads between frames see the latest frame, and the
    split still equals the single handle after every frame."""
    from pathtracerdemo_amd.renderer import Renderer
    W, H = 160, 120
    one = make(scene3, W, H)
    bands = [make(scene3, W, H, row_begin=a, row_end=b) for a, b in ((0, 37), (37, 90), (90, 120))]
    img = np.zeros((H, W, 4), np.float32)
    for f in range(4):
        one.Update()
        one.Render()
        for b in bands:
            b.Update()
        Renderer.render_bands(bands, img if f % 2 else None)
        hist = np.concatenate([b.read_history() for b in bands])
        assert_same(hist, one.read_history(), f"spatial output, frame {f + 1}")
        assert_same(np.concatenate([b.read_image() for b in bands]), one.read_image(), f"radiance, frame {f + 1}")
    for r in [one] + bands:
        r.close()


# tests/test_gpu_reuse.py's interactive camera path (5 units/s at 60 Hz, a yaw turn, still frames)
MOTION_PATH = [((0.0, 0.0, 6.0), 0.0), ((0.083, 0.0, 6.0), 0.0), ((0.166, 0.0, 5.95), 0.0),
               ((0.25, 0.02, 5.9), 1.5), ((0.25, 0.02, 5.9), 3.0), ((0.2, 0.02, 5.85), 4.5),
               ((0.2, 0.02, 5.85), 4.5), ((0.12, 0.0, 5.8), 3.0)]


def pose(r, loc, yaw, pitch=0.0):
    r.GetCamera().set_location(*loc)
    r.GetCamera().set_yaw(yaw)
    r.GetCamera().set_pitch(pitch)
    r.Update()


@pytest.mark.parametrize("cuts,overlap", [([32, 64], False), ([30, 63], True)])
def test_moving_camera_bands_bit_identical(scene3, cuts, overlap):
    """A moving camera through band handles (ptx_render_bands, peer copies): each band reprojects
    its history, the previous frame's spatial output of the rows above / below it arriving first
    as the motion halo (reuse_radius rows, the neighbours' band rows); after every frame of the
    path the split equals the single handle bit for bit, no reprojection left a band's motion
    halo, and the reprojected history was used."""
    from pathtracerdemo_amd.renderer import Renderer
    W, H = 96, 96
    one = make(scene3, W, H)
    bounds = [0] + cuts + [H]
    bands = [make(scene3, W, H, row_begin=a, row_end=b, halo_overlap=overlap) for a, b in zip(bounds, bounds[1:])]
    for f, (loc, yaw) in enumerate(MOTION_PATH, start=1):
        pose(one, loc, yaw)
        one.Render()
        for b in bands:
            pose(b, loc, yaw)
        Renderer.render_bands(bands)
        hist = np.concatenate([b.read_history() for b in bands])
        assert_same(hist, one.read_history(), f"spatial output, frame {f}")
        assert_same(np.concatenate([b.read_reservoir() for b in bands]), one.read_reservoir(), f"temporal output, frame {f}")
        assert_same(np.concatenate([b.read_image() for b in bands]), one.read_image(), f"radiance, frame {f}")
    assert sum(b.read_counters()["motion_clips"] for b in bands) == 0
    assert (one.read_reservoir()[..., 29] > 1).mean() > 0.3  # the history survived the moves
    for r in [one] + bands:
        r.close()


def test_band_motion_past_the_halo_is_split_invariant(scene3, oracle_mod):
    """A pitch jump that moves rows by more than the motion halo (R = 6 rows): the build's motion
    rule gives no history to a reprojection more than R rows away in EVERY handle (oracle
    motion_rows), so the 2-band split still equals one handle bit for bit, both count the same
    clipped pixels (PTX_COUNTER_MOTION_CLIP), and the one handle equals the oracle."""
    from pathtracerdemo_amd.renderer import Renderer
    from helpers import uniform_for
    W, H, R = 64, 96, 6
    one = make(scene3, W, H, radius=R)
    bands = [make(scene3, W, H, radius=R, row_begin=a, row_end=b) for a, b in ((0, 48), (48, 96))]
    fr = oracle_mod.Frame(uniform_for(scene3, W, H, 1), scene3.scene, scene3.geometry, scene3.accel)
    fr.reuse = (R, 3, 20)
    for f, pitch in enumerate((0.0, 0.0, 12.0, 12.0, 5.0), start=1):
        pose(one, (0.0, 0.0, 6.0), 0.0, pitch)
        one.Render()
        for b in bands:
            pose(b, (0.0, 0.0, 6.0), 0.0, pitch)
        img = np.zeros((H, W, 4), np.float32)
        Renderer.render_bands(bands, img)
        assert np.isfinite(img).all()
        assert_same(np.concatenate([b.read_reservoir() for b in bands]), one.read_reservoir(), f"temporal output, frame {f}")
        assert_same(np.concatenate([b.read_history() for b in bands]), one.read_history(), f"spatial output, frame {f}")
        assert_same(img, one.read_image(), f"radiance, frame {f}")
        fr.set_camera(one.uniform)
        fr.set_frame_index(f)
        fr.run_reuse_frame(threads=16)
        assert_same(one.read_image(), fr.accum, f"oracle radiance, frame {f}")
    clips = sum(b.read_counters()["motion_clips"] for b in bands)
    assert clips > 0 and clips == one.read_counters()["motion_clips"]
    for r in [one] + bands:
        r.close()


def test_communicator_band_moving_camera(scene3):
    """The RCCL band path (ptx_comm_init, world 1: no neighbours) along the moving-camera path:
    its motion temporal pass matches the plain handle's frame by frame."""
    from pathtracerdemo_amd.renderer import Renderer
    W, H = 96, 64
    a, b = make(scene3, W, H), make(scene3, W, H)
    b.comm_init(Renderer.comm_unique_id(), 0, 1)
    for f, (loc, yaw) in enumerate(MOTION_PATH[:5], start=1):
        for r in (a, b):
            pose(r, loc, yaw)
            r.Render()
        assert_same(b.read_history(), a.read_history(), f"spatial output, frame {f}")
        assert_same(b.read_image(), a.read_image(), f"radiance, frame {f}")
    for r in (a, b):
        r.close()


@pytest.mark.parametrize("cuts", [[48], [30, 63]])
def test_gi_moving_camera_bands_bit_identical(scene3, oracle_mod, cuts):
    """ReSTIR GI under a moving camera as band handles (ptx_render_bands: the motion halo brings
    the neighbours' rows of the previous spatial output, the static halo their G-buffer rows, which
    the moved frame's reprojection reads as the previous G-buffer): along the moving path plus a
    pitch jump past the R = 6 row halo, the split equals one handle bit for bit after every frame,
    both clip the same reprojections, and the one handle equals the oracle."""
    from pathtracerdemo_amd.renderer import Renderer
    from helpers import uniform_for
    W, H, R = 64, 96, 6
    one = make(scene3, W, H, "gi", radius=R)
    bounds = [0] + cuts + [H]
    bands = [make(scene3, W, H, "gi", radius=R, row_begin=a, row_end=b) for a, b in zip(bounds, bounds[1:])]
    fr = oracle_mod.Frame(uniform_for(scene3, W, H, 1), scene3.scene, scene3.geometry, scene3.accel)
    fr.reuse = (R, 3, 20)
    path = [(loc, yaw, 0.0) for loc, yaw in MOTION_PATH[:5]] + [((0.2, 0.02, 5.85), 4.5, 10.0),
                                                                  ((0.2, 0.02, 5.85), 4.5, 10.0)]
    for f, (loc, yaw, pitch) in enumerate(path, start=1):
        pose(one, loc, yaw, pitch)
        one.Render()
        for b in bands:
            pose(b, loc, yaw, pitch)
        img = np.zeros((H, W, 4), np.float32)
        Renderer.render_bands(bands, img)
        assert_same(np.concatenate([b.read_reservoir() for b in bands]), one.read_reservoir(), f"GI temporal output, frame {f}")
        assert_same(np.concatenate([b.read_history() for b in bands]), one.read_history(), f"GI spatial output, frame {f}")
        assert_same(img, one.read_image(), f"GI radiance, frame {f}")
        fr.set_camera(one.uniform)
        fr.set_frame_index(f)
        fr.run_gi_frame(threads=16)
        assert_same(one.read_image(), fr.accum, f"oracle GI radiance, frame {f}")
    clips = sum(b.read_counters()["motion_clips"] for b in bands)
    assert clips > 0 and clips == one.read_counters()["motion_clips"]
    assert (one.read_reservoir()[..., 11] > 1).mean() > 0.3
    for r in [one] + bands:
        r.close()
