"""ReSTIR GI (BASELINE configs[4]) on the CPU oracle: the build-defined rules of DESIGN.md §GI.

No reference code exists for GI, so the restatement is
pinned by what resampling requires of it: the reused estimator converges to the plain
one-candidate estimator's image (unbiased reconnection shift + pairwise MIS), the candidate
pdf is its sampler's true density (the condition a reconnection shift needs, which the
reference's PDF_BSDF does not meet for its SampleBSDF), and the shift is self-consistent.
"""
import numpy as np
import pytest

from helpers import uniform_for

W = H = 32
NORMAL = [0.0, 0.0, 1.0]
VIEW = np.array([0.3, 0.1, 0.9]) / np.linalg.norm([0.3, 0.1, 0.9])


def gi_frames(O, cs, n, mode, prm=(30, 3, 20), f0=1):
    """Per-frame radiance (n, H, W) of plain GI (the init candidate alone), spatial-only
    reuse (no history) or the full temporal + spatial pipeline."""
    fr = O.Frame(uniform_for(cs, W, H), cs.scene, cs.geometry, cs.accel)
    fr.reuse = prm
    out = np.zeros((n, H, W))
    for i, f in enumerate(range(f0, f0 + n)):
        fr.set_frame_index(f)
        fr.accum[:] = 0  # accum = mix(0, c, 1/(F+1)): the frame's own estimate, scaled
        fr.run(O.PASS_GBUFFER, 8)
        fr.run_gi(O.GI_PASS_INIT, 8)
        if mode == "plain":
            fr.gi_hist[:] = fr.gi_res
        else:
            fr.hist_valid = mode == "full" and f > f0
            fr.run_gi(O.GI_PASS_TEMPORAL, 8)
            fr.run_gi(O.GI_PASS_SPATIAL, 8)
        fr.run_gi(O.GI_PASS_FINAL, 8)
        out[i] = fr.accum[..., :3].astype(np.float64).mean(-1) * (f + 1)
    return out, (fr.gbuffer[..., 0] >> 31) == 1


@pytest.mark.parametrize("scene,prm", [("scene1", (3, 3, 0)), ("scene1", (30, 8, 0)), ("scene3", (3, 3, 0))])
def test_gi_spatial_reuse_is_unbiased_per_pixel(request, oracle_mod, scene, prm):
    """768 independent frames each: per-pixel z-scores of the mean difference vs the plain
    estimator have mean ~0 (the reference's SampleBSDF/PDF_BSDF as the candidate sampler
    gave mean z > 1.4 and +47 % image mean here)."""
    cs = request.getfixturevalue(scene)
    a, valid = gi_frames(oracle_mod, cs, 768, "plain", f0=100000)
    b, _ = gi_frames(oracle_mod, cs, 768, "spatial", prm)
    se = np.sqrt(a.var(0) / len(a) + b.var(0) / len(b)) + 1e-30
    z = ((b.mean(0) - a.mean(0)) / se)[valid]
    assert abs(z.mean()) < 0.2, z.mean()
    assert (np.abs(z) > 4.5).mean() < 0.01


def test_gi_temporal_spatial_converges_to_plain(oracle_mod, scene1):
    """The full pipeline (history capped at 20) over 1024 correlated frames: 8x8-block means
    within 4 % of plain's, far lower per-frame variance."""
    a, valid = gi_frames(oracle_mod, scene1, 1024, "plain", f0=100000)
    b, _ = gi_frames(oracle_mod, scene1, 1024, "full")
    blocks = lambda m: (m * valid).reshape(4, 8, 4, 8).sum((1, 3)) / np.maximum(valid.reshape(4, 8, 4, 8).sum((1, 3)), 1)
    ba, bb = blocks(a.mean(0)), blocks(b.mean(0))
    dense = valid.reshape(4, 8, 4, 8).sum((1, 3)) >= 16
    assert np.abs(bb / ba - 1)[dense].max() < 0.04, bb / ba
    assert abs(b.mean(0)[valid].mean() / a.mean(0)[valid].mean() - 1) < 0.015
    assert np.median(b.var(0)[valid] / a.var(0)[valid]) < 0.3


@pytest.mark.parametrize("mat", [[0.8, 0.8, 0.8, 0.0, 1.0, 0.0, 1.5], [0.8, 0.8, 0.8, 1.0, 0.3, 0.0, 1.5],
                                 [1.0, 1.0, 0.0, 0.0, 0.3, 0.9, 1.5]])
def test_gi_candidate_pdf_is_the_true_density(oracle_mod, mat):
    """E[|n.L| / pdf] over the sampler's own draws = the integral of |n.L| over its support
    (pi per hemisphere): exact for the GI sampler, every draw has pdf > 0."""
    O = oracle_mod
    seed, acc, n = 987654321, 0.0, 20000
    for _ in range(n):
        d, pdf, seed = O.gi_sample_dir(NORMAL, mat, VIEW, seed)
        assert pdf > 0.0 and abs(np.linalg.norm(d) - 1) < 1e-5
        acc += abs(d[2]) / pdf
    support = np.pi * ((mat[5] < 1.0) + (mat[5] > 0.0))
    assert abs(acc / n / support - 1) < 0.04, acc / n / support  # 4 sigma at T = 0.9


def test_reference_bsdf_pdf_is_not_its_sampling_density(oracle_mod):
    """Why GI does not draw its candidate with the reference's SampleBSDF: for a transmissive
    material PDF_BSDF is far from the density SampleBSDF draws with (E[|n.L|/pdf] ~ 2.5x the
    sphere's 2 pi), so a reconnection shift weighted by it is biased."""
    O = oracle_mod
    mat = [1.0, 1.0, 0.0, 0.0, 0.3, 0.9, 1.5]
    seed, acc, n = 12345, 0.0, 4000
    for _ in range(n):
        d, _, seed = O.sample_bsdf(NORMAL, mat, VIEW, seed)
        p = O.pdf_bsdf(NORMAL, mat, VIEW, d)
        acc += abs(d[2]) / p if p > 0 else 0.0
    assert acc / n / (2 * np.pi) > 1.5


def test_gi_shift_in_its_own_domain_reproduces_the_candidate(oracle_mod, scene3):
    """gi_shift of a pixel's own candidate into its own pixel gives back its stored
    contribution and q (up to the direction's rounding: the candidate used its sampled L1,
    the shift normalize(x2 - x1)); visible by construction."""
    O = oracle_mod
    fr = O.Frame(uniform_for(scene3, W, H), scene3.scene, scene3.geometry, scene3.accel)
    fr.run(O.PASS_GBUFFER, 4)
    fr.run_gi(O.GI_PASS_INIT, 4)
    checked = 0
    for y in range(0, H, 2):
        for x in range(0, W, 2):
            s = fr.gi_res[y, x]
            f = s[12:15].view(np.float32)
            if s[11] == 0 or not (s[0] >> 31) or f.sum() <= 0:
                continue
            ok, fs, q = fr.gi_shift(x, y, s)
            assert ok
            np.testing.assert_allclose(fs, f, rtol=2e-3, atol=1e-7)
            np.testing.assert_allclose(q, s[15:16].view(np.float32)[0], rtol=1e-4)
            checked += 1
    assert checked > 20


def test_gi_passes_are_deterministic_across_threads(oracle_mod, scene3):
    outs = []
    for threads in (1, 5):
        fr = oracle_mod.Frame(uniform_for(scene3, 20, 14), scene3.scene, scene3.geometry, scene3.accel)
        for f in (1, 2):
            fr.set_frame_index(f)
            fr.run_gi_frame(threads=threads)
        outs.append((fr.accum.copy(), fr.gi_hist.copy(), fr.direct.copy()))
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)


# ------------------------------------------------------------------ GI temporal reuse under camera motion
POSE_A = dict(location=(0.0, 0.0, 6.0))
POSE_B = dict(location=(0.15, 0.05, 6.1), yaw=2.0)  # test_reuse_oracle.py's poses


def gi_motion_estimates(O, cs, n, f0, reuse=True):
    """n independent two-frame sequences (pose B, then pose A): the pose-A frame's own estimate
    with the pose-B history reprojected (gi_temporal_motion_pixel) + spatial reuse, or plain
    GI (the init candidate alone) at pose A."""
    out = np.zeros((n, H, W))
    reused = 0
    for i in range(n):
        f = f0 + 2 * i
        fr = O.Frame(uniform_for(cs, W, H, f, **POSE_B), cs.scene, cs.geometry, cs.accel)
        if reuse:
            fr.run_gi_frame(threads=8)
        fr.set_camera(uniform_for(cs, W, H, f, **POSE_A))
        fr.set_frame_index(f + 1)
        fr.accum[:] = 0
        if reuse:
            assert fr.camera_moved()
            fr.run_gi_frame(threads=8)
            reused += int((fr.gi_res[..., 11] > 1).sum())
        else:
            fr.run(O.PASS_GBUFFER, 8)
            fr.run_gi(O.GI_PASS_INIT, 8)
            fr.gi_hist[:] = fr.gi_res
            fr.run_gi(O.GI_PASS_FINAL, 8)
        out[i] = fr.accum[..., :3].astype(np.float64).mean(-1) * (f + 2)
    return out, (fr.gbuffer[..., 0] >> 31) == 1, reused


@pytest.mark.parametrize("scene", ["scene1", "scene3"])
def test_gi_motion_temporal_reuse_is_unbiased_per_pixel(request, oracle_mod, scene):
    """GI temporal reuse with a moved camera (the history at the reprojection of the primary
    hit, reconnection-shifted out of the previous frame's domain, pairwise MIS with the shift of
    the canonical sample back) + spatial reuse vs plain GI at the new pose: per-pixel z-scores
    over 512 independent two-frame sequences have mean ~0, and the history is used for most
    pixels and lowers the variance."""
    O = oracle_mod
    cs = request.getfixturevalue(scene)
    a, valid, _ = gi_motion_estimates(O, cs, 512, 300000, reuse=False)
    b, _, reused = gi_motion_estimates(O, cs, 512, 100000)
    assert reused > 0.6 * 512 * valid.sum(), reused
    se = np.sqrt(a.var(0) / len(a) + b.var(0) / len(b)) + 1e-30
    z = ((b.mean(0) - a.mean(0)) / se)[valid]
    assert abs(z.mean()) < 0.2, z.mean()
    assert (np.abs(z) > 4.5).mean() < 0.01
    assert np.median(b.var(0)[valid] / a.var(0)[valid]) < 0.8


def test_gi_motion_reprojection_is_the_identity_for_a_still_camera(oracle_mod, scene3):
    """The GI motion rule with the previous pose equal to the current one: every pixel with a hit
    reprojects to itself, its history shifts back onto itself, and its output confidence is the
    same-pixel temporal pass's (1 + min(C_hist, cap)), its sample the same pixel's."""
    O = oracle_mod
    fr = O.Frame(uniform_for(scene3, W, H, 1), scene3.scene, scene3.geometry, scene3.accel)
    fr.run_gi_frame(threads=8)
    fr.set_frame_index(2)
    fr.run(O.PASS_GBUFFER, 8)
    fr.run_gi(O.GI_PASS_INIT, 8)
    hist = fr.gi_hist.copy()
    fr.run_gi_temporal_motion(threads=8)
    valid = (fr.gbuffer[..., 0] >> 31) == 1
    want = 1 + np.minimum(hist[..., 11], 20)
    np.testing.assert_array_equal(fr.gi_res[..., 11][valid], want[valid])
