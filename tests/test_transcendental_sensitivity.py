"""How far WGSL's implementation-defined transcendentals can move the image.

WGSL leaves `pow` (SH/PT_1_InitPass.wgsl:859, Fresnel) and `sin` / `cos` (:945-946,
:963-964, BSDF sampling angles) to the backend: pow is typically exp2(y * log2 x) and sin /
cos only promise an absolute error of 2^-11 on [-pi, pi].  The oracle and the HIP kernels
share one fixed f32 definition of each (pt_oracle.c pow5_ / sincos_, ptx_shading.h), which is
what makes them bit-exact with each other; these tests measure what that choice costs
against other admissible backends, on oracle builds that swap the definitions (PTO_TRANSC):

  * libm powf / sinf / cosf                        -> image rel. L2 ~1e-5 (C1), ~1e-6 (C3)
  * pow lowered as exp2(5 log2 x)                  -> indistinguishable from libm
  * sin / cos off by e absolute (hashed sign)      -> 1.8e-2 (C1) / 3.1e-2 (C3) at e = 2^-11;
    the north-star bar 1e-3 holds for e <= 2^-17 (C1 5e-4 floor: a 256x256 4-frame image
    has few samples, so the few 1-spp paths that flip weigh more)

So "1e-3 relative L2 vs the WebGPU reference" is achievable against any backend whose sin /
cos are within ~2^-17 (every mainstream GPU's hardware sin is), and not against one that uses
the spec's full 2^-11 allowance: at 1 spp a `Random() < P` decision or a sampled direction
that moves by 5e-4 re-routes whole paths.  Parity here stays bit-exact against the fixed
definitions; these numbers bound the gap to a real WebGPU backend.
"""
import ctypes

import pytest

from tests.helpers import rel_l2, uniform_for


def render(oracle_mod, cs, W, H, frames, variant, rect=None):
    fr = oracle_mod.Frame(uniform_for(cs, W, H, 1), cs.scene, cs.geometry, cs.accel, variant=variant)
    for f in range(1, frames + 1):
        fr.set_frame_index(f)
        fr.run(oracle_mod.PASS_RESTIR, threads=8, rect=rect)
    img = fr.accum if rect is None else fr.accum[rect[1]:rect[3], rect[0]:rect[2]]
    return img[..., :3]


@pytest.fixture(scope="module")
def c1_fixed(oracle_mod, scene1):
    return render(oracle_mod, scene1, 256, 256, 4, "")


def test_libm_transcendentals_within_north_star_bar(oracle_mod, scene1, c1_fixed):
    err = rel_l2(render(oracle_mod, scene1, 256, 256, 4, "libm"), c1_fixed)
    assert 0.0 < err < 1e-4, err  # measured 2.8e-5: a handful of ulp-level differences


def test_pow_as_exp2_log2_is_harmless(oracle_mod, scene1, c1_fixed):
    err = rel_l2(render(oracle_mod, scene1, 256, 256, 4, "wgsl_pow"), c1_fixed)
    assert err < 1e-4, err


def test_sincos_at_wgsl_bound_exceeds_bar_and_small_error_meets_it(oracle_mod, scene1, c1_fixed):
    lib = oracle_mod.lib("wgsl_sincos")
    lib.pto_set_sincos_error.argtypes = [ctypes.c_float]
    try:
        lib.pto_set_sincos_error(2.0 ** -11)
        coarse = rel_l2(render(oracle_mod, scene1, 256, 256, 4, "wgsl_sincos"), c1_fixed)
        lib.pto_set_sincos_error(2.0 ** -17)
        fine = rel_l2(render(oracle_mod, scene1, 256, 256, 4, "wgsl_sincos"), c1_fixed)
    finally:
        lib.pto_set_sincos_error(2.0 ** -11)
    assert 1e-2 < coarse < 5e-2, coarse  # measured 1.76e-2
    assert fine < 1e-3, fine             # measured 5.3e-4


def test_c3_window_sensitivity(oracle_mod, scene3):
    """C3 (32 lights) at 1080p, one 64-row window, one frame: libm 5.9e-7, 2^-11 sin/cos 3.1e-2."""
    rect = (0, 512, 1920, 576)
    base = render(oracle_mod, scene3, 1920, 1080, 1, "", rect)
    assert rel_l2(render(oracle_mod, scene3, 1920, 1080, 1, "libm", rect), base) < 1e-5
    lib = oracle_mod.lib("wgsl_sincos")
    lib.pto_set_sincos_error.argtypes = [ctypes.c_float]
    lib.pto_set_sincos_error(2.0 ** -11)
    assert rel_l2(render(oracle_mod, scene3, 1920, 1080, 1, "wgsl_sincos", rect), base) > 1e-2
