"""Known-answer tests pinning the CPU oracle (oracle/pt_oracle.c) -- CPU only.

The reference ships no tests or golden data, so the oracle is pinned by
(1) published constants of the algorithms it restates, (2) an independent numpy/pure
Python restatement (tests/numpy_ref.py) and (3) analytic properties.
"""
import numpy as np
import pytest

import numpy_ref as ref


def test_pcg_known_answers(oracle_mod):
    # PCG RXS-M-XS hash (Jarzynski & Olano 2020, "Hash Functions for GPU Rendering"),
    # SH/PT_1_InitPass.wgsl:810-815; pcg(0) = 129708002 is the published value.
    expect = [129708002, 2831084092, 2055130248, 2131687100]
    assert [oracle_mod.pcg(i) for i in range(4)] == expect
    assert [ref.pcg(i) for i in range(4)] == expect
    rng = np.random.default_rng(7)
    for s in rng.integers(0, 2 ** 32, size=2000, dtype=np.uint64):
        assert oracle_mod.pcg(int(s)) == ref.pcg(int(s))


def test_random_is_hash_over_2_pow_32(oracle_mod):
    import ctypes
    lib = oracle_mod.lib()
    for s in [0, 1, 12345, 2 ** 32 - 1]:
        seed = ctypes.c_uint32(s)
        r = lib.pto_random(ctypes.byref(seed))
        exp, nxt = ref.random(s)
        assert np.float32(r) == exp and seed.value == nxt
    # f32(u32) rounds to nearest: hashes within 128 of 2^32 give exactly 1.0 (WGSL quirk)
    assert np.float32(np.float32(4294967295) / np.float32(4294967295.0)) == 1.0


def test_init_seed_formula(oracle_mod):
    """InitializeRandomSeed (SH/PT_1_InitPass.wgsl:823-826): u32 wrap-around."""
    x, y, f = 1919, 1079, 123456
    seed_in = (x * 1973 + y * 9277 + f * 26699) & 0xFFFFFFFF
    assert oracle_mod.pcg(seed_in) == ref.pcg(seed_in)


MISS = float(np.float32(1e11))


def test_ray_triangle_epsilons(oracle_mod):
    o = [0.25, 0.25, 1.0]
    d = [0.0, 0.0, -1.0]
    p0, p1, p2 = [0, 0, 0], [1, 0, 0], [0, 1, 0]
    assert oracle_mod.ray_triangle(o, d, p0, p1, p2, 1e-4) == pytest.approx(1.0)
    # behind the origin / at tMin -> miss (1e11)
    assert oracle_mod.ray_triangle([0.25, 0.25, -1.0], d, p0, p1, p2, 1e-4) == MISS
    # outside the barycentric range
    assert oracle_mod.ray_triangle([0.9, 0.9, 1.0], d, p0, p1, p2, 1e-4) == MISS
    # |det| between the G-buffer (1e-8) and the secondary-pass (1e-4) thresholds:
    # the same small triangle is hit by PT_01 and missed by PT_1
    s = 5e-3
    q0, q1, q2 = [0, 0, 0], [s, 0, 0], [0, s, 0]
    oo = [s / 4, s / 4, 1.0]
    assert oracle_mod.ray_triangle(oo, d, q0, q1, q2, 1e-8) == pytest.approx(1.0)
    assert oracle_mod.ray_triangle(oo, d, q0, q1, q2, 1e-4) == MISS


@pytest.mark.parametrize("metal,rough", [(0.0, 1.0), (0.0, 0.3), (1.0, 0.5), (0.5, 0.01)])
def test_brdf_matches_float64_restatement(oracle_mod, metal, rough):
    n = np.array([0, 0, 1], np.float32)
    albedo = np.array([0.8, 0.4, 0.2], np.float32)
    mat = np.array([*albedo, metal, rough, 0.0, 1.5], np.float32)
    rng = np.random.default_rng(3)
    for _ in range(50):
        v = rng.normal(size=3); v[2] = abs(v[2]) + 0.1; v /= np.linalg.norm(v)
        l = rng.normal(size=3); l[2] = abs(l[2]) + 0.1; l /= np.linalg.norm(l)
        got = oracle_mod.bsdf(n, mat, v.astype(np.float32), l.astype(np.float32))
        exp = ref.brdf(n, albedo, metal, rough, v, l)
        np.testing.assert_allclose(got, exp, rtol=2e-4, atol=1e-6)


def test_bsdf_transmission_split(oracle_mod):
    """BSDF = (1-T) BRDF in the same hemisphere, T * BTDF across (SH/PT_1_InitPass.wgsl:922-929)."""
    n = np.array([0, 0, 1], np.float32)
    mat_t = np.array([1, 1, 0, 0.0, 0.2, 1.0, 1.5], np.float32)   # fully transmissive
    v = np.array([0, 0.6, 0.8], np.float32)
    l_same = np.array([0.6, 0, 0.8], np.float32)
    l_across = np.array([0.1, -0.5, -0.86], np.float32)
    assert np.all(oracle_mod.bsdf(n, mat_t, v, l_same) == 0)
    assert np.all(oracle_mod.bsdf(n, mat_t, v, l_across) >= 0)
    mat_o = mat_t.copy(); mat_o[5] = 0.0
    assert np.all(oracle_mod.bsdf(n, mat_o, v, l_across) == 0)


def test_sample_bsdf_consumes_four_randoms(oracle_mod):
    """SampleBSDF draws exactly 4 Random(): lobe/transmission picks + 2 for the direction."""
    n = [0, 0, 1]
    v = [0, 0.6, 0.8]
    for mat in ([0.8, 0.8, 0.8, 0.0, 1.0, 0.0, 1.5], [0.5, 0.5, 0.5, 1.0, 0.3, 0.0, 1.5],
                [1, 1, 0, 0.0, 0.01, 1.0, 1.5]):
        for seed in range(0, 4000, 97):
            d, lobe, s2 = oracle_mod.sample_bsdf(n, mat, v, seed)
            assert s2 == seed + 4
            assert lobe in (0, 1)
            if mat[5] == 0.0 and lobe == 0:  # cosine lobe lies in the upper hemisphere
                assert d[2] >= 0 and abs(np.linalg.norm(d) - 1) < 1e-5


def test_pdf_brdf_integrates_to_about_one(oracle_mod):
    """Monte Carlo check: the opaque BRDF pdf integrates to ~1 over the hemisphere."""
    n = np.array([0, 0, 1], np.float32)
    mat = np.array([0.5, 0.5, 0.5, 0.0, 0.6, 0.0, 1.5], np.float32)
    v = np.array([0.0, 0.3, 0.95], np.float32); v /= np.linalg.norm(v)
    rng = np.random.default_rng(11)
    N = 20000
    u1, u2 = rng.random(N), rng.random(N)
    # uniform hemisphere directions, pdf 1/(2 pi)
    z = u1; r = np.sqrt(1 - z * z); phi = 2 * np.pi * u2
    dirs = np.stack([r * np.cos(phi), r * np.sin(phi), z], 1).astype(np.float32)
    vals = np.array([oracle_mod.pdf_bsdf(n, mat, v, l) for l in dirs])
    est = vals.mean() * 2 * np.pi
    assert 0.85 < est < 1.15


def test_fixed_transcendentals_are_faithful(oracle_mod):
    """The shared f32 sin/cos/pow5 (both sides use them instead of libm/ocml) stay within
    2 ulp of the float64 truth over the sampling domain [0, 2*PI_F] (plus pow5 on [0, 1])."""
    xs = np.float32(2.0 * 3.141592) * np.linspace(0.0, 1.0, 20001, dtype=np.float32)
    xs = np.concatenate([xs, np.float32([0.0, 1e-30, 1e-7, 0.7853981, 0.7853982, 6.283184])])
    for fn, ref in ((oracle_mod.fixed_sin, np.sin), (oracle_mod.fixed_cos, np.cos)):
        got = np.array([fn(float(x)) for x in xs], np.float32)
        truth = ref(xs.astype(np.float64))
        ulp = np.spacing(np.maximum(np.abs(truth), 2.0 ** -24).astype(np.float32)).astype(np.float64)
        err = np.abs(got.astype(np.float64) - truth) / ulp
        assert err.max() <= 2.0, (fn.__name__, float(xs[np.argmax(err)]), err.max())
    ps = np.linspace(0.0, 1.0, 5001, dtype=np.float32)
    got = np.array([oracle_mod.fixed_pow5(float(p)) for p in ps], np.float32).astype(np.float64)
    truth = ps.astype(np.float64) ** 5
    ulp = np.spacing(np.maximum(truth, 2.0 ** -126).astype(np.float32)).astype(np.float64)
    assert (np.abs(got - truth) / ulp).max() <= 3.0
