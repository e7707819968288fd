"""The shared-reciprocal f3 division of ptx_device.h (`operator/(f3, float)`, PTX_SHARED_DIV).

On gfx950 the compiler's f32 `a / s` is v_div_scale x2, v_rcp, the FMA chain, v_div_fmas and
v_div_fixup -- a correctly rounded quotient.  The kernels' f3 / s shares one refined reciprocal
over three numerators and, inside the operand window where v_div_scale is an identity, runs
the same chain without the scale steps.  This checks on the CPU, with exact FMA arithmetic,
that the chain is correctly rounded in that window for every reciprocal v_rcp_f32 may return
(within 1 ulp of 1/s): two correctly rounded results are the same bits, so the GPU's fast path
equals the compiler's division there (the GPU tests then check the kernels bit for bit).
"""
from fractions import Fraction

import numpy as np

F32 = np.float32


def rn32(x: Fraction) -> np.float32:
    """Round an exact rational to the nearest f32 (ties to even), no double rounding."""
    q = F32(float(x))
    best = None
    for c in (np.nextafter(q, F32(-np.inf)), q, np.nextafter(q, F32(np.inf))):
        d = abs(Fraction(float(c)) - x)
        if best is None or d < best[0] or (d == best[0] and (int(c.view(np.uint32)) & 1) == 0):
            best = (d, c)
    return F32(best[1])


def fma(a, b, c) -> np.float32:
    return rn32(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c)))


def mul(a, b) -> np.float32:
    return rn32(Fraction(float(a)) * Fraction(float(b)))


def chain(a, s, y0):
    """ptx_device.h: y = fma(fma(-s, y0, 1), y0, y0); div_by_rcp(a, s, y) before v_div_fixup."""
    y = fma(fma(-s, y0, F32(1)), y0, y0)
    q = mul(a, y)
    r = fma(-s, q, a)
    q = fma(r, y, q)
    r = fma(-s, q, a)
    return fma(r, y, q)


def test_chain_is_correctly_rounded_in_the_window():
    rng = np.random.default_rng(7)
    n = 0
    for _ in range(1500):
        s = F32(rng.uniform(0.5, 1.0) * 2.0 ** int(rng.integers(-40, 41)))  # frexp exponent in [-40, 40]
        if rng.random() < 0.2:  # mantissas at the ends of the binade (the hard reciprocals)
            s = F32(np.ldexp(F32(1) - F32(2.0 ** -24) * int(rng.integers(0, 4)), int(rng.integers(-40, 40))))
        ys = F32(1) / s
        for y0 in (np.nextafter(ys, F32(0)), ys, np.nextafter(ys, F32(np.inf))):  # v_rcp_f32: within 1 ulp
            for _ in range(3):
                a = F32(rng.uniform(0.5, 1.0) * 2.0 ** int(rng.integers(-50, 51)) * (1 if rng.random() < 0.5 else -1))
                if rng.random() < 0.2:  # exact quotients and their neighbours
                    a = np.nextafter(F32(s * F32(int(rng.integers(1, 1 << 12)))), F32(np.inf) if rng.random() < .5 else F32(0))
                    if not (2.0 ** -51 <= abs(float(a)) < 2.0 ** 50):
                        continue
                assert chain(a, s, y0) == a / s, (a, s, y0)
                n += 1
    assert n > 10000
