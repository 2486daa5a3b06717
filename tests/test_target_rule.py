"""The resampler's division-free target test (csrc/pf_kernels.hpp target_le) against the reference's division.

The stratified resampler (PE:666-682) compares targets r_k = fl(fl(k + U_k) / N) with the running-max
cumulative weight x.  target_le decides r_k <= x from the sign of fma(x, N, -a) (a = fl(k + U_k)) and falls back
to the division only when a lies within ~2^-50 relative of x*N.  Here the same rule runs in Python: the fma is
the correctly rounded exact residual (fractions.Fraction), Python's float division is IEEE.  Cases are
adversarial: x at, just below and just above fl(a/N), and at the band edges, for N up to 10M."""
from fractions import Fraction
import math

import numpy as np
import pytest


def fma(x, y, z):
    if math.isinf(x) or math.isinf(y) or math.isinf(z):
        return x * y + z  # IEEE: inf propagates (no finite rounding involved)
    return float(Fraction(x) * Fraction(y) + Fraction(z))  # one rounding, like v_fma_f64


def target_le(a, N, x):
    xn = x * N
    thr = fma(xn, 2.0 ** -50, 2.0 ** -1000)
    e = fma(x, float(N), -a)
    if e >= 0.0:
        return True
    if -e > thr:
        return False
    return a / N <= x


@pytest.mark.parametrize("N", [1, 3, 1000, 100_000, 1_000_000, 10_000_000])
def test_rule_equals_division(N):
    rng = np.random.default_rng(N)
    k = rng.integers(0, N, 400)
    U = rng.integers(0, 2 ** 53, 400) * 2.0 ** -53  # u53 draws
    fallbacks = 0
    for kk, u in zip(k, U):
        a = float(kk) + float(u)
        r = a / N
        for x in (r, math.nextafter(r, math.inf), math.nextafter(r, -math.inf), r * (1 + 2 ** -49), r * (1 - 2 ** -49),
                  r * (1 + 2 ** -51), r * (1 - 2 ** -51), (a + 0.5) / N, 0.0, 1.0, math.inf):
            assert target_le(a, N, x) == (r <= x), (a, N, x)
            e = fma(x, float(N), -a)
            fallbacks += e < 0.0 and -e <= fma(x * N, 2.0 ** -50, 2.0 ** -1000)
    assert fallbacks < 400 * 8  # the division runs only in the narrow band


def test_zero_target_and_zero_x():
    assert target_le(0.0, 10, 0.0)          # r_0 = 0 with U = 0
    assert not target_le(2.0 ** -53, 10, 0.0)
