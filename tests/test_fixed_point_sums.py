"""The fixed-point wave sums of k_resample / k_weigh_pk (pf_kernels.hpp wave_incl_sum_fx, pf_weigh_pk.hpp
pk_wave_partial) against the fp64 DPP scan they replace, in numpy.

Claim: every fp32 weight of an M >= 4 frame is a multiple of 2^-21 (its score terms Mt + q^2 are >= 4 and the
penalties are integers), so for a wave whose weights all lie in [0, 32) the u32 scan of w * 2^21 is exact and every
fp64 association of the same weights (the kernels' row_shr / row_bcast scan, the butterfly total) gives the same
bits.  The weights here are built the way score_unordered builds them (fp32 operations in its order)."""
import numpy as np

F = np.float32


def scores(rng, n, m=5, tol=F(3.0), tol_pf=F(4.0), downgrade=0b00100):
    """score_unordered (pf_kernels.hpp) in fp32: accepted markers add Mt + q^2, then the penalties."""
    d = rng.uniform(0.0, 5.0, size=(n, m)).astype(F)
    d[rng.random((n, m)) < 0.1] = F(np.inf)
    blob = rng.integers(0, 6, size=(n, m))
    rtol = F(1.0) / tol
    mt = F(m)
    pr = np.zeros(n, dtype=F)
    dups = np.zeros(n, dtype=np.int64)
    ndg = np.zeros(n, dtype=np.int64)
    acc = d <= tol_pf
    for j in range(m):
        q = (tol - d[:, j]) * rtol
        t = mt + q * q
        pr = np.where(acc[:, j], pr + t, pr).astype(F)
        dup = np.zeros(n, dtype=bool)
        for e in range(j):
            dup |= acc[:, e] & (blob[:, e] == blob[:, j])
        dups += (acc[:, j] & dup).astype(np.int64)
        ndg += (acc[:, j] & bool((downgrade >> j) & 1)).astype(np.int64)
    pen = (3 * dups * (dups + 1) // 2 + 2 * ndg).astype(F)
    return (pr - pen).astype(F)


def dpp_scan_f64(x):
    """wave_incl_sum: row_shr 1/2/4/8 with zero fill inside 16-lane rows, then row_bcast 15 (rows 1, 3) and
    row_bcast 31 (rows 2, 3), in fp64, the kernels' association."""
    x = x.astype(np.float64).copy()
    lane = np.arange(64)
    for s in (1, 2, 4, 8):
        src = lane - s
        v = np.where((src >= 0) & (src // 16 == lane // 16), x[np.clip(src, 0, 63)], 0.0)
        x = x + v
    row = lane // 16
    b15 = np.where(np.isin(row, (1, 3)), x[row * 16 - 1], 0.0)
    x = x + b15
    b31 = np.where(np.isin(row, (2, 3)), x[31], 0.0)
    return x + b31


def test_weights_on_the_2pow21_grid():
    rng = np.random.default_rng(7)
    w = scores(rng, 200000)
    pos = w[w >= 0]
    scaled = pos.astype(np.float64) * 2.0 ** 21
    assert np.all(scaled == np.round(scaled)), "a weight off the 2^-21 grid"
    assert np.all(pos < 32.0)


def test_fixed_point_scan_equals_fp64_scan():
    rng = np.random.default_rng(11)
    w = scores(rng, 64 * 4000)
    waves = w.reshape(-1, 64)
    checked = 0
    for wv in waves:
        if np.any(wv < 0) or np.any(wv >= 32):
            continue  # the kernels keep the fp64 scan for such a wave
        ints = (wv.astype(np.float64) * 2.0 ** 21).astype(np.uint64)
        prefix = np.cumsum(ints)
        assert prefix[-1] < 2 ** 32
        fx = prefix.astype(np.float64) * 2.0 ** -21
        f64 = dpp_scan_f64(wv)
        assert np.array_equal(fx.view(np.uint64), f64.view(np.uint64))
        checked += 1
    assert checked > 3000
