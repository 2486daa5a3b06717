"""An independent O(N log N) restatement of the stratified resampler (PE:666-682), for checking the engine's
resample counts at full BASELINE sizes (1M-10M particles) where the oracle's O(N^2) cumulative scan cannot
run.  Test infrastructure only (imported by tests/), never by the product.

What the reference computes (PE:627-682): normalise the weights by their fp64 sum, then for each stratified
target r_k = (k + U_k) / N take the first particle i whose sequential cumulative sum c_i reaches r_k.  The
first such i is also the first i whose running maximum max(c_0..c_i) reaches r_k, so the assignment is a
binary search over the running maximum.  Here the cumulative sums are formed in x87 extended precision
(numpy longdouble: 64-bit significand) of the exact fp32-valued weights, divided by the extended sum: that
is the real-valued normalised cumulative weight to ~1e-16, i.e. the value both the reference's sequential
fp64 scan and the engine's parallel scan approximate (each within a few hundred ulp).
A target within `delta` of a boundary is FRAGILE: there the two roundings may put it on a neighbouring
particle (tests/test_gpu_resample_boundary.py builds such a case on purpose: 14 ulp apart).  Every other
target has exactly one correct particle.

The Philox4x32-10 stream of the resampling targets is restated in numpy (counter {k, 2 << 24, frame_lo,
frame_hi}, key = seed, u53 from the first two words: pf_rng.hpp, oracle/pf_oracle.cpp); tests/
test_resample_search.py pins it against the oracle's Philox and its KAT.
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 (Salmon et al., SC'11) on uint32 counter arrays; scalar key words."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) & MASK32 for c in (c0, c1, c2, c3))
    k0, k1 = int(k0) & 0xFFFFFFFF, int(k1) & 0xFFFFFFFF
    for r in range(10):
        if r:
            k0 = (k0 + W0) & 0xFFFFFFFF
            k1 = (k1 + W1) & 0xFFFFFFFF
        p0 = M0 * c0
        p1 = M1 * c2
        n0 = (p1 >> np.uint64(32)) ^ c1 ^ np.uint64(k0)
        n1 = p1 & MASK32
        n2 = (p0 >> np.uint64(32)) ^ c3 ^ np.uint64(k1)
        n3 = p0 & MASK32
        c0, c1, c2, c3 = n0, n1, n2, n3
    return c0, c1, c2, c3


def philox_targets(N, seed, frame_idx):
    """r_k = fl(fl(k + U_k) / N), k = 0..N-1, the Philox resampling stream (kTagResample = 2)."""
    k = np.arange(N, dtype=np.uint64)
    z = np.zeros(N, dtype=np.uint64)
    o0, o1, _, _ = philox4x32_10(k, z + np.uint64(2 << 24), z + np.uint64(frame_idx & 0xFFFFFFFF),
                                 z + np.uint64((frame_idx >> 32) & 0xFFFFFFFF), seed & 0xFFFFFFFF, seed >> 32)
    u = ((o0 >> np.uint64(5)).astype(np.float64) * 67108864.0 + (o1 >> np.uint64(6)).astype(np.float64)) \
        * (1.0 / 9007199254740992.0)
    return (np.arange(N, dtype=np.float64) + u) / N


def assign(weights, r):
    """First-index assignment of every target against the running max of the real-valued normalised
    cumulative weights; returns (idx, runmax) with idx = N where no particle reaches the target."""
    w = np.asarray(weights, dtype=np.longdouble)
    S = w.sum()
    c = np.cumsum(w) / S
    R = np.maximum.accumulate(c)
    return np.searchsorted(R, np.asarray(r, dtype=np.longdouble), side="left"), R


def compare_counts(gpu_counts, weights, r, delta=1e-12):
    """Check the engine's counts against the exact assignment.  delta bounds |engine c_i - exact c_i| with a
    wide margin (the engine's three-level fp64 scan errs by at most ~(8 + 64 + groups) ulp, < 1e-13 at 10M;
    DESIGN.md §4.4).  Returns a dict of statistics; raises AssertionError on a mismatch outside the fragile
    set.  A fragile target may land on any particle whose running max lies within delta of it."""
    gpu = np.asarray(gpu_counts, dtype=np.int64)
    N = gpu.size
    idx, R = assign(weights, r)
    exact = np.bincount(idx[idx < N], minlength=N)[:N]
    rl = np.asarray(r, dtype=np.longdouble)
    lo = np.searchsorted(R, rl - delta, side="left")   # first particle that may take the target
    hi = np.searchsorted(R, rl + delta, side="left")   # last particle that may take it (N: none)
    fragile_t = np.flatnonzero(hi > lo)
    fragile = np.zeros(N + 1, dtype=bool)
    for t in fragile_t:  # few (~2 delta N^2 / N per frame)
        fragile[lo[t]:min(hi[t], N - 1) + 1] = True
    fragile = fragile[:N]
    diff = gpu - exact
    bad = np.flatnonzero((diff != 0) & ~fragile)
    assert bad.size == 0, (f"{bad.size} counts differ outside the fragile set; first {bad[:10].tolist()}: "
                           f"gpu {gpu[bad[:10]].tolist()} exact {exact[bad[:10]].tolist()}")
    assert gpu.sum() == exact.sum(), (gpu.sum(), exact.sum())
    assert np.abs(diff).sum() <= 2 * fragile_t.size, (np.abs(diff).sum(), fragile_t.size)
    return {"N": N, "fragile_targets": int(fragile_t.size), "fragile_particles": int(fragile.sum()),
            "differing": int(np.count_nonzero(diff)), "not_found": int(np.count_nonzero(idx >= N))}
