"""The integer wave reductions of pf_kernels.hpp, simulated lane by lane in numpy (no GPU).

* The reduction pattern of wave_argmin_dist / the winner-key maxima: quad_perm [1,0,3,2], quad_perm [2,3,0,1],
  row_half_mirror, row_mirror, then row_bcast15 (rows 1, 3) and row_bcast31 (rows 2, 3).  Lane 63 ends with the
  whole wave's result even though the bcast steps leave the rows they do not write holding garbage (mov_dpp without
  bound_ctrl: an undefined old value), which the test fills with random values.
* wave_argmin_dist (pose_pairs): the minimum of the fp32 distances' bits, then the lowest
  original index among the lanes holding it, equals wave_argmin's lexicographic (distance, index) minimum for
  distances >= +0 that are never NaN (+inf lanes and ties included)."""
import numpy as np

LANE = np.arange(64)


def dpp_src(ctrl):
    """source lane of every lane for a DPP control, or -1 where the row is not written"""
    row, i = LANE // 16, LANE % 16
    if ctrl == "xor1":
        return LANE ^ 1
    if ctrl == "xor2":
        return LANE ^ 2
    if ctrl == "half_mirror":
        return (LANE // 8) * 8 + 7 - (LANE % 8)
    if ctrl == "mirror":
        return row * 16 + 15 - i
    if ctrl == "bcast15":
        return np.where(np.isin(row, (1, 3)), row * 16 - 1, -1)
    if ctrl == "bcast31":
        return np.where(np.isin(row, (2, 3)), 31, -1)
    raise ValueError(ctrl)


def reduce_lane63(k, op, rng):
    k = k.copy()
    for ctrl in ("xor1", "xor2", "half_mirror", "mirror", "bcast15", "bcast31"):
        src = dpp_src(ctrl)
        garbage = rng.integers(np.iinfo(np.int32).min, np.iinfo(np.int32).max, size=64, dtype=np.int64)
        moved = np.where(src >= 0, k[np.clip(src, 0, 63)], garbage)
        k = op(k, moved)
    return int(k[63])


def test_pattern_reduces_the_whole_wave():
    rng = np.random.default_rng(3)
    for _ in range(2000):
        k = rng.integers(-2**31, 2**31 - 1, size=64, dtype=np.int64)
        assert reduce_lane63(k, np.minimum, rng) == k.min()
        assert reduce_lane63(k, np.maximum, rng) == k.max()


def lex_min(d, idx):
    best, arg = np.float32(np.inf), 0x7FFFFFFF
    for v, o in zip(d, idx):  # any order: the lexicographic minimum
        if v < best or (v == best and o < arg):
            best, arg = v, o
    return best, arg


def test_argmin_dist_equals_lexicographic_min():
    rng = np.random.default_rng(5)
    for case in range(3000):
        B = int(rng.integers(1, 64))
        d = np.full(64, np.inf, dtype=np.float32)
        idx = np.full(64, 0x7FFFFFFF, dtype=np.int64)
        vals = rng.choice(np.float32([0.0, 0.25, 1.0, 2.5, 7.0]), size=B) if case % 2 else \
            rng.uniform(0, 50, size=B).astype(np.float32)
        vals[rng.random(B) < 0.1] = np.inf
        d[:B] = vals
        idx[:B] = rng.permutation(200)[:B]  # the table's original blob indices, not the lane order
        keys = d.view(np.int32).astype(np.int64)
        K = reduce_lane63(keys, np.minimum, rng)
        c = np.where(keys == K, idx, 0x7FFFFFFF)
        I = reduce_lane63(c, np.minimum, rng)
        best, arg = lex_min(d, idx)
        assert np.int32(K).view(np.float32).tobytes() == np.float32(best).tobytes()
        assert I == arg
