"""Cell lists longer than one in the one-launch frame (k_frame2's column minima in phases over the markers,
DESIGN.md §4.2c; pf_kernels.hpp column_minima<..., PHASED>).

Every blob gets a twin 0.25-0.4 px away on each axis, so the cells around a blob list its twin too and a marker
that projects near a blob walks a list of two or more: the phased form's rare path.  The pruned one-launch frame
must give exactly the brute-force scan's records and weights, and exactly what the two-launch shape (the
per-marker form of the same grid walk, k_weigh_stream) gives."""
import numpy as np
import pytest

import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn
from test_gpu_parity import make_engine

pytestmark = pytest.mark.gpu


def twinned(blobs, rng):
    off = rng.uniform(0.25, 0.4, size=blobs.shape) * rng.choice([-1.0, 1.0], size=blobs.shape)
    both = np.concatenate([blobs, blobs + off])
    return both.astype(np.float32).astype(np.float64)


def test_long_cell_lists_one_launch_equals_brute_force_and_two_launches():
    N = 50_000
    st = syn.make_stream(syn.StreamConfig("t", M=5, B=40, N=N), 3)
    rng = np.random.default_rng(5)
    frames = [(fr, twinned(np.asarray(fr.blobs, dtype=np.float64), rng)) for fr in st.frames]
    runs = {}
    for fused, prune in ((2, True), (2, False), (0, True)):
        eng = make_engine(N, st.markers, st.K, pf.STATE_F32, pf.RNG_PHILOX, prune=prune, fused=fused)
        try:
            eng.set_prior(st.prior(fast=True))
            recs = []
            for f, (fr, blobs) in enumerate(frames):
                out = eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=blobs,
                                              dt=fr.dt, seed=41 + f, frame_idx=f)).as_dict()
                recs.append((out, eng.get_weights()))
            runs[(fused, prune)] = recs
        finally:
            eng.close()
    ref = runs[(2, False)]
    assert any(o["accepted"] for o, _ in ref)  # the markers do match (twinned) blobs
    for key in ((2, True), (0, True)):
        for f, ((a, wa), (b, wb)) in enumerate(zip(runs[key], ref)):
            for k, v in a.items():
                assert np.array_equal(np.asarray(v), np.asarray(b[k])), (key, f, k)
            assert np.array_equal(wa, wb), (key, f)
