"""Resample counts at the BASELINE sizes against an independent stratified assignment.

The oracle's resampler is the reference's O(N^2) cumulative scan (PE:668-682) and cannot run at 1M-10M
particles.  Here the engine's counts are checked against tests/stratified_ref.py: the real-valued normalised
cumulative weights of the engine's OWN weights (extended precision), their running maximum, and a binary
search of the Philox targets r_k = (k + U_k) / N, restated in numpy.  Counts must be identical at every
particle except where a target lies within delta = 1e-12 of a cumulative boundary (there the reference's
sequential fp64 scan and the engine's parallel one may round it onto a neighbour: the 14-ulp window of
tests/test_gpu_resample_boundary.py), and their sum must be equal.

Configurations: C2's one-launch shape (100k, k_frame2), C3 (M=12, B=200 heavy, 1M, fp32), C4 (10M, fp16
state), C5's per-GPU stream (1M, fp32), each on a steady frame and on a frame with one LED hidden (all 80
iterations, so the kept slot and the resample stream follow the best iteration).
"""
import numpy as np
import pytest

import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn
import stratified_ref as sref
from test_gpu_parity import make_engine

pytestmark = pytest.mark.gpu

CASES = {
    "C2": (pf.STATE_F32, pf.SHAPE_FRAME2),
    "C3": (pf.STATE_F32, pf.SHAPE_TWO_LAUNCH),
    "C4": (pf.STATE_F16, pf.SHAPE_TWO_LAUNCH),
    "C5": (pf.STATE_F32, pf.SHAPE_TWO_LAUNCH),
}


@pytest.mark.parametrize("name", list(CASES))
def test_counts_match_exact_stratified_assignment(name):
    state, shape = CASES[name]
    cfg = syn.CONFIGS[name]
    st = syn.make_stream(cfg, 2)
    eng = make_engine(cfg.N, st.markers, st.K, state, pf.RNG_PHILOX)
    eng.set_prior(st.prior(fast=True))
    stats = []
    try:
        for f, fr in enumerate(st.frames):
            blobs, kw = fr.blobs, {}
            if f == 1:  # one LED's blob hidden: the exit rule never fires (PE:616), 80 iterations
                uv0 = syn.project(st.K, fr.truth, st.markers)[0]
                blobs = np.delete(blobs, int(np.argmin(np.sum((blobs - uv0) ** 2, axis=1))), axis=0)
                if name == "C3":  # 12 LEDs among 200 heavy outliers: an outlier near LED 0 can still let the exit
                    kw = {"force_iters": 80}  # rule fire, so the 80 iterations are forced (pfmpe_frame_in.force_iters)
            seed = 5151 + 7 * f
            out = eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=blobs, dt=fr.dt,
                                          seed=seed, frame_idx=f, **kw)).as_dict()
            assert eng.info(pf.INFO_LAST_SHAPE) == shape
            assert out["accepted"] == 1 and out["resampled"] == 1
            if f == 1:
                assert out["iters"] == 80
            w = eng.get_weights()  # the kept iteration's weights
            counts = eng.get_counts()
            r = sref.philox_targets(cfg.N, seed, f)
            s = sref.compare_counts(counts, w, r)
            assert s["not_found"] == 0
            assert out["winner_idx"] == int(np.argmax(counts))
            stats.append(s)
            del w, counts, r
    finally:
        eng.close()
    print(name, stats)
