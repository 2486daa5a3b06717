"""The oracle against the committed golden fixtures (tests/golden/, made by make_golden.py).

The reference ships no tests or fixtures and cannot be built here, so the fixtures are the oracle's own
outputs, frozen after the oracle passed its known-answer tests (test_oracle_kat.py): this file guards the
checker against drift.  tests/test_gpu_golden.py runs the same fixtures through the HIP engine.
"""
import os

import numpy as np
import pytest

from oracle import pforacle as orc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
STREAMS = ["pf_c1_reference_rng", "pf_c1_philox", "pf_m12_heavy_philox"]
INT_KEYS = ("iters", "kept_iter", "accepted", "resampled", "most_likely_idx", "winner_idx", "n_corr", "flag_fail")


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz")))


def test_likelihood_vectors():
    g = load("likelihood_vectors")
    for c in range(len(g["P"])):
        M, B = int(g["M"][c]), int(g["B"][c])
        proj, blobs, dg = g["proj"][c][:M], g["blobs"][c][:B], g["downgrade"][c][:M]
        for closed in (False, True):
            P, pairs = orc.likelihood(proj, blobs, float(g["tol"][c]), float(g["tol_pf"][c]), dg, closed=closed)
            assert P == g["P"][c], (c, closed)
            n = int(g["npairs"][c])
            assert len(pairs) == n and np.array_equal(pairs, g["pairs"][c][:n]), (c, closed)


@pytest.mark.parametrize("name", STREAMS)
def test_stream_fixture(name):
    g = load(name)
    prm = orc.make_params(rng_mode=int(g["rng_mode"]))
    prior = g["prior0"]
    for f in range(len(g["seed"])):
        B = int(g["B"][f])
        out, arr = orc.pf_step(g["markers"], g["K"], prm, prior, g["cur"][f], g["pred"][f], g["predm"][f],
                               g["blobs"][f][:B], dt=float(g["dt"][f]), seed=int(g["seed"][f]),
                               frame_idx=int(g["frame_idx"][f]))
        for k in INT_KEYS:
            assert out[k] == g[k][f], (name, f, k)
        n = out["n_corr"]
        assert np.array_equal(out["pairs"], g["pairs"][f][:n])
        np.testing.assert_allclose(arr["weights"], g["weights"][f], rtol=0, atol=1e-12)
        assert np.array_equal(arr["counts"], g["counts"][f])
        np.testing.assert_allclose(out["winner_pose"], g["winner_pose"][f], rtol=0, atol=1e-12)
        if out["resampled"]:
            prior = arr["resampled"]
    np.testing.assert_allclose(prior, g["final_prior"], rtol=0, atol=1e-12)
