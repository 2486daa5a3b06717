"""The HIP engine (fp64 parity mode, through the C-ABI) against the committed golden fixtures.

Bar: every discrete output identical (iterations, kept iteration, accept/flag, most-likely index, winner,
correspondences, per-particle resample counts); weights, poses and the final prior within 1e-9.
"""
import os

import numpy as np
import pytest

import pf_monocular_pose_estimator_amd as pf

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
STREAMS = ["pf_c1_reference_rng", "pf_c1_philox", "pf_m12_heavy_philox"]
INT_KEYS = ("iters", "kept_iter", "accepted", "resampled", "most_likely_idx", "winner_idx", "n_corr", "flag_fail")


@pytest.mark.parametrize("name", STREAMS)
@pytest.mark.parametrize("bank", [False, True])
@pytest.mark.parametrize("fused", [2, 1, 0])  # flat one launch / tree one launch / two launches
def test_engine_reproduces_fixture(name, bank, fused):
    g = dict(np.load(os.path.join(GOLDEN, name + ".npz")))
    N = g["prior0"].shape[0]
    eng = pf.Engine(device=0, max_particles=N, max_blobs=int(g["B"].max()), state_dtype=pf.STATE_F64)
    eng.set_model(g["markers"], g["K"])
    prm = pf.default_params()
    prm.rng_mode = int(g["rng_mode"])
    eng.set_params(prm)
    eng.set_option(pf.OPT_RECORD_COUNTS, 1)
    eng.set_option(pf.OPT_FUSED, int(fused))
    eng.set_prior(g["prior0"])
    nf = len(g["seed"])
    if bank:
        eng.stage_blob_bank([g["blobs"][f][:int(g["B"][f])] for f in range(nf)])
    for f in range(nf):
        B = int(g["B"][f])
        kw = dict(B=B, bank_frame=f) if bank else dict(blobs=g["blobs"][f][:B])
        fr = eng.make_frame(g["cur"][f], g["pred"][f], g["predm"][f], dt=float(g["dt"][f]), seed=int(g["seed"][f]),
                            frame_idx=int(g["frame_idx"][f]), **kw)
        out = eng.step(fr).as_dict()
        for k in INT_KEYS:
            assert out[k] == g[k][f], (name, f, k, out[k], g[k][f])
        n = out["n_corr"]
        assert np.array_equal(out["pairs"], g["pairs"][f][:n])
        assert out["highest_prob"] == pytest.approx(float(g["highest_prob"][f]), abs=1e-9)
        np.testing.assert_allclose(eng.get_weights(), g["weights"][f], rtol=0, atol=1e-9)
        np.testing.assert_allclose(out["winner_pose"], g["winner_pose"][f], rtol=0, atol=1e-9)
        np.testing.assert_allclose(out["most_likely_pose"], g["most_likely_pose"][f], rtol=0, atol=1e-9)
        if out["resampled"]:
            assert np.array_equal(eng.get_counts(), g["counts"][f])
    np.testing.assert_allclose(eng.get_particles(1), g["final_prior"], rtol=0, atol=1e-9)
    eng.close()
