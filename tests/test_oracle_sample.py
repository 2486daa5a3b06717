"""orc_pf_sample (the oracle's per-particle restatement used by tests/test_gpu_packed_oracle.py) is orc_pf_step's own
motion model and likelihood: for every particle of whole frames (a steady frame, an 80-iteration frame with the
noise growth and the predictionMatrix composition, it_since_init = 1) the sampled propagated pose and weight equal
the full step's kept set and weights bit for bit."""
import numpy as np
import pytest

from oracle import pforacle as orc
from pf_monocular_pose_estimator_amd import synthetic as syn


@pytest.mark.parametrize("case", ["steady", "occluded", "it1"])
def test_pf_sample_equals_pf_step(case):
    st = syn.make_stream(syn.StreamConfig("t", M=5, B=20, N=600), 1)
    fr = st.frames[0]
    prior = st.prior()
    blobs, it = fr.blobs, 2
    cur, pred = np.array(fr.current_pose), np.array(fr.predicted_pose)
    if case == "occluded":  # LED 0 hidden and particles 0 / 1 5 cm off: 80 iterations, a late one kept
        uv0 = syn.project(st.K, fr.truth, st.markers)[0]
        blobs = np.delete(blobs, int(np.argmin(np.sum((blobs - uv0) ** 2, axis=1))), axis=0)
        cur[3] += 0.05
        pred[3] += 0.05
    if case == "it1":
        it = 1
    prm = orc.make_params(rng_mode=orc.RNG_PHILOX)
    seed = 1
    out, arr = orc.pf_step(st.markers, st.K, prm, prior, cur, pred, fr.prediction, blobs,
                           it_since_init=it, dt=fr.dt, seed=seed, frame_idx=5)
    if case == "occluded":
        assert out["iters"] == 80 and out["kept_iter"] > 10 and out["kept_iter"] % 10 != 0
    idx = np.arange(prior.shape[0])
    p, w = orc.pf_sample(st.markers, st.K, prm, idx, prior, cur, pred, fr.prediction, blobs,
                         out["kept_iter"], it_since_init=it, dt=fr.dt, seed=seed, frame_idx=5)
    assert np.array_equal(p, arr["propagated"])
    assert np.array_equal(w, arr["weights"])


def test_pf_sample_refuses_reference_stream():
    st = syn.make_stream(syn.StreamConfig("t", M=5, B=20, N=10), 1)
    fr = st.frames[0]
    with pytest.raises(RuntimeError):
        orc.pf_sample(st.markers, st.K, orc.make_params(rng_mode=orc.RNG_REFERENCE), [2], st.prior()[2:3],
                      fr.current_pose, fr.predicted_pose, fr.prediction, fr.blobs, 0)
