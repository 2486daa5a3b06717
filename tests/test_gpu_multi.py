"""Batched frames of independent streams (pfmpe_step_multi): several contexts' frames in one launch sequence.

The reference runs one particle filter per tracked object / camera stream (the per-object loop at
pf_mpe_lib/src/pose_estimator.cpp:89, per-object state PE:113-114, 726-727); the streams never interact.
Bar: every stream of a batch produces EXACTLY what its own pfmpe_step produces — every record field, the
weights, the propagated and the resampled sets bit for bit — over several frames, with streams of different
N, M, B, an occluded stream (all 80 re-draw iterations, so later iteration rounds run a subset of the batch),
a stream whose blobs are empty (re-initialisation branch) and blobs from a staged bank.  One fp64 stream is
also checked against the CPU oracle directly.
"""
import numpy as np
import pytest

import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn
from oracle import pforacle as orc

pytestmark = pytest.mark.gpu


def _engine(N, M, state, rng, fused=2):
    st = syn.make_stream(syn.StreamConfig("m", M=M, B=50, N=N), 1)
    eng = pf.Engine(device=0, max_particles=N, state_dtype=state)
    eng.set_option(pf.OPT_FUSED, fused)
    eng.set_model(st.markers, st.K)
    prm = pf.default_params()
    prm.rng_mode = rng
    eng.set_params(prm)
    eng.set_option(pf.OPT_RECORD_COUNTS, 1)
    return eng


# (N, M, B, heavy, how): how = "" normal, "occlude" one LED hidden, "empty" B = 0, "bank" staged blobs
STREAMS = [
    (1000, 5, 20, False, ""),
    (4099, 5, 50, False, "occlude"),
    (2048, 12, 200, True, ""),
    (777, 5, 50, False, "empty"),
    (100_000, 5, 50, False, "bank"),
    (300, 5, 3, False, ""),  # B < M: the sorted score path
]


def _streams(n_frames):
    out = []
    for s, (N, M, B, heavy, how) in enumerate(STREAMS):
        cfg = syn.StreamConfig(f"s{s}", M=M, B=B, N=N, heavy=heavy, seed=s)
        st = syn.make_stream(cfg, n_frames, t0=0.5 + 0.1 * s)
        frames = []
        for f, fr in enumerate(st.frames):
            blobs = fr.blobs
            if how == "occlude":  # LED 0's blob goes missing: max weight < M*min(5, B), all 80 iterations
                uv0 = syn.project(st.K, fr.truth, st.markers)[0]
                blobs = np.delete(blobs, int(np.argmin(np.sum((blobs - uv0) ** 2, axis=1))), axis=0)
            elif how == "empty":
                blobs = np.zeros((0, 2))
            frames.append((fr, blobs))
        out.append((st, frames, how))
    return out


def _frame(eng, fr, blobs, how, seed, f):
    if how == "bank":
        return eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, B=len(blobs), dt=fr.dt, seed=seed,
                              frame_idx=f, bank_frame=f)
    return eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=blobs, dt=fr.dt, seed=seed,
                          frame_idx=f)


def _snapshot(eng, out):
    d = out.as_dict()
    snap = {"rec": d, "w": eng.get_weights(), "p0": eng.get_particles(0)}
    if d["resampled"]:
        snap["p1"] = eng.get_particles(1)
        snap["counts"] = eng.get_counts()
    return snap


def _same(a, b, tag):
    for k, v in a["rec"].items():
        if isinstance(v, np.ndarray):
            assert np.array_equal(v, b["rec"][k]), (tag, k)
        else:
            assert v == b["rec"][k], (tag, k, v, b["rec"][k])
    for k in ("w", "p0", "p1", "counts"):
        assert (k in a) == (k in b), (tag, k)
        if k in a:
            assert np.array_equal(a[k], b[k]), (tag, k)


@pytest.mark.parametrize("state,rng", [(pf.STATE_F64, pf.RNG_REFERENCE), (pf.STATE_F32, pf.RNG_PHILOX),
                                       (pf.STATE_F16, pf.RNG_PHILOX)])
def test_multi_equals_single_streams(state, rng):
    n_frames = 3
    streams = _streams(n_frames)
    batch, solo = [], []
    for (st, frames, how), (N, M, *_rest) in zip(streams, STREAMS):
        pair = []
        for fused in (2, 0):  # the solo engine takes its default shape; the batch always runs two launches
            eng = _engine(N, M, state, rng, fused=fused)
            eng.set_prior(st.prior(N))
            if how == "bank":
                eng.stage_blob_bank([b for _, b in frames])
            pair.append(eng)
        batch.append(pair[1])
        solo.append(pair[0])
    try:
        for f in range(n_frames):
            seeds = [1000 + 17 * s + f for s in range(len(streams))]
            ins = [_frame(batch[s], streams[s][1][f][0], streams[s][1][f][1], streams[s][2], seeds[s], f)
                   for s in range(len(streams))]
            outs = pf.Engine.step_multi(batch, ins)
            for s, (st, frames, how) in enumerate(streams):
                fr, blobs = frames[f]
                ref_out = solo[s].step(_frame(solo[s], fr, blobs, how, seeds[s], f))
                _same(_snapshot(batch[s], outs[s]), _snapshot(solo[s], ref_out), (state, s, f))
                if how == "occlude":
                    assert outs[s].iters == 80
                if how == "empty":
                    assert outs[s].flag_fail == pf.FLAG_REINIT
            assert batch[0].info(pf.INFO_LAST_SHAPE) == pf.SHAPE_TWO_LAUNCH
    finally:
        for e in batch + solo:
            e.close()


def test_multi_fp64_stream_matches_oracle():
    """A batched fp64 stream against the CPU restatement (PE:475-733), beside two other streams."""
    cfg = syn.StreamConfig("m", M=5, B=20, N=1000)
    st = syn.make_stream(cfg, 1)
    fr = st.frames[0]
    prior = st.prior()
    engs = []
    try:
        for s in range(3):
            e = _engine(1000 + 500 * s, 5, pf.STATE_F64, pf.RNG_REFERENCE)
            e.set_prior(prior if s == 0 else st.prior(1000 + 500 * s))
            engs.append(e)
        ins = [e.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=fr.blobs, dt=fr.dt, seed=99 + s,
                            frame_idx=0) for s, e in enumerate(engs)]
        out = pf.Engine.step_multi(engs, ins)[0].as_dict()
        prm = pf.default_params()
        ref, arr = orc.pf_step(st.markers, st.K, orc.make_params(rng_mode=pf.RNG_REFERENCE), prior, fr.current_pose,
                               fr.predicted_pose, fr.prediction, fr.blobs, dt=fr.dt, seed=99, frame_idx=0)
        for k in ("iters", "kept_iter", "accepted", "most_likely_idx", "winner_idx", "n_corr", "flag_fail"):
            assert out[k] == ref[k], k
        assert np.array_equal(out["pairs"], ref["pairs"])
        np.testing.assert_allclose(engs[0].get_weights(), arr["weights"], rtol=0, atol=1e-9)
        np.testing.assert_allclose(engs[0].get_particles(1), arr["resampled"], rtol=0, atol=1e-9)
        assert np.array_equal(engs[0].get_counts(), arr["counts"])
        assert prm.max_iter == 80
    finally:
        for e in engs:
            e.close()


def test_multi_rejects_mixed_contexts():
    a = _engine(500, 5, pf.STATE_F32, pf.RNG_PHILOX)
    b = _engine(500, 5, pf.STATE_F64, pf.RNG_PHILOX)
    st = syn.make_stream(syn.StreamConfig("m", M=5, B=20, N=500), 1)
    fr = st.frames[0]
    try:
        for e in (a, b):
            e.set_prior(st.prior(500))
        ins = [e.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=fr.blobs, dt=fr.dt, seed=1,
                            frame_idx=0) for e in (a, b)]
        with pytest.raises(pf.PFError):
            pf.Engine.step_multi([a, b], ins)
        with pytest.raises(pf.PFError):
            pf.Engine.step_multi([a, a], [ins[0], ins[0]])
        out = pf.Engine.step_multi([a], [ins[0]])  # a one-stream batch is fine
        assert out[0].accepted in (0, 1)
    finally:
        a.close()
        b.close()
