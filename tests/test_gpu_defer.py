"""Deferred resampling (PFMPE_OPT_DEFER_RESAMPLE, default on) against the materialised new prior.

A two-launch frame with the kept propagated set writes the new prior's owner indices instead of the particles
(k_resample), and the kept buffer becomes the prior's storage; every later reader of the prior goes through the
owner indices: the weighing passes (one-block, streaming, packed), both one-launch shapes (k_frame, k_frame2),
the regeneration in k_resample, the ROI, the read-backs, and batches.  Everything observable must be the same
bits as with deferral off, frame after frame, including frames whose shape differs from the previous frame's
(a one-launch frame reading a deferred prior, a deferred frame reading a one-launch frame's prior)."""
import numpy as np
import pytest

import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn
from test_gpu_parity import make_engine

pytestmark = pytest.mark.gpu

D = np.array([0.01, -0.02, 0.001, 0.0005, 0.0])  # a distortion vector for the ROI


def _frames(st):
    out = []
    for f, fr in enumerate(st.frames):
        blobs, kw = fr.blobs, {}
        if f == 1:  # LED 0 hidden: 80 iterations, the kept slot may be either
            uv0 = syn.project(st.K, fr.truth, st.markers)[0]
            blobs = np.delete(blobs, int(np.argmin(np.sum((blobs - uv0) ** 2, axis=1))), axis=0)
        if f == 3:
            kw = {"it_since_init": 1}
        out.append((fr, blobs, kw))
    return out


def _snap(eng, out, fr):
    s = {"out": out, "w": eng.get_weights(), "p0": eng.get_particles(0), "p1": eng.get_particles(1),
         "roi": eng.predict_roi(fr.prediction, fr.predicted_pose, D, syn.IMAGE_W, syn.IMAGE_H, 5)}
    if out["resampled"]:
        s["counts"] = eng.get_counts()
    return s


def _same(a, b):
    for f, (x, y) in enumerate(zip(a, b)):
        for k, v in x["out"].items():
            assert np.array_equal(np.asarray(v), np.asarray(y["out"][k])), (f, k)
        assert x.keys() == y.keys(), f
        for k in x:
            if k == "out":
                continue
            if k == "roi":
                for kk in x[k]:
                    assert np.array_equal(np.asarray(x[k][kk]), np.asarray(y[k][kk])), (f, k, kk)
            else:
                assert np.array_equal(x[k], y[k]), (f, k)


@pytest.mark.parametrize("state", [pf.STATE_F32, pf.STATE_F16, pf.STATE_F64])
def test_deferred_equals_materialised_across_shapes(state):
    """N = 120,017 fits a one-launch frame (470 blocks), so the shape can be switched frame by frame:
    two-launch (deferred), k_frame2 (reads it), two-launch (deferred), k_frame (reads it), two-launch (deferred),
    two-launch regenerating (keep off: k_resample regenerates from the deferred prior)."""
    N = 120_017
    st = syn.make_stream(syn.StreamConfig("t", M=5, B=50, N=N), 6)
    frames = _frames(st)
    shapes = [(0, 1), (2, 1), (0, 1), (1, 1), (0, 1), (0, 0)]  # (PFMPE_OPT_FUSED, keep propagated)
    runs, seen = [], []
    for defer in (1, 0):
        eng = make_engine(N, st.markers, st.K, state, pf.RNG_PHILOX)
        eng.set_option(pf.OPT_DEFER_RESAMPLE, defer)
        eng.set_prior(st.prior(fast=True))
        snaps, sh = [], []
        try:
            for f, ((fr, blobs, kw), (fused, keep)) in enumerate(zip(frames, shapes)):
                eng.set_option(pf.OPT_FUSED, fused)
                eng.set_option(pf.OPT_KEEP_PROPAGATED, keep)
                out = eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=blobs,
                                              dt=fr.dt, seed=900 + f, frame_idx=f, **kw)).as_dict()
                sh.append(eng.info(pf.INFO_LAST_SHAPE))
                snaps.append(_snap(eng, out, fr))
        finally:
            eng.close()
        runs.append(snaps)
        seen.append(sh)
    assert seen[0] == seen[1], seen
    if state != pf.STATE_F64:  # fp64 one-launch shapes may fall back to two launches (register cap): not pinned
        assert seen[0][1] == pf.SHAPE_FRAME2 and seen[0][0] == pf.SHAPE_TWO_LAUNCH, seen[0]
    assert frames[1][0] is not None and runs[0][1]["out"]["iters"] == 80
    _same(runs[0], runs[1])


@pytest.mark.parametrize("state", [pf.STATE_F32, pf.STATE_F16])
def test_deferred_batches_equal_materialised(state):
    """Three streams as one batch per frame (pfmpe_step_multi), deferral on vs off, 4 frames; then one
    pfmpe_step of each stream (its own two-launch frame reading the batch's deferred prior)."""
    sizes = [200_000, 77_777, 300_001]
    streams = [syn.make_stream(syn.StreamConfig("t", M=5, B=50, N=N, seed=11 + i), 5) for i, N in enumerate(sizes)]
    results = []
    for defer in (1, 0):
        engs = []
        try:
            for st, N in zip(streams, sizes):
                e = make_engine(N, st.markers, st.K, state, pf.RNG_PHILOX, fused=0)
                e.set_option(pf.OPT_DEFER_RESAMPLE, defer)
                e.set_prior(st.prior(fast=True))
                engs.append(e)
            snaps = []
            for f in range(4):
                ins = [e.make_frame(st.frames[f].current_pose, st.frames[f].predicted_pose, st.frames[f].prediction,
                                    blobs=st.frames[f].blobs, dt=st.frames[f].dt, seed=500 + 7 * i + f, frame_idx=f)
                       for i, (e, st) in enumerate(zip(engs, streams))]
                outs = pf.Engine.step_multi(engs, ins)
                snaps.append([_snap(e, o.as_dict(), st.frames[f]) for e, o, st in zip(engs, outs, streams)])
            for i, (e, st) in enumerate(zip(engs, streams)):
                fr = st.frames[4]
                o = e.step(e.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=fr.blobs,
                                        dt=fr.dt, seed=600 + i, frame_idx=4)).as_dict()
                snaps.append([_snap(e, o, fr)])
            results.append(snaps)
        finally:
            for e in engs:
                e.close()
    for a, b in zip(*results):
        _same(a, b)
