"""k_weigh_pk / k_weigh_pk12 (two particles per lane, packed fp32; csrc/pf_weigh_pk.hpp) against k_weigh_stream.

The packed pass must give the same bits as the one-particle-per-lane streaming pass it replaces (every fp32
operation is the same operation in each lane of a v_pk_* instruction): the frame records, the weights, the
propagated and the resampled sets and the resample counts are compared for equality, frame by frame, over the
cases the pass has code for:
  * fp16 (C4's storage) and fp32 (C5's) state, N not a multiple of 128 (a partial last task and a partial wave);
  * a steady frame (iteration 0: no predictionMatrix), an 80-iteration frame (one LED hidden: the
    predictionMatrix composition from iteration 1, the noise growth from iteration 10, the kept slot moving);
  * it_since_init = 1 (no prediction, fac = 1 draw ranges);
  * downgraded markers and self-occlusion (two markers 1 mm apart, one blob for both): the penalty branch;
  * the kept propagated set on (one-stream default) and off (regeneration in k_resample);
  * 12 markers (k_weigh_pk12, C3's pass): heavy clutter (200 blobs with near outliers, longer grid lists), the
    80-iteration frame, penalties with two marker pairs on shared blobs and downgraded markers.
The pass is also checked to be the one that ran (PFMPE_INFO_LAST_WEIGH_PASS).
"""
import numpy as np
import pytest

import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn
from test_gpu_parity import make_engine

pytestmark = pytest.mark.gpu


def _run(st, N, state, diag, frames, markers=None, downgrade=None, keep=1):
    eng = make_engine(N, markers if markers is not None else st.markers, st.K, state, pf.RNG_PHILOX, fused=0,
                      downgrade=downgrade)
    eng.set_option(pf.OPT_DIAG, diag)
    eng.set_option(pf.OPT_KEEP_PROPAGATED, keep)
    eng.set_prior(st.prior(fast=True))
    snaps, passes = [], []
    try:
        for f, (fr, blobs, kw) in enumerate(frames):
            out = eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=blobs, dt=fr.dt,
                                          seed=404 + f, frame_idx=f, **kw)).as_dict()
            passes.append(eng.info(pf.INFO_LAST_WEIGH_PASS))
            snap = {"out": out, "w": eng.get_weights(), "p0": eng.get_particles(0)}
            if out["resampled"]:
                snap["p1"] = eng.get_particles(1)
                snap["counts"] = eng.get_counts()
            snaps.append(snap)
    finally:
        eng.close()
    return snaps, passes


def _assert_same(a_runs, b_runs):
    for f, (a, b) in enumerate(zip(a_runs, b_runs)):
        for k, v in a["out"].items():
            assert np.array_equal(np.asarray(v), np.asarray(b["out"][k])), (f, k, v, b["out"][k])
        for k in ("w", "p0", "p1", "counts"):
            assert (k in a) == (k in b), (f, k)
            if k in a:
                assert np.array_equal(a[k], b[k]), (f, k, np.flatnonzero(
                    np.any(np.asarray(a[k]).reshape(len(a[k]), -1) != np.asarray(b[k]).reshape(len(b[k]), -1),
                           axis=1))[:10])


def _frames(st, occlude_second=True):
    out = []
    for f, fr in enumerate(st.frames):
        blobs, kw = fr.blobs, {}
        if f == 1 and occlude_second:  # LED 0's blob hidden: the exit rule never fires, 80 iterations
            uv0 = syn.project(st.K, fr.truth, st.markers)[0]
            blobs = np.delete(blobs, int(np.argmin(np.sum((blobs - uv0) ** 2, axis=1))), axis=0)
        if f == 2:
            kw = {"it_since_init": 1}
        out.append((fr, blobs, kw))
    return out


@pytest.mark.parametrize("state", [pf.STATE_F16, pf.STATE_F32])
@pytest.mark.parametrize("keep", [1, 0])
def test_pk_pass_is_bit_identical(state, keep):
    N = 1_200_017
    st = syn.make_stream(syn.StreamConfig("t", M=5, B=50, N=N), 3)
    frames = _frames(st)
    a, pa = _run(st, N, state, pf.DIAG_FORCE_STREAM, frames, keep=keep)
    b, pb = _run(st, N, state, pf.DIAG_FORCE_STREAM | pf.DIAG_NO_PK, frames, keep=keep)
    assert pa == [pf.WEIGH_PK] * 3 and pb == [pf.WEIGH_STREAM] * 3, (pa, pb)
    assert a[1]["out"]["iters"] == 80
    _assert_same(a, b)


@pytest.mark.parametrize("state", [pf.STATE_F16, pf.STATE_F32])
def test_pk_pass_penalties(state):
    """Downgraded markers and self-occlusion: marker 4 sits 1 mm beside marker 3 and its own blob is removed, so
    both take marker 3's blob (the 3 * s penalty); markers 1 and 3 are downgraded (the -2 penalty)."""
    N = 300_000
    st = syn.make_stream(syn.StreamConfig("t", M=5, B=50, N=N), 2)
    markers = np.array(st.markers, dtype=np.float64).copy()
    markers[4] = markers[3] + np.array([0.001, 0.0, 0.0])
    frames = []
    for fr in st.frames:
        uv = syn.project(st.K, fr.truth, markers)
        blobs = fr.blobs.copy()
        # the blob nearest marker 4's projection becomes marker 3's (one blob for both)
        i4 = int(np.argmin(np.sum((blobs - uv[4]) ** 2, axis=1)))
        blobs[i4] = uv[3]
        frames.append((fr, blobs, {}))
    dg = np.array([0, 1, 0, 1, 0], dtype=np.uint8)
    a, pa = _run(st, N, state, pf.DIAG_FORCE_STREAM, frames, markers=markers, downgrade=dg)
    b, pb = _run(st, N, state, pf.DIAG_FORCE_STREAM | pf.DIAG_NO_PK, frames, markers=markers, downgrade=dg)
    assert pa == [pf.WEIGH_PK] * 2 and pb == [pf.WEIGH_STREAM] * 2, (pa, pb)
    # the penalties actually occur: some weights are not M + q^2 sums (below the 4-marker floor or negative)
    assert any((s["w"] < 20).sum() > 0 for s in a)
    _assert_same(a, b)


@pytest.mark.parametrize("state", [pf.STATE_F16, pf.STATE_F32])
def test_pk12_pass_is_bit_identical(state):
    """The 12-marker packed pass against k_weigh_stream<float, 1, 12>: C3's clutter (200 blobs, near and far
    outliers), N not a multiple of 128, the steady / 80-iteration (forced: the clutter can satisfy the exit rule with
    11 LEDs) / it_since_init = 1 frames."""
    N = 1_000_033
    st = syn.make_stream(syn.StreamConfig("t", M=12, B=200, N=N, heavy=True), 3)
    frames = _frames(st)
    frames[1] = (frames[1][0], frames[1][1], {"force_iters": 80})
    a, pa = _run(st, N, state, pf.DIAG_FORCE_STREAM, frames)
    b, pb = _run(st, N, state, pf.DIAG_FORCE_STREAM | pf.DIAG_NO_PK, frames)
    assert pa == [pf.WEIGH_PK] * 3 and pb == [pf.WEIGH_STREAM] * 3, (pa, pb)
    assert a[1]["out"]["iters"] == 80
    _assert_same(a, b)


@pytest.mark.parametrize("state", [pf.STATE_F16, pf.STATE_F32])
def test_pk12_pass_penalties(state):
    """12 markers with self-occlusion in two places (marker 11 beside marker 10, marker 5 beside marker 2, each
    pair sharing one blob: dups = 2, the 3 * s * (s + 1) / 2 penalty) and downgraded markers 1, 7 and 10."""
    N = 300_001
    st = syn.make_stream(syn.StreamConfig("t", M=12, B=200, N=N, heavy=True), 2)
    markers = np.array(st.markers, dtype=np.float64).copy()
    markers[11] = markers[10] + np.array([0.001, 0.0, 0.0])
    markers[5] = markers[2] + np.array([0.0, 0.001, 0.0])
    frames = []
    for fr in st.frames:
        uv = syn.project(st.K, fr.truth, markers)
        blobs = fr.blobs.copy()
        for a_, b_ in ((11, 10), (5, 2)):
            i = int(np.argmin(np.sum((blobs - uv[a_]) ** 2, axis=1)))
            blobs[i] = uv[b_]
        frames.append((fr, blobs, {}))
    dg = np.zeros(12, dtype=np.uint8)
    dg[[1, 7, 10]] = 1
    a, pa = _run(st, N, state, pf.DIAG_FORCE_STREAM, frames, markers=markers, downgrade=dg)
    b, pb = _run(st, N, state, pf.DIAG_FORCE_STREAM | pf.DIAG_NO_PK, frames, markers=markers, downgrade=dg)
    assert pa == [pf.WEIGH_PK] * 2 and pb == [pf.WEIGH_STREAM] * 2, (pa, pb)
    _assert_same(a, b)


def test_pk_pass_default_at_c4_c5():
    """The default two-launch weighing pass at C4 / C5 (fp16 / fp32, 5 markers, 50 blobs) is k_weigh_pk, and at C3
    (fp32, 12 markers, 200 blobs) k_weigh_pk12 (both report PFMPE_WEIGH_PK)."""
    for name, state in (("C5", pf.STATE_F32), ("C4", pf.STATE_F16), ("C3", pf.STATE_F32)):
        cfg = syn.CONFIGS[name]
        st = syn.make_stream(cfg, 1)
        fr = st.frames[0]
        eng = make_engine(cfg.N, st.markers, st.K, state, pf.RNG_PHILOX)
        try:
            eng.set_prior(st.prior(fast=True))
            eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=fr.blobs, dt=fr.dt,
                                    seed=9, frame_idx=0))
            assert eng.info(pf.INFO_LAST_SHAPE) == pf.SHAPE_TWO_LAUNCH
            assert eng.info(pf.INFO_LAST_WEIGH_PASS) == pf.WEIGH_PK, name
        finally:
            eng.close()


@pytest.mark.parametrize("M,B,heavy", [(5, 50, False), (12, 200, True)])
@pytest.mark.parametrize("N", [3, 129, 4_099])
def test_pk_passes_small_n(M, B, heavy, N):
    """Tiny particle counts through the packed passes (forced streaming): a task holding particles 0 and 1 (the
    current / predicted poses, PE:547-551) with almost every lane past N, a second task with none, one partial wave
    (129), and a partial last block (4,099); steady / 80-iteration / it_since_init = 1 frames, fp32 state."""
    st = syn.make_stream(syn.StreamConfig("t", M=M, B=B, N=N, heavy=heavy), 3)
    frames = _frames(st)
    frames[1] = (frames[1][0], frames[1][1], {"force_iters": 80})
    a, pa = _run(st, N, pf.STATE_F32, pf.DIAG_FORCE_STREAM, frames)
    b, pb = _run(st, N, pf.STATE_F32, pf.DIAG_FORCE_STREAM | pf.DIAG_NO_PK, frames)
    assert pa == [pf.WEIGH_PK] * 3 and pb == [pf.WEIGH_STREAM] * 3, (pa, pb)
    _assert_same(a, b)
