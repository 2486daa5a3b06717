"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle on identical inputs.

Bars (SURVEY.md §7 "minimum slice", north_star):
  * fp64 state (PFMPE_STATE_F64), either RNG stream: every discrete output identical to the oracle
    (iterations, kept iteration, accept, most-likely index, resample counts, winner, correspondences);
    weights within 1e-9 absolute, poses within 1e-9 (ulp-level differences only: sin/cos libraries).
  * fp32 state (the throughput path): weights within 2e-3 absolute for >= 99.5 % of particles (a marker
    sitting within ~1e-5 px of the tol_PF gate may flip), accept decision identical, counts sum to N,
    winner/pose tolerance 1e-4 m / 1e-3 rad against the oracle's winner pose where the winners agree.
"""
import numpy as np
import pytest

import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn
from oracle import pforacle as orc

pytestmark = pytest.mark.gpu

RNG = {"ref": pf.RNG_REFERENCE, "philox": pf.RNG_PHILOX}
STATE = {"f64": pf.STATE_F64, "f32": pf.STATE_F32, "f16": pf.STATE_F16}


def make_engine(N, markers, K, state, rng, prune=True, downgrade=None, params=None, fused=2):
    eng = pf.Engine(device=0, max_particles=max(N, 1), state_dtype=state)
    eng.set_option(pf.OPT_FUSED, int(fused))  # 2 flat / 1 tree one-launch frame, 0 two launches
    eng.set_model(markers, K, downgrade)
    prm = params or pf.default_params()
    prm.rng_mode = rng
    eng.set_params(prm)
    eng.set_option(pf.OPT_RECORD_COUNTS, 1)
    eng.set_option(pf.OPT_PRUNE, 1 if prune else 0)
    return eng


def orc_params_from(prm):
    return orc.OrcParams(prm.tol, prm.tol_pf, prm.ang_min, prm.ang_max, prm.trans_min, prm.trans_max, prm.growth,
                         prm.max_iter, prm.exit_cap, prm.accept_cap, prm.rng_mode)


def step_both(eng, prm, markers, K, prior, cur, pred, predm, blobs, seed, frame_idx, it=2, dt=0.02,
              force_iters=0, cam=None, downgrade=None):
    fr = eng.make_frame(cur, pred, predm, blobs=blobs, dt=dt, seed=seed, frame_idx=frame_idx, it_since_init=it,
                        force_iters=force_iters, cam_move_inv=cam)
    out = eng.step(fr).as_dict()
    gpu = {"weights": eng.get_weights(), "propagated": eng.get_particles(0)}
    if out["resampled"]:
        gpu["counts"] = eng.get_counts()
        gpu["resampled"] = eng.get_particles(1)
    ref, arr = orc.pf_step(markers, K, orc_params_from(prm), prior, cur, pred, predm, blobs, it_since_init=it, dt=dt,
                           seed=seed, frame_idx=frame_idx, force_iters=force_iters, cam_move_inv=cam,
                           downgrade=downgrade)
    return out, gpu, ref, arr


def assert_exact(out, gpu, ref, arr, N):
    for k in ("iters", "kept_iter", "accepted", "resampled", "most_likely_idx", "winner_idx", "n_corr", "flag_fail"):
        assert out[k] == ref[k], (k, out[k], ref[k])
    assert np.array_equal(out["pairs"], ref["pairs"])
    np.testing.assert_allclose(gpu["weights"], arr["weights"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(gpu["propagated"], arr["propagated"], rtol=0, atol=1e-9)
    assert out["highest_prob"] == pytest.approx(ref["highest_prob"], abs=1e-9)
    assert out["prob_sum"] == pytest.approx(ref["prob_sum"], rel=1e-12, abs=1e-9)
    np.testing.assert_allclose(out["winner_pose"], ref["winner_pose"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(out["most_likely_pose"], ref["most_likely_pose"], rtol=0, atol=1e-9)
    if out["resampled"]:
        assert np.array_equal(gpu["counts"], arr["counts"])
        assert int(gpu["counts"].sum()) <= N
        np.testing.assert_allclose(gpu["resampled"], arr["resampled"], rtol=0, atol=1e-9)


CASES = [  # (N, M, B, heavy)
    (1000, 5, 20, False),
    (4099, 5, 50, False),
    (2048, 12, 200, True),
]


@pytest.mark.parametrize("rng", ["ref", "philox"])
@pytest.mark.parametrize("N,M,B,heavy", CASES)
@pytest.mark.parametrize("prune", [True, False])
@pytest.mark.parametrize("fused", [2, 1, 0])  # flat one launch / tree one launch / two launches
def test_fp64_exact_trajectory(rng, N, M, B, heavy, prune, fused):
    cfg = syn.StreamConfig("t", M=M, B=B, N=N, heavy=heavy)
    n_frames = 10
    st = syn.make_stream(cfg, n_frames)
    prm = pf.default_params()
    prm.rng_mode = RNG[rng]
    eng = make_engine(N, st.markers, st.K, pf.STATE_F64, RNG[rng], prune=prune, fused=fused)
    prior = st.prior()
    eng.set_prior(prior)
    for fr in st.frames:
        out, gpu, ref, arr = step_both(eng, prm, st.markers, st.K, prior, fr.current_pose, fr.predicted_pose,
                                       fr.prediction, fr.blobs, seed=1000 + fr.index, frame_idx=fr.index)
        assert_exact(out, gpu, ref, arr, N)
        if out["resampled"]:
            prior = arr["resampled"]
    eng.close()


@pytest.mark.parametrize("rng", ["ref", "philox"])
@pytest.mark.parametrize("fused", [2, 1, 0])  # flat one launch / tree one launch / two launches
def test_fp64_exit_rule_runs_all_iterations(rng, fused):
    """One LED occluded -> max weight < M*min(5,B): the loop runs all 80 iterations with noise growth
    and keeps the earliest strictly-best iteration (PE:606-624)."""
    N = 96
    cfg = syn.StreamConfig("t", M=5, B=12, N=N)
    st = syn.make_stream(cfg, 1)
    fr = st.frames[0]
    true_px = syn.project(st.K, fr.truth, st.markers)
    outliers = np.random.default_rng(5).uniform([0, 0], [syn.IMAGE_W, syn.IMAGE_H], size=(7, 2))
    blobs = np.vstack([true_px[1:], outliers]).astype(np.float32).astype(np.float64)
    prm = pf.default_params()
    prm.rng_mode = RNG[rng]
    eng = make_engine(N, st.markers, st.K, pf.STATE_F64, RNG[rng], fused=fused)
    prior = st.prior()
    eng.set_prior(prior)
    out, gpu, ref, arr = step_both(eng, prm, st.markers, st.K, prior, fr.current_pose, fr.predicted_pose,
                                   fr.prediction, blobs, seed=77, frame_idx=3)
    assert ref["iters"] == 80
    assert_exact(out, gpu, ref, arr, N)
    eng.close()


@pytest.mark.parametrize("state", ["f64", "f32"])
@pytest.mark.parametrize("N", [1, 2, 3, 257])
@pytest.mark.parametrize("fused", [2, 1, 0])  # flat one launch / tree one launch / two launches
def test_small_particle_counts(state, N, fused):
    cfg = syn.StreamConfig("t", M=5, B=20, N=N)
    st = syn.make_stream(cfg, 2)
    prm = pf.default_params()
    prm.rng_mode = pf.RNG_REFERENCE
    eng = make_engine(N, st.markers, st.K, STATE[state], pf.RNG_REFERENCE, fused=fused)
    prior = st.prior()
    eng.set_prior(prior)
    for fr in st.frames:
        prior_used = eng.get_particles(1)
        out, gpu, ref, arr = step_both(eng, prm, st.markers, st.K, prior_used, fr.current_pose, fr.predicted_pose,
                                       fr.prediction, fr.blobs, seed=5 + fr.index, frame_idx=fr.index)
        if state == "f64":
            assert_exact(out, gpu, ref, arr, N)
        else:
            assert out["accepted"] == ref["accepted"]
            np.testing.assert_allclose(gpu["weights"], arr["weights"], atol=2e-3)
    eng.close()


@pytest.mark.parametrize("state", ["f64", "f32"])
@pytest.mark.parametrize("fused", [2, 1, 0])  # flat one launch / tree one launch / two launches
def test_no_blobs_reinitialises(state, fused):
    N = 300
    cfg = syn.StreamConfig("t", M=5, B=20, N=N)
    st = syn.make_stream(cfg, 1)
    fr = st.frames[0]
    eng = make_engine(N, st.markers, st.K, STATE[state], pf.RNG_PHILOX, fused=fused)
    prm = pf.default_params()
    eng.set_prior(st.prior())
    # B = 0: exit threshold M*min(5, B) = 0, so the reference stops after one iteration (PE:616)
    for blobs, iters in ((np.zeros((0, 2)), 1), (np.array([[5000.0, 5000.0], [6000.0, -40.0]]), 80)):
        out, gpu, ref, arr = step_both(eng, prm, st.markers, st.K, st.prior(), fr.current_pose, fr.predicted_pose,
                                       fr.prediction, blobs, seed=9, frame_idx=1)
        assert out["accepted"] == 0 and ref["accepted"] == 0
        assert out["flag_fail"] == pf.FLAG_REINIT
        assert out["iters"] == ref["iters"] == iters
        assert out["most_likely_idx"] == ref["most_likely_idx"]
        assert out["winner_idx"] == -1
    eng.close()


def test_fp64_fewer_blobs_than_markers_and_downgrade_and_cam_motion():
    N = 512
    cfg = syn.StreamConfig("t", M=5, B=3, N=N)
    st = syn.make_stream(cfg, 1)
    fr = st.frames[0]
    dg = np.array([1, 0, 0, 1, 0], np.uint8)
    cam = syn.to12(syn.se3_exp([0.002, -0.001, 0.003, 0.001, 0.0005, -0.002]))
    prm = pf.default_params()
    prm.rng_mode = pf.RNG_REFERENCE
    prm.accept_cap = 2
    eng = make_engine(N, st.markers, st.K, pf.STATE_F64, pf.RNG_REFERENCE, downgrade=dg, params=prm)
    prior = st.prior()
    eng.set_prior(prior)
    true_px = syn.project(st.K, fr.truth, st.markers)
    blobs = true_px[[0, 2, 4]].astype(np.float32).astype(np.float64)
    for it, force in ((2, 0), (1, 4), (2, 13)):
        out, gpu, ref, arr = step_both(eng, prm, st.markers, st.K, prior, fr.current_pose, fr.predicted_pose,
                                       fr.prediction, blobs, seed=31 + it, frame_idx=2, it=it, force_iters=force,
                                       cam=cam, downgrade=dg)
        assert_exact(out, gpu, ref, arr, N)
        if force:
            assert out["iters"] == force
        eng.set_prior(prior)
    eng.close()


def _collapsed_scenario():
    """Hand-built prior with both strongly positive and NEGATIVE weights (self-occlusion penalties),
    to exercise the running-max semantics of the cumulative search (SURVEY.md §7 hard part 3)."""
    K = syn.K_README
    s = 0.02
    markers = np.array([[-s, -s, 0.0], [s, -s, 0.0], [s, s, 0.0], [-s, s, 0.0]])
    T_true = np.eye(4)
    T_true[:3, 3] = [0.0, 0.0, 2.0]
    T_far = np.eye(4)
    T_far[:3, 3] = [0.0, 0.0, 40.0]
    px_true = syn.project(K, T_true, markers)
    centre = syn.project(K, T_far, markers).mean(axis=0) + np.array([3.4, 0.0])
    blobs = np.vstack([px_true, centre[None]])
    N = 64
    poses = []
    for n in range(N):
        poses.append(syn.to12(T_true if n % 3 else T_far))
    return K, markers, np.array(poses), blobs, syn.to12(T_true)


@pytest.mark.parametrize("rng", ["ref", "philox"])
def test_fp64_negative_weights_running_max(rng):
    K, markers, prior, blobs, truth = _collapsed_scenario()
    N = prior.shape[0]
    prm = pf.default_params()
    prm.rng_mode = RNG[rng]
    prm.ang_min = prm.ang_max = prm.trans_min = prm.trans_max = 0.0
    eng = make_engine(N, markers, K, pf.STATE_F64, RNG[rng], params=prm)
    eng.set_prior(prior)
    ident = np.eye(4)[:3].reshape(12)
    out, gpu, ref, arr = step_both(eng, prm, markers, K, prior, truth, truth, ident, blobs, seed=3, frame_idx=0, it=1)
    assert (arr["weights"] < 0).any() and (arr["weights"] > 15).any()
    assert out["accepted"] == 1
    assert_exact(out, gpu, ref, arr, N)
    eng.close()


def rotation_angle(R1, R2):
    """Angle between two rotations from the chord ||R1 - R2||_F = 2 sqrt(2) sin(theta / 2).  Unlike
    arccos((tr(R1^T R2) - 1) / 2) this stays accurate for small angles and slightly non-orthonormal
    (fp32-sourced) matrices, where the arccos form turns 1e-7 errors into ~1e-3 rad."""
    d = np.linalg.norm(np.asarray(R1) - np.asarray(R2))
    return float(2.0 * np.arcsin(min(1.0, d / (2.0 * np.sqrt(2.0)))))


@pytest.mark.parametrize("rng", ["ref", "philox"])
@pytest.mark.parametrize("N,M,B,heavy", [(20000, 5, 50, False), (8192, 12, 200, True)])
def test_fp32_tolerance(rng, N, M, B, heavy):
    """fp32 throughput path vs the fp64 oracle.  Weights may differ discretely where a marker sits within
    ~1e-5 px of the tol_PF gate; such a flip shifts every later stratum boundary, so counts are checked
    against the oracle's resampler run on the GPU's OWN weights (exact), and outputs are checked by the
    north_star criterion: refined (Gauss-Newton) poses within 1e-4 m / 1e-3 rad."""
    cfg = syn.StreamConfig("t", M=M, B=B, N=N, heavy=heavy)
    n_frames = 10
    st = syn.make_stream(cfg, n_frames)
    prm = pf.default_params()
    prm.rng_mode = RNG[rng]
    eng = make_engine(N, st.markers, st.K, pf.STATE_F32, RNG[rng])
    eng.set_prior(st.prior())
    compared = 0
    for fr in st.frames:
        prior_used = eng.get_particles(1)  # float-representable values: the oracle starts from the same set
        seed = 50 + fr.index
        out, gpu, ref, arr = step_both(eng, prm, st.markers, st.K, prior_used, fr.current_pose, fr.predicted_pose,
                                       fr.prediction, fr.blobs, seed=seed, frame_idx=fr.index)
        assert out["accepted"] == ref["accepted"]
        assert out["iters"] == ref["iters"]
        dw = np.abs(gpu["weights"] - arr["weights"])
        assert np.sum(dw > 2e-3) <= max(3, N // 1000), np.sort(dw)[-10:]
        dp = np.abs(gpu["propagated"] - arr["propagated"])
        assert dp[:, [0, 1, 2, 4, 5, 6, 8, 9, 10]].max() < 1e-5 and dp[:, [3, 7, 11]].max() < 1e-5
        if out["resampled"]:
            c = gpu["counts"].astype(np.int64)
            c_ref, _ = orc.stratified_resample(gpu["weights"], RNG[rng], seed, fr.index, out["iters"])
            assert np.sum(c != c_ref) <= 2, np.where(c != c_ref)[0][:10]
            w = out["winner_idx"]
            assert c[w] == c.max() and np.argmax(c) == w
            np.testing.assert_allclose(out["winner_pose"], gpu["propagated"][w], atol=1e-6)
            proj = np.array([orc.project(st.K, gpu["propagated"][w], X) for X in st.markers])
            _, pairs = orc.likelihood(proj, fr.blobs, prm.tol, prm.tol_pf)
            assert np.array_equal(out["pairs"], pairs)
            if np.array_equal(out["pairs"], ref["pairs"]):
                pg, _, _ = orc.optimise_pose(st.markers, st.K, fr.blobs, out["pairs"], out["winner_pose"])
                pr, _, _ = orc.optimise_pose(st.markers, st.K, fr.blobs, ref["pairs"], ref["winner_pose"])
                assert np.abs(pg[[3, 7, 11]] - pr[[3, 7, 11]]).max() < 1e-4
                assert rotation_angle(syn.to44(pg)[:3, :3], syn.to44(pr)[:3, :3]) < 1e-3
                compared += 1
    # the pose criterion must actually have been applied (not vacuously skipped on differing winners)
    assert compared >= n_frames - 1, compared
    eng.close()


@pytest.mark.parametrize("N", [1_000_000])
def test_fp32_large_n_properties(N):
    """BASELINE-size property checks (the O(N^2) oracle cannot run at 1M): counts sum to N, every new
    prior particle is a copy of a propagated particle, weights of a random subset match the oracle
    likelihood evaluated in fp64 on the GPU's own propagated poses."""
    cfg = syn.StreamConfig("t", M=5, B=50, N=N)
    st = syn.make_stream(cfg, 1)
    fr = st.frames[0]
    prm = pf.default_params()
    eng = make_engine(N, st.markers, st.K, pf.STATE_F32, pf.RNG_PHILOX)
    eng.set_prior(st.prior())
    out = eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=fr.blobs, dt=fr.dt,
                                  seed=4, frame_idx=0))
    assert out.accepted == 1
    w = eng.get_weights()
    prop = eng.get_particles(0)
    counts = eng.get_counts().astype(np.int64)
    post = eng.get_particles(1)
    assert counts.sum() == N  # every target finds a particle in practice (normalised total == 1)
    owner = np.repeat(np.arange(N), counts)
    np.testing.assert_array_equal(post, prop[owner])
    rng = np.random.default_rng(0)
    sub = rng.choice(N, 1500, replace=False)
    bad = 0
    for n in sub:
        proj = np.array([orc.project(st.K, prop[n], X) for X in st.markers])
        P, _ = orc.likelihood(proj, fr.blobs, prm.tol, prm.tol_pf)
        bad += abs(P - w[n]) > 2e-3
    assert bad <= 3
    assert out.winner_idx == int(np.argmax(counts))
    eng.close()


def test_blob_bank_matches_host_blobs():
    N = 5000
    cfg = syn.StreamConfig("t", M=5, B=50, N=N)
    st = syn.make_stream(cfg, 3)
    a = make_engine(N, st.markers, st.K, pf.STATE_F32, pf.RNG_PHILOX)
    b = make_engine(N, st.markers, st.K, pf.STATE_F32, pf.RNG_PHILOX)
    a.set_prior(st.prior())
    b.set_prior(st.prior())
    b.stage_blob_bank([f.blobs for f in st.frames])
    for fr in st.frames:
        oa = a.step(a.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=fr.blobs, dt=fr.dt,
                                 seed=8, frame_idx=fr.index)).as_dict()
        ob = b.step(b.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, B=len(fr.blobs),
                                 bank_frame=fr.index, dt=fr.dt, seed=8, frame_idx=fr.index)).as_dict()
        for k in ("iters", "winner_idx", "accepted", "highest_prob", "prob_sum"):
            assert oa[k] == ob[k]
        np.testing.assert_array_equal(a.get_particles(1), b.get_particles(1))
    a.close()
    b.close()


def test_api_errors_on_gpu():
    eng = pf.Engine(device=0, max_particles=100, state_dtype=pf.STATE_F32)
    with pytest.raises(pf.PFError):
        eng.step(eng.make_frame(np.eye(4)[:3], np.eye(4)[:3], np.eye(4)[:3], blobs=np.zeros((1, 2))))
    eng.set_model(syn.MARKERS_5, syn.K_README)
    with pytest.raises(pf.PFError):
        eng.set_prior(np.zeros((101, 12)))
    with pytest.raises(pf.PFError):
        eng.set_model(np.zeros((17, 3)), syn.K_README)
    eng.close()


def test_frame_record_integrity_long_run():
    """50 consecutive frames: every published record is self-consistent (its pairs are the oracle
    likelihood pairs of its own winner pose, flags agree) — guards the host-mapped record hand-off."""
    N = 3000
    cfg = syn.StreamConfig("t", M=5, B=50, N=N)
    st = syn.make_stream(cfg, 50)
    eng = make_engine(N, st.markers, st.K, pf.STATE_F64, pf.RNG_PHILOX)
    prm = pf.default_params()
    eng.set_prior(st.prior())
    for fr in st.frames:
        out = eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=fr.blobs, dt=fr.dt,
                                      seed=77 + fr.index, frame_idx=fr.index)).as_dict()
        assert out["accepted"] == 1 and out["flag_fail"] == pf.FLAG_ACCEPTED and out["resampled"] == 1
        proj = np.array([orc.project(st.K, out["winner_pose"], X) for X in st.markers])
        _, pairs = orc.likelihood(proj, fr.blobs, prm.tol, prm.tol_pf)
        assert np.array_equal(out["pairs"], pairs), fr.index
        assert out["n_corr"] == len(pairs)
    eng.close()


@pytest.mark.gpu
def test_step_batch_matches_step_loop():
    """pfmpe_step_batch is the same frames through the same engine, looped in C."""
    N = 5000
    cfg = syn.StreamConfig("t", M=5, B=50, N=N)
    st = syn.make_stream(cfg, 12)
    res = []
    for batch in (False, True):
        eng = make_engine(N, st.markers, st.K, pf.STATE_F64, pf.RNG_PHILOX)
        eng.set_prior(st.prior())
        eng.stage_blob_bank([f.blobs for f in st.frames])
        frames = [eng.make_frame(f.current_pose, f.predicted_pose, f.prediction, B=len(f.blobs), bank_frame=f.index,
                                 dt=f.dt, seed=5 + f.index, frame_idx=f.index) for f in st.frames]
        outs = eng.step_batch(frames) if batch else [eng.step(f) for f in frames]
        res.append(([o.as_dict() if hasattr(o, "as_dict") else o for o in outs], eng.get_particles(1)))
        eng.close()
    (a, pa), (b, pb) = res
    assert len(a) == len(b) == 12
    for x, y in zip(a, b):
        for k in ("iters", "kept_iter", "winner_idx", "accepted", "n_corr"):
            assert x[k] == y[k]
        assert np.array_equal(x["winner_pose"], y["winner_pose"])
    assert np.array_equal(pa, pb)


@pytest.mark.parametrize("rng", ["philox", "ref"])
def test_fp64_exact_multi_group(rng):
    """N = 140k: 547 blocks > one reduction group, so the 2-level hand-off tree (group waves + top wave,
    carried group prefixes) runs; every discrete output must still match the oracle exactly."""
    N = 140_000
    cfg = syn.StreamConfig("t", M=5, B=50, N=N)
    st = syn.make_stream(cfg, 1)
    prm = pf.default_params()
    prm.rng_mode = RNG[rng]
    eng = make_engine(N, st.markers, st.K, pf.STATE_F64, RNG[rng])
    prior = st.prior(fast=True)
    eng.set_prior(prior)
    fr = st.frames[0]
    out, gpu, ref, arr = step_both(eng, prm, st.markers, st.K, prior, fr.current_pose, fr.predicted_pose,
                                   fr.prediction, fr.blobs, seed=4242, frame_idx=fr.index)
    assert_exact(out, gpu, ref, arr, N)
    eng.close()


@pytest.mark.parametrize("fused", [2, 1, 0])  # flat one launch / tree one launch / two launches
def test_fp16_state(fused):
    """fp16-delta state (BASELINE.json configs[3]): per frame the oracle starts from the engine's own
    dequantised prior, so propagation/weights match as in fp32; the resampled set equals the selected
    propagated particles within fp16 quantisation of deltas to the anchor (|delta| * 2^-11)."""
    N, M, B = 20_000, 5, 50
    cfg = syn.StreamConfig("t", M=M, B=B, N=N)
    st = syn.make_stream(cfg, 4)
    prm = pf.default_params()
    eng = make_engine(N, st.markers, st.K, pf.STATE_F16, pf.RNG_PHILOX, fused=fused)
    eng.set_prior(st.prior())
    p0 = eng.get_particles(1)
    assert np.abs(p0 - st.prior()).max() < 2e-4  # import quantisation
    for fr in st.frames:
        prior_used = eng.get_particles(1)
        seed = 90 + fr.index
        out, gpu, ref, arr = step_both(eng, prm, st.markers, st.K, prior_used, fr.current_pose, fr.predicted_pose,
                                       fr.prediction, fr.blobs, seed=seed, frame_idx=fr.index)
        assert out["accepted"] == ref["accepted"] == 1
        dw = np.abs(gpu["weights"] - arr["weights"])
        assert np.sum(dw > 2e-3) <= max(3, N // 1000)
        c = gpu["counts"].astype(np.int64)
        assert c.sum() == N
        src = np.repeat(np.arange(N), c)  # stratified slots in particle order
        err = np.abs(gpu["resampled"] - gpu["propagated"][src])
        delta = np.abs(gpu["propagated"][src] - np.asarray(fr.current_pose).reshape(1, 12))
        assert np.all(err <= delta * 2.0 ** -10 + 1e-7), err.max()
    eng.close()


def test_fp16_state_tracks_fp32():
    """30 frames of a C2-shaped stream, fp16 vs fp32 state.  The tracker's output is the Gauss-Newton
    refinement of the winner over its correspondences (PE:2011-2035): wherever the two runs' winners carry
    the same correspondences their refined poses must coincide (the least-squares optimum depends only
    on pairs and blobs), and they must carry the same correspondences in most frames."""
    N = 50_000
    cfg = syn.StreamConfig("t", M=5, B=50, N=N)
    st = syn.make_stream(cfg, 30)
    runs = {}
    for name, state in (("f32", pf.STATE_F32), ("f16", pf.STATE_F16)):
        eng = make_engine(N, st.markers, st.K, state, pf.RNG_PHILOX)
        eng.set_prior(st.prior())
        outs = []
        for fr in st.frames:
            out = eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=fr.blobs, dt=fr.dt,
                                          seed=3 + fr.index, frame_idx=fr.index)).as_dict()
            assert out["accepted"] == 1
            outs.append(out)
        runs[name] = outs
        eng.close()
    same, compared, its = 0, 0, []
    for fr, a, b in zip(st.frames, runs["f32"], runs["f16"]):
        # the same correspondence SET (extraction order may differ where two markers' distances are close;
        # GN does not depend on it)
        if not np.array_equal(np.sort(a["pairs"], axis=0), np.sort(b["pairs"], axis=0)) or \
                sorted(map(tuple, a["pairs"])) != sorted(map(tuple, b["pairs"])):
            continue
        same += 1
        pa, _, ia = orc.optimise_pose(st.markers, st.K, fr.blobs, a["pairs"], a["winner_pose"])
        pb, _, ib = orc.optimise_pose(st.markers, st.K, fr.blobs, b["pairs"], b["winner_pose"])
        its.append((ia, ib))
        if ia >= 500 or ib >= 500:
            continue  # GN hit its iteration cap in a flat valley (PE:1883-1893): no unique optimum reached
        compared += 1
        assert np.abs(pa[[3, 7, 11]] - pb[[3, 7, 11]]).max() < 1e-4
        assert rotation_angle(syn.to44(pa)[:3, :3], syn.to44(pb)[:3, :3]) < 1e-3
    assert same >= 25, same
    assert compared >= 20, its


@pytest.mark.parametrize("state", ["f64", "f32", "f16"])
def test_predict_roi_matches_oracle(state):
    """ROI prediction (§8f next row 1, PE:396-412): the GPU box over N x M projections of
    camMoveInv * prior_j * predictionMatrix plus the predicted pose, then the reference's corner
    distortion / clamp / cv::Rect, against the oracle on the engine's own prior: bit-exact box, equal ROI."""
    N = 30_000
    cfg = syn.StreamConfig("t", M=5, B=50, N=N)
    st = syn.make_stream(cfg, 3)
    eng = make_engine(N, st.markers, st.K, STATE[state], pf.RNG_PHILOX)
    eng.set_prior(st.prior())
    cam = np.eye(4)
    cam[:3, 3] = [0.01, -0.004, 0.002]
    for fr in st.frames:
        prior = eng.get_particles(1)
        for cm, border in ((None, 20), (cam[:3].reshape(12), 5)):
            got = eng.predict_roi(fr.prediction, fr.predicted_pose, syn.D_README, syn.IMAGE_W, syn.IMAGE_H, border,
                                  cam_move_inv=cm)
            roi, bbox = orc.predict_roi(st.markers, st.K, syn.D_README, prior,
                                        np.eye(4)[:3].reshape(12) if cm is None else cm, fr.prediction,
                                        fr.predicted_pose, syn.IMAGE_W, syn.IMAGE_H, border)
            assert np.array_equal(got["bbox"], bbox), (got["bbox"], bbox)
            assert got["roi"] == roi
        eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=fr.blobs, dt=fr.dt,
                                seed=7 + fr.index, frame_idx=fr.index))
    # prediction far outside the image: the whole image
    far = np.eye(4)[:3].reshape(12).copy()
    far[11] = -5.0  # behind the camera: mirrored projections
    got = eng.predict_roi(np.eye(4)[:3].reshape(12), far, syn.D_README, syn.IMAGE_W, syn.IMAGE_H, 10,
                          cam_move_inv=far)
    roi, _ = orc.predict_roi(st.markers, st.K, syn.D_README, eng.get_particles(1), far,
                             np.eye(4)[:3].reshape(12), far, syn.IMAGE_W, syn.IMAGE_H, 10)
    assert got["roi"] == roi
    eng.close()


@pytest.mark.parametrize("state", ["f64", "f32", "f16"])
@pytest.mark.parametrize("occlude", [False, True])  # True: one LED hidden -> all 80 iterations, kept slot moves
def test_kept_propagated_set_is_bit_identical(state, occlude):
    """Two-launch path: gathering the stored propagated set (PFMPE_OPT_KEEP_PROPAGATED=1, the fp16 default) and
    regenerating it in k_resample (=0) give byte-identical frame records and new priors, frame after frame
    (the stored set follows the weights' slot, so a multi-iteration frame keeps the best iteration's set)."""
    N, M, B = 3000, 5, 30
    cfg = syn.StreamConfig("t", M=M, B=B, N=N)
    st = syn.make_stream(cfg, 3)
    runs = []
    for keep in (1, 0):
        eng = make_engine(N, st.markers, st.K, STATE[state], pf.RNG_PHILOX, fused=0)
        eng.set_option(pf.OPT_KEEP_PROPAGATED, keep)
        eng.set_prior(st.prior())
        recs, priors = [], []
        for fr in st.frames:
            blobs = fr.blobs
            if occlude:
                true_px = syn.project(st.K, fr.truth, st.markers)
                outl = np.random.default_rng(fr.index).uniform([0, 0], [syn.IMAGE_W, syn.IMAGE_H], size=(B - M + 1, 2))
                blobs = np.vstack([true_px[1:], outl])
            out = eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=blobs, dt=fr.dt,
                                          seed=11, frame_idx=fr.index)).as_dict()
            recs.append(out)
            priors.append(eng.get_particles(1))
        eng.close()
        runs.append((recs, priors))
    (ra, pa), (rb, pb) = runs
    for oa, ob in zip(ra, rb):
        for k in oa:
            assert np.array_equal(np.asarray(oa[k]), np.asarray(ob[k])), k
    if occlude:
        assert ra[0]["iters"] > 1 and ra[0]["kept_iter"] >= 0
    for a, b in zip(pa, pb):
        assert np.array_equal(a, b)
