"""GPU parity at the frame shapes the benchmark configurations actually run (VERDICT r01 "Next" 1, 6).

* C2's shape: N = 100,000 -> 391 blocks in 7 groups of 64, the flat one-launch frame (k_frame2) and the tree
  one-launch frame (k_frame), fp64 state, both RNG streams: every discrete output equals the oracle's
  (pose_estimator.cpp:535-690), the shape is asserted through pfmpe_get_info.
* The k_frame2 partial hand-off under a lagging reader (partials alternate by iteration parity).
* The one-launch recovery path: a frame abandoned at the wait bound is redone with two launches and gives
  the record a clean two-launch run gives; later frames stay correct; PFMPE_OPT_FUSED_REARM re-arms.
* The in-process guard: two contexts stepping concurrently on one device never deadlock and give the
  results they give alone.
* Full-size property checks of C3 (M=12, B=200 heavy, N=1M, fp32) and C4 (N=10M, fp16 state).
"""
import threading

import numpy as np
import pytest

import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn
from oracle import pforacle as orc
from test_gpu_parity import RNG, assert_exact, make_engine, step_both

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rng", ["ref", "philox"])
@pytest.mark.parametrize("fused,shape", [(2, pf.SHAPE_FRAME2), (1, None)])
def test_fp64_exact_c2_shape(rng, fused, shape):
    """(fused=1: k_frame's fp64 build is not register-capped, so at 391 blocks the residency rule sends it to
    the two-launch path; the frame must be exact whichever shape runs.)"""
    N = 100_000
    cfg = syn.StreamConfig("t", M=5, B=50, N=N)
    st = syn.make_stream(cfg, 1)
    prm = pf.default_params()
    prm.rng_mode = RNG[rng]
    eng = make_engine(N, st.markers, st.K, pf.STATE_F64, RNG[rng], fused=fused)
    prior = st.prior(fast=True)
    eng.set_prior(prior)
    fr = st.frames[0]
    out, gpu, ref, arr = step_both(eng, prm, st.markers, st.K, prior, fr.current_pose, fr.predicted_pose,
                                   fr.prediction, fr.blobs, seed=2024, frame_idx=fr.index)
    if shape is not None:
        assert eng.info(pf.INFO_LAST_SHAPE) == shape
    assert eng.info(pf.INFO_FUSED_FALLBACKS) == 0
    assert_exact(out, gpu, ref, arr, N)
    eng.close()


def _occluded_blobs(st, fr, B, seed):
    true_px = syn.project(st.K, fr.truth, st.markers)
    outl = np.random.default_rng(seed).uniform([0, 0], [syn.IMAGE_W, syn.IMAGE_H], size=(B - len(true_px) + 1, 2))
    return np.vstack([true_px[1:], outl]).astype(np.float32).astype(np.float64)


@pytest.mark.parametrize("state", [pf.STATE_F64, pf.STATE_F32])
def test_frame2_lagging_reader_is_exact(state):
    """k_frame2 with its last block sleeping ~20 us before loading the block partials, on frames that run
    many iterations (one LED occluded, so the exit rule never fires and most iterations do not improve the
    best weight: the case where the slot-indexed partials were reused).  The records and new priors must
    equal the two-launch run's byte for byte; fp64 also equals the oracle.  The same frames with DIAG_MIN_SIDE
    (k_frame2 runs the zmin scans it otherwise skips when no weight is negative) give the same bytes."""
    N, B = 20_000, 30
    cfg = syn.StreamConfig("t", M=5, B=B, N=N)
    st = syn.make_stream(cfg, 2)
    prm = pf.default_params()
    prm.rng_mode = pf.RNG_PHILOX
    runs = []
    for fused, diag in ((2, pf.DIAG_LAG_LOADS), (2, pf.DIAG_MIN_SIDE), (0, 0)):
        eng = make_engine(N, st.markers, st.K, state, pf.RNG_PHILOX, fused=fused)
        eng.set_option(pf.OPT_DIAG, diag)
        eng.set_prior(st.prior())
        recs, priors = [], []
        for fr in st.frames:
            blobs = _occluded_blobs(st, fr, B, fr.index)
            prior = eng.get_particles(1)
            o = eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=blobs, dt=fr.dt,
                                        seed=13, frame_idx=fr.index, force_iters=12)).as_dict()
            assert o["iters"] == 12
            assert eng.info(pf.INFO_LAST_SHAPE) == (pf.SHAPE_FRAME2 if fused else pf.SHAPE_TWO_LAUNCH)
            recs.append(o)
            priors.append(eng.get_particles(1))
            if state == pf.STATE_F64 and fused:
                ref, arr = orc.pf_step(st.markers, st.K, orc.make_params(rng_mode=pf.RNG_PHILOX), prior,
                                       fr.current_pose, fr.predicted_pose, fr.prediction, blobs, dt=fr.dt, seed=13,
                                       frame_idx=fr.index, force_iters=12)
                for k in ("iters", "kept_iter", "accepted", "winner_idx", "most_likely_idx"):
                    assert o[k] == ref[k], k
                if o["resampled"]:
                    np.testing.assert_allclose(priors[-1], arr["resampled"], rtol=0, atol=1e-9)
        assert eng.info(pf.INFO_FUSED_FALLBACKS) == 0
        eng.close()
        runs.append((recs, priors))
    rb, pb = runs[-1]
    for ra, pa in runs[:-1]:
        for oa, ob in zip(ra, rb):
            for k in oa:
                assert np.array_equal(np.asarray(oa[k]), np.asarray(ob[k])), k
        for a, b in zip(pa, pb):
            assert np.array_equal(a, b)


def test_one_launch_recovery_path():
    """A one-launch frame abandoned at the wait bound (simulated: every block gives up its first weighing
    wait) is redone with two launches: the step returns OK with the record a clean two-launch run gives,
    the fallback is counted and reported, later frames stay identical to the two-launch run, and with
    PFMPE_OPT_FUSED_REARM = 2 the context returns to one-launch frames after two clean frames."""
    N = 30_000
    cfg = syn.StreamConfig("t", M=5, B=50, N=N)
    st = syn.make_stream(cfg, 6)
    ref_eng = make_engine(N, st.markers, st.K, pf.STATE_F32, pf.RNG_PHILOX, fused=0)
    eng = make_engine(N, st.markers, st.K, pf.STATE_F32, pf.RNG_PHILOX, fused=2)
    eng.set_option(pf.OPT_FUSED_REARM, 2)
    eng.set_option(pf.OPT_WAIT_BOUND_US, 200_000)
    for e in (ref_eng, eng):
        e.set_prior(st.prior())
    shapes = []
    for fr in st.frames:
        mk = dict(blobs=fr.blobs, dt=fr.dt, seed=21 + fr.index, frame_idx=fr.index)
        if fr.index == 1:
            eng.set_option(pf.OPT_DIAG, pf.DIAG_ABANDON)
        a = eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, **mk)).as_dict()
        shapes.append(eng.info(pf.INFO_LAST_SHAPE))
        if fr.index == 1:
            eng.set_option(pf.OPT_DIAG, 0)
            assert eng.info(pf.INFO_FUSED_FALLBACKS) == 1
            assert eng.info(pf.INFO_FUSED) == 0
            assert "abandoned" in eng.last_error()
        b = ref_eng.step(ref_eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, **mk)).as_dict()
        for k in a:
            assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), (fr.index, k)
        np.testing.assert_array_equal(eng.get_particles(1), ref_eng.get_particles(1))
    # frame 0 one launch; frame 1 abandoned -> two launches; frames 2, 3 two launches (clean); re-armed at 4
    assert shapes == [pf.SHAPE_FRAME2, pf.SHAPE_TWO_LAUNCH, pf.SHAPE_TWO_LAUNCH, pf.SHAPE_TWO_LAUNCH,
                      pf.SHAPE_FRAME2, pf.SHAPE_FRAME2], shapes
    assert eng.info(pf.INFO_FUSED_FALLBACKS) == 1
    eng.close()
    ref_eng.close()


def test_concurrent_contexts_on_one_device():
    """Two contexts (two camera streams) stepped from two threads on one device: the in-process guard lets
    at most one one-launch frame spin at a time, so no frame is abandoned, and every record and new prior
    equals that stream's run alone."""
    N, F = 100_000, 16
    streams = [syn.make_stream(syn.StreamConfig("t", M=5, B=50, N=N, seed=s), F) for s in (0, 1)]

    def run(st, seed, out):
        eng = make_engine(N, st.markers, st.K, pf.STATE_F32, pf.RNG_PHILOX, fused=2)
        eng.set_prior(st.prior())
        eng.stage_blob_bank([f.blobs for f in st.frames])
        frames = [eng.make_frame(f.current_pose, f.predicted_pose, f.prediction, B=len(f.blobs), bank_frame=f.index,
                                 dt=f.dt, seed=seed + f.index, frame_idx=f.index) for f in st.frames]
        recs = [o.as_dict() for o in eng.step_batch(frames)]
        out.append((recs, eng.get_particles(1), eng.info(pf.INFO_FUSED_FALLBACKS), eng.info(pf.INFO_GUARD_SKIPS)))
        eng.close()

    alone = []
    for i, st in enumerate(streams):
        res = []
        run(st, 100 * i, res)
        alone.append(res[0])
    together = [[], []]
    th = [threading.Thread(target=run, args=(st, 100 * i, together[i])) for i, st in enumerate(streams)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    for i in range(2):
        recs, post, fallbacks, _ = together[i][0]
        assert fallbacks == 0
        for a, b in zip(recs, alone[i][0]):
            for k in a:
                assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), (i, k)
        np.testing.assert_array_equal(post, alone[i][1])


def _full_size_properties(name, state, max_bad_frac):
    cfg = syn.CONFIGS[name]
    st = syn.make_stream(cfg, 1)
    fr = st.frames[0]
    prm = pf.default_params()
    eng = make_engine(cfg.N, st.markers, st.K, state, pf.RNG_PHILOX)
    eng.set_prior(st.prior(fast=True))
    out = eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=fr.blobs, dt=fr.dt,
                                  seed=4, frame_idx=0)).as_dict()
    assert eng.info(pf.INFO_LAST_SHAPE) == pf.SHAPE_TWO_LAUNCH  # these sizes run as two launches
    assert out["accepted"] == 1
    N = cfg.N
    w = eng.get_weights()
    counts = eng.get_counts().astype(np.int64)
    assert counts.sum() == N  # every stratified target finds a particle (normalised total == 1)
    assert out["winner_idx"] == int(np.argmax(counts))  # first maximum (PE:685-686)
    owner = np.repeat(np.arange(N), counts)  # slot k holds the particle whose range covers k
    rng = np.random.default_rng(0)
    prop = eng.get_particles(0)
    post = eng.get_particles(1)
    if state == pf.STATE_F16:
        delta = np.abs(prop[owner] - np.asarray(fr.current_pose).reshape(1, 12))
        assert np.all(np.abs(post - prop[owner]) <= delta * 2.0 ** -10 + 1e-7)
    else:
        np.testing.assert_array_equal(post, prop[owner])
    del post
    np.testing.assert_allclose(out["winner_pose"], prop[out["winner_idx"]], atol=1e-6)
    proj = np.array([orc.project(st.K, prop[out["winner_idx"]], X) for X in st.markers])
    _, pairs = orc.likelihood(proj, fr.blobs, prm.tol, prm.tol_pf)
    assert np.array_equal(out["pairs"], pairs)
    # the oracle likelihood (fp64, literal minCoeff form) on a sample of the GPU's own propagated poses
    sub = rng.choice(N, 1500, replace=False)
    bad = 0
    for n in sub:
        proj = np.array([orc.project(st.K, prop[n], X) for X in st.markers])
        P, _ = orc.likelihood(proj, fr.blobs, prm.tol, prm.tol_pf)
        bad += abs(P - w[n]) > 2e-3
    assert bad <= max(3, int(max_bad_frac * len(sub)))
    assert out["highest_prob"] == pytest.approx(float(w.max()), abs=1e-6)
    eng.close()


def test_c3_full_size_properties():
    _full_size_properties("C3", pf.STATE_F32, 0.002)


def test_c4_full_size_properties():
    _full_size_properties("C4", pf.STATE_F16, 0.002)


@pytest.mark.parametrize("state,N,M,B,heavy,rng,prune", [
    (pf.STATE_F64, 140_000, 5, 50, False, pf.RNG_PHILOX, True),
    (pf.STATE_F32, 1_200_000, 5, 50, False, pf.RNG_PHILOX, True),
    (pf.STATE_F16, 1_200_000, 12, 200, True, pf.RNG_PHILOX, True),
    (pf.STATE_F32, 1_200_000, 12, 200, True, pf.RNG_PHILOX, True),  # C3's instantiation (VERDICT r05 missing 2)
    (pf.STATE_F32, 300_000, 5, 50, False, pf.RNG_REFERENCE, False),  # reference stream, unpruned scan
    (pf.STATE_F16, 3_000_000, 5, 50, False, pf.RNG_PHILOX, True),  # 109 groups: k_top_wide over 2 tiles
    (pf.STATE_F64, 1_100_000, 5, 50, False, pf.RNG_REFERENCE, True),  # fp64, 66 groups: k_top_wide
])
def test_streaming_weighing_is_bit_identical(state, N, M, B, heavy, rng, prune):
    """The two-launch path's streaming weighing pass (k_weigh_stream + k_group + k_top: resident blocks
    looping over the 256-particle blocks, the next particle's state prefetched) against the
    one-block-per-256-particles k_propagate_weigh: identical records, weights, propagated and resampled sets
    over a steady frame and an 80-iteration frame (one LED hidden), one tile of groups (140k) and several
    (1.2M: 4,688 blocks in 74 groups; 3M: 109 groups), fp64 / fp32 / fp16 state, both RNG streams, pruned and
    unpruned.  Beyond one tile of groups the streaming pass's top is k_top_wide (16 waves, the per-tile passes
    in parallel); the one-block pass keeps propagate_top's serial tiles.  The packed pass (k_weigh_pk, taken by
    default where it applies: fp32 compute, Philox, 5 markers) is a third variant of the same pass."""
    cfg = syn.StreamConfig("t", M=M, B=B, N=N, heavy=heavy)
    st = syn.make_stream(cfg, 2)
    prior = st.prior(fast=True)
    res = []
    variants = [(pf.DIAG_FORCE_STREAM | pf.DIAG_NO_PK, (pf.WEIGH_STREAM,)),
                (pf.DIAG_FORCE_STREAM, (pf.WEIGH_STREAM, pf.WEIGH_PK)),
                (pf.DIAG_NO_STREAM, (pf.WEIGH_BLOCKS,))]
    for diag, passes in variants:
        eng = make_engine(N, st.markers, st.K, state, rng, prune=prune, fused=0)
        eng.set_option(pf.OPT_DIAG, diag)
        eng.set_prior(prior)
        snaps = []
        for f, fr in enumerate(st.frames):
            blobs = fr.blobs
            kw = {}
            if f == 1:  # LED 0's blob hidden: all 80 iterations, the kept slot moves (forced with clutter)
                uv0 = syn.project(st.K, fr.truth, st.markers)[0]
                blobs = np.delete(blobs, int(np.argmin(np.sum((blobs - uv0) ** 2, axis=1))), axis=0)
                kw = {"force_iters": 80} if heavy else {}
            out = eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=blobs, dt=fr.dt,
                                          seed=77 + f, frame_idx=f, **kw)).as_dict()
            snap = {"out": out, "w": eng.get_weights(), "p0": eng.get_particles(0)}
            if out["resampled"]:
                snap["p1"] = eng.get_particles(1)
                snap["counts"] = eng.get_counts()
            snaps.append(snap)
        assert eng.info(pf.INFO_LAST_SHAPE) == pf.SHAPE_TWO_LAUNCH
        assert eng.info(pf.INFO_LAST_WEIGH_PASS) in passes, (diag, eng.info(pf.INFO_LAST_WEIGH_PASS))
        eng.close()
        res.append(snaps)
    assert res[0][1]["out"]["iters"] == 80
    for other in res[:2]:
        for a, b in zip(other, res[2]):
            for k, v in a["out"].items():
                assert np.array_equal(np.asarray(v), np.asarray(b["out"][k])), k
            for k in ("w", "p0", "p1", "counts"):
                assert (k in a) == (k in b)
                if k in a:
                    assert np.array_equal(a[k], b[k]), k
