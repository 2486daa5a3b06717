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


def _streams(n_frames, cfgs=STREAMS):
    out = []
    for s, (N, M, B, heavy, how) in enumerate(cfgs):
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


def _check_batch(state, rng, n_frames, cfgs=STREAMS, strict_occlude=True, passes_out=None):
    streams = _streams(n_frames, cfgs)
    batch, solo, occl_iters, passes = [], [], [], []
    for (st, frames, how), (N, M, *_rest) in zip(streams, cfgs):
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
                    occl_iters.append(outs[s].iters)
                    assert outs[s].iters == 80 or not strict_occlude
                if how == "empty":
                    assert outs[s].flag_fail == pf.FLAG_REINIT
            assert batch[0].info(pf.INFO_LAST_SHAPE) == pf.SHAPE_TWO_LAUNCH
            passes.append(batch[0].info(pf.INFO_LAST_WEIGH_PASS))
    finally:
        for e in batch + solo:
            e.close()
    if passes_out is not None:
        passes_out.extend(passes)
    return occl_iters


@pytest.mark.parametrize("state,rng", [(pf.STATE_F64, pf.RNG_REFERENCE), (pf.STATE_F32, pf.RNG_PHILOX),
                                       (pf.STATE_F16, pf.RNG_PHILOX)])
def test_multi_equals_single_streams(state, rng):
    _check_batch(state, rng, 3)


def test_multi_restaging_after_later_rounds():
    """Every frame's later iteration rounds (the occluded stream) stage a one-stream layout into the batch's
    host image; the next frame's first round stages the full layout at the same addresses.  The staging launch
    must read the image the host just wrote, never a cached copy of the previous round's."""
    cfgs = [(4099, 5, 50, False, "occlude"), (300, 5, 3, False, ""), (1000, 5, 20, False, ""),
            (2048, 12, 200, True, "")]
    iters = _check_batch(pf.STATE_F64, pf.RNG_REFERENCE, 8, cfgs, strict_occlude=False)
    assert sum(i > 1 for i in iters[:-1]) >= 2, iters  # frames with later rounds, each followed by another frame


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


# ---------------------------------------------------------------------------------------------------------
# Large streams (a batch of 8 x 10M fp16 streams faulted once, and the batched tests stopped at
# 100k particles / 7 groups per stream).  At 3M particles a stream has 11,719 blocks in 184 groups of 64 (the
# in-launch tree hand-off walks 3 tiles of groups), at 10M 39,063 blocks in 611 groups (10 tiles).  Each
# batched stream must equal its own pfmpe_step bit for bit: every record field, the kept weights and the
# resampled set (compared as SHA-1 digests: 10M x 12 doubles per stream).

def _big_streams(S, N, n_frames, seed0=0):
    return [syn.make_stream(syn.StreamConfig("big", M=5, B=50, N=N, seed=seed0 + s), n_frames) for s in range(S)]


def _big_engine(st, N, state=pf.STATE_F16):
    e = pf.Engine(device=0, max_particles=N, state_dtype=state)
    e.set_option(pf.OPT_FUSED, 0)
    e.set_model(st.markers, st.K)
    e.set_params(pf.default_params())
    if getattr(st, "_prior", None) is None or len(st._prior) != N:  # one prior per stream (batch and solo engines)
        st._prior = st.prior(N)
    e.set_prior(st._prior)
    e.stage_blob_bank([f.blobs for f in st.frames])
    return e


def _big_frame(e, st, f, s):
    fr = st.frames[f]
    return e.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, B=len(fr.blobs), bank_frame=f, dt=fr.dt,
                        seed=(s << 32) + 17 + f, frame_idx=f)


def _digest(a):
    import hashlib
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()


def _big_compare(batch, solo, outs, streams, f):
    for s, st in enumerate(streams):
        ref = solo[s].step(_big_frame(solo[s], st, f, s))
        a, b = outs[s].as_dict(), ref.as_dict()
        for k in a:
            if isinstance(a[k], np.ndarray):
                assert np.array_equal(a[k], b[k]), (s, f, k)
            else:
                assert a[k] == b[k], (s, f, k, a[k], b[k])
        assert _digest(batch[s].get_weights()) == _digest(solo[s].get_weights()), (s, f, "weights")
        if a["resampled"]:
            assert _digest(batch[s].get_particles(1)) == _digest(solo[s].get_particles(1)), (s, f, "resampled set")


@pytest.mark.parametrize("S,N,frames", [(2, 3_000_000, 2), (2, 10_000_000, 2)])
def test_multi_large_fp16_streams_bit_identical(S, N, frames):
    streams = _big_streams(S, N, frames)
    batch = [_big_engine(st, N) for st in streams]
    solo = [_big_engine(st, N) for st in streams]
    try:
        for f in range(frames):
            outs = pf.Engine.step_multi(batch, [_big_frame(batch[s], st, f, s) for s, st in enumerate(streams)])
            assert all(o.accepted == 1 for o in outs)
            _big_compare(batch, solo, outs, streams, f)
    finally:
        for e in batch + solo:
            e.close()


def test_multi_large_concurrent_batches():
    """4 x 10M fp16 streams: one batch of all four (156,252 blocks, just below the batch limit), then the same
    streams as two concurrent batches of two on two host threads (the configuration of the round-2 fault);
    every stream equals its pfmpe_step run."""
    import threading
    S, N, frames = 4, 10_000_000, 2
    streams = _big_streams(S, N, frames, seed0=10)
    batch = [_big_engine(st, N) for st in streams]
    solo = [_big_engine(st, N) for st in streams]
    try:
        outs = pf.Engine.step_multi(batch, [_big_frame(batch[s], st, 0, s) for s, st in enumerate(streams)])
        _big_compare(batch, solo, outs, streams, 0)
        res, errs = {}, []

        def run(part):
            try:
                o = pf.Engine.step_multi([batch[s] for s in part], [_big_frame(batch[s], streams[s], 1, s) for s in part])
                res.update(zip(part, o))
            except Exception as ex:  # noqa: BLE001
                errs.append(repr(ex))

        th = [threading.Thread(target=run, args=(p,)) for p in ([0, 2], [1, 3])]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs, errs
        _big_compare(batch, solo, [res[s] for s in range(S)], streams, 1)
    finally:
        for e in batch + solo:
            e.close()


def test_multi_block_limit():
    """A batch above PFMPE_OPT_MULTI_MAX_BLOCKS is refused with PFMPE_E_CAP and nothing runs; the same
    streams then batch normally under the default limit."""
    st = syn.make_stream(syn.StreamConfig("m", M=5, B=50, N=100_000), 1)
    fr = st.frames[0]
    engs = [_engine(100_000, 5, pf.STATE_F32, pf.RNG_PHILOX) for _ in range(2)]
    try:
        for e in engs:
            e.set_prior(st.prior())
        ins = [e.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=fr.blobs, dt=fr.dt, seed=5 + s,
                            frame_idx=0) for s, e in enumerate(engs)]
        engs[0].set_option(pf.OPT_MULTI_MAX_BLOCKS, 500)  # 2 x 391 blocks
        with pytest.raises(pf.PFError) as ei:
            pf.Engine.step_multi(engs, ins)
        assert ei.value.code == pf.E_CAP
        with pytest.raises(pf.PFError):
            engs[0].set_option(pf.OPT_MULTI_MAX_BLOCKS, 160_001)
        engs[0].set_option(pf.OPT_MULTI_MAX_BLOCKS, 160_000)
        outs = pf.Engine.step_multi(engs, ins)
        assert all(o.accepted == 1 for o in outs)
        bad = engs[1].make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=np.zeros((2000, 2)),
                                 dt=fr.dt, seed=1, frame_idx=1)
        with pytest.raises(pf.PFError) as ei:  # B above max_blobs: the stream's own pfmpe_step code
            pf.Engine.step_multi(engs, [ins[0], bad])
        assert ei.value.code == pf.E_CAP
    finally:
        for e in engs:
            e.close()


@pytest.mark.parametrize("state", [pf.STATE_F32, pf.STATE_F16])
def test_multi_interleaved_with_single_steps(state):
    """a batch runs on the leader's stream, each member's pfmpe_step / read-backs on its own.
    Frames alternate per stream between the batch and pfmpe_step (and each frame's counts are read right
    away), with the leader changing between frames; every stream must equal a stream stepped only with
    pfmpe_step.  N = 300k: two-launch frames, so kernels are still retiring when records arrive."""
    S, N, frames = 3, 300_000, 6
    streams = _big_streams(S, N, frames, seed0=30)
    mixed = [_big_engine(st, N, state) for st in streams]
    solo = [_big_engine(st, N, state) for st in streams]
    for e in mixed + solo:
        e.set_option(pf.OPT_RECORD_COUNTS, 1)
    try:
        for f in range(frames):
            batched = [s for s in range(S) if (s + f) % 3 != 0]  # two streams batched, one stepped alone
            lead = batched[f % len(batched)]
            order = [lead] + [s for s in batched if s != lead]
            outs = dict(zip(order, pf.Engine.step_multi([mixed[s] for s in order],
                                                        [_big_frame(mixed[s], streams[s], f, s) for s in order])))
            for s in range(S):
                if s not in outs:
                    outs[s] = mixed[s].step(_big_frame(mixed[s], streams[s], f, s))
                counts = mixed[s].get_counts()
                ref = solo[s].step(_big_frame(solo[s], streams[s], f, s))
                assert outs[s].as_dict()["winner_idx"] == ref.winner_idx, (s, f)
                assert np.array_equal(counts, solo[s].get_counts()), (s, f)
                assert np.array_equal(outs[s].as_dict()["winner_pose"], ref.as_dict()["winner_pose"]), (s, f)
        for s in range(S):
            assert _digest(mixed[s].get_particles(1)) == _digest(solo[s].get_particles(1)), s
    finally:
        for e in mixed + solo:
            e.close()


def test_multi_member_after_leader_frames():
    """after a batch the leader keeps stepping alone (its own frames on the batch stream) while the member
    still holds the batch's fence; the leader records the fence before its first later frame (seal_lead_fence).  The
    member's read-back and next frame must then see exactly the batch's result, and a second batch of the same two
    contexts after that (the fence re-armed) must too.  Every output equals the streams' own pfmpe_step runs."""
    S, N, frames = 2, 3_000_000, 5
    streams = _big_streams(S, N, frames, seed0=50)
    batch = [_big_engine(st, N) for st in streams]
    solo = [_big_engine(st, N) for st in streams]
    try:
        outs = pf.Engine.step_multi(batch, [_big_frame(batch[s], st, 0, s) for s, st in enumerate(streams)])
        for s in range(S):
            r = solo[s].step(_big_frame(solo[s], streams[s], 0, s)).as_dict()
            o = outs[s].as_dict()
            for k in o:
                assert np.array_equal(np.asarray(o[k]), np.asarray(r[k])), (s, k)
        # the member's read-back right after the batch
        assert _digest(batch[1].get_weights()) == _digest(solo[1].get_weights())
        for f in (1, 2):  # the leader alone, the member idle
            a = batch[0].step(_big_frame(batch[0], streams[0], f, 0)).as_dict()
            b = solo[0].step(_big_frame(solo[0], streams[0], f, 0)).as_dict()
            assert a["winner_idx"] == b["winner_idx"] and np.array_equal(a["winner_pose"], b["winner_pose"]), f
        m = batch[1].step(_big_frame(batch[1], streams[1], 1, 1)).as_dict()  # the member's next frame, own stream
        r = solo[1].step(_big_frame(solo[1], streams[1], 1, 1)).as_dict()
        assert m["winner_idx"] == r["winner_idx"] and np.array_equal(m["winner_pose"], r["winner_pose"])
        outs = pf.Engine.step_multi(batch, [_big_frame(batch[0], streams[0], 3, 0), _big_frame(batch[1], streams[1], 2, 1)])
        ra = solo[0].step(_big_frame(solo[0], streams[0], 3, 0)).as_dict()
        rb = solo[1].step(_big_frame(solo[1], streams[1], 2, 1)).as_dict()
        for o, r in zip(outs, (ra, rb)):
            assert o.as_dict()["winner_idx"] == r["winner_idx"]
        for s in range(S):
            assert _digest(batch[s].get_particles(1)) == _digest(solo[s].get_particles(1)), s
    finally:
        for e in batch + solo:
            e.close()


@pytest.mark.parametrize("state,rng", [(pf.STATE_F16, pf.RNG_PHILOX), (pf.STATE_F64, pf.RNG_REFERENCE)])
def test_multi_corrupt_descriptor_is_reported(state, rng):
    """a stream descriptor the device reads differently from what the host wrote is refused
    before any of its pointers is followed.  PFMPE_DIAG 8192 alters the first stream's key word in the host image
    after its tag was computed (a key word, never a pointer: nothing wild could be dereferenced even if the check
    failed).  The batch must return PFMPE_E_STATE naming the differing word with both values; no context's prior
    may change (the failed batch is as if it never ran), and the same contexts then batch normally and equal their
    own pfmpe_step runs."""
    cfgs = [(1000, 5, 20, False, ""), (4099, 5, 50, False, ""), (2048, 12, 200, True, "")]
    streams = _streams(2, cfgs)
    batch, solo = [], []
    for (st, frames, how), (N, M, *_r) in zip(streams, cfgs):
        for lst, fused in ((batch, 0), (solo, 2)):
            eng = _engine(N, M, state, rng, fused=fused)
            eng.set_prior(st.prior(N))
            lst.append(eng)
    try:
        before = [e.get_particles(1) for e in batch]
        batch[0].set_option(pf.OPT_DIAG, pf.DIAG_CORRUPT_DESC)
        ins = [_frame(batch[s], streams[s][1][0][0], streams[s][1][0][1], "", 500 + s, 0) for s in range(len(cfgs))]
        with pytest.raises(pf.PFError) as ei:
            pf.Engine.step_multi(batch, ins)
        assert ei.value.code == pf.E_STATE, str(ei.value)
        msg = str(ei.value)
        assert "stream 0" in msg and "staging check" in msg and "host 0x" in msg and "device 0x" in msg, msg
        for e, b in zip(batch, before):
            assert np.array_equal(e.get_particles(1), b)
        batch[0].set_option(pf.OPT_DIAG, 0)
        for f in range(2):
            seeds = [700 + 3 * s + f for s in range(len(cfgs))]
            ins = [_frame(batch[s], streams[s][1][f][0], streams[s][1][f][1], "", seeds[s], f) for s in range(len(cfgs))]
            outs = pf.Engine.step_multi(batch, ins)
            for s in range(len(cfgs)):
                fr, blobs = streams[s][1][f]
                ref = solo[s].step(_frame(solo[s], fr, blobs, "", seeds[s], f))
                _same(_snapshot(batch[s], outs[s]), _snapshot(solo[s], ref), (state, s, f))
    finally:
        for e in batch + solo:
            e.close()


@pytest.mark.parametrize("state", [pf.STATE_F32, pf.STATE_F16])
def test_multi_streaming_pk_batch_equals_single_streams(state):
    """The streaming packed batch (k_weigh_pk_multi + the batched group / top hand-off; every stream 5 LEDs with
    B >= M, fp32 or fp16, Philox): per-stream workgroup shares of different sizes, one occluded stream (all 80
    iterations: later rounds run a subset), one stream beyond one tile of groups (3M particles: 108 groups, the
    k_group_multi + k_top_wide_multi hand-off), N not a multiple of 128.  Every stream bit-identical to its own
    pfmpe_step (whose two-launch frames run k_weigh_pk), over 3 frames."""
    cfgs = [(100_000, 5, 50, False, ""), (4099, 5, 50, False, "occlude"), (3_000_017, 5, 50, False, ""),
            (777, 5, 20, False, "")]
    _check_batch(state, pf.RNG_PHILOX, 3, cfgs, passes_out=(passes := []))
    assert passes and all(p == pf.WEIGH_PK for p in passes), passes


def test_multi_abandoned_finish_leaves_no_state():
    """A batch in which one stream's finishing wave gives up (that context's PFMPE_DIAG 131072) fails as a whole
    (no record for that stream); every stream's keys and arrival shards are zeroed, and the next batch, on different
    frames, equals solo engines that never saw the failed batch."""
    cfgs = [(100_000, 5, 50, False, ""), (4099, 5, 50, False, "")]
    streams = _streams(3, cfgs)
    batch, solo = [], []
    for (st, frames, how), (N, M, *_rest) in zip(streams, cfgs):
        for lst in (batch, solo):
            e = _engine(N, M, pf.STATE_F32, pf.RNG_PHILOX, fused=0)
            e.set_prior(st.prior(N))
            lst.append(e)
    try:
        def ins_for(engs, f):
            return [_frame(engs[s], streams[s][1][f][0], streams[s][1][f][1], "", 1000 + 17 * s + f, f)
                    for s in range(len(streams))]
        pf.Engine.step_multi(batch, ins_for(batch, 0))
        for s in range(len(streams)):
            solo[s].step(ins_for(solo, 0)[s])
        batch[1].set_option(pf.OPT_DIAG, pf.DIAG_ABANDON_FINISH)
        with pytest.raises(pf.PFError):
            pf.Engine.step_multi(batch, ins_for(batch, 1))
        batch[1].set_option(pf.OPT_DIAG, 0)
        outs = pf.Engine.step_multi(batch, ins_for(batch, 2))
        assert batch[0].info(pf.INFO_LAST_RESAMPLE) == pf.RESAMPLE_OWNERS
        for s in range(len(streams)):
            ref = solo[s].step(ins_for(solo, 2)[s])
            _same(_snapshot(batch[s], outs[s]), _snapshot(solo[s], ref), ("after abandon", s))
    finally:
        for e in batch + solo:
            e.close()
