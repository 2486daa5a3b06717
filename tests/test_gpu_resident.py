"""The resident frame server (PFMPE_OPT_RESIDENT, k_frame2_srv; csrc/pf_kernels.hpp).

The server runs k_frame2's frame body with its blocks kept on the device between frames; the host hands each frame
over through a pinned mailbox instead of a launch.  It must be invisible in the results: every frame's record,
weights, propagated and resampled sets equal a launched k_frame2 run's (which the frame-shape tests pin to the
oracle), whatever the mix of frames and calls:
  * C2's shape (N = 100,000, 391 blocks), host blobs (inline tables) and banked frames, fp32 and fp64, with and
    without read-backs between frames (each read-back ends the server; the next frame starts it again);
  * more frames than one dispatch's ring (kSrvSlots = 256): the server ends by itself and is restarted;
  * a table larger than the server's LDS (B grows): restarted with more;
  * idle gaps past the host's restart bound and past the kernel's own idle bound;
  * a frame abandoned at the wait bound (DIAG_ABANDON): redone by launches, the fallback counted;
  * a second context on the device while the server holds the one-launch slot: it runs two launches;
  * destroy with the server running.
"""
import time

import numpy as np
import pytest

import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn
from test_gpu_parity import make_engine

pytestmark = pytest.mark.gpu


def _engine(N, st, state, resident, fused=2):
    eng = make_engine(N, st.markers, st.K, state, pf.RNG_PHILOX, fused=fused)
    eng.set_option(pf.OPT_RESIDENT, 1 if resident else 0)
    eng.set_prior(st.prior(fast=True))
    return eng


def _frames(st, nframes, bank=False, B_of=None):
    """(frame kwargs) per frame, cycling over the stream's frames with fresh seeds"""
    out = []
    for f in range(nframes):
        fr = st.frames[f % len(st.frames)]
        kw = dict(dt=fr.dt, seed=900 + f, frame_idx=f)
        if bank:
            kw["bank_frame"] = f % len(st.frames)
            kw["B"] = len(fr.blobs)
        else:
            blobs = fr.blobs if B_of is None else fr.blobs[:B_of(f)]
            kw["blobs"] = blobs
        out.append((fr.current_pose, fr.predicted_pose, fr.prediction, kw))
    return out


def _run(eng, frames, read_every=0, sleep_at=None):
    recs, reads = [], []
    for f, (cur, pred, predm, kw) in enumerate(frames):
        if sleep_at and f in sleep_at:
            time.sleep(sleep_at[f])
        recs.append(eng.step(eng.make_frame(cur, pred, predm, **kw)).as_dict())
        if read_every and f % read_every == 0:
            reads.append((eng.get_weights(), eng.get_particles(0), eng.get_particles(1)))
    return recs, reads


def _same_records(a, b):
    assert len(a) == len(b)
    for f, (x, y) in enumerate(zip(a, b)):
        for k, v in x.items():
            assert np.array_equal(np.asarray(v), np.asarray(y[k])), (f, k, v, y[k])


def _same_reads(a, b):
    assert len(a) == len(b)
    for f, (x, y) in enumerate(zip(a, b)):
        for i in range(3):
            assert np.array_equal(x[i], y[i]), (f, i)


@pytest.mark.parametrize("state", [pf.STATE_F32, pf.STATE_F64])
@pytest.mark.parametrize("bank", [False, True])
def test_resident_equals_launched_c2(state, bank):
    N = 100_000
    st = syn.make_stream(syn.StreamConfig("t", M=5, B=50, N=N, seed=5), 6)
    frames = _frames(st, 12, bank=bank)
    runs = {}
    for resident in (True, False):
        eng = _engine(N, st, state, resident)
        try:
            if bank:
                eng.stage_blob_bank([fr.blobs for fr in st.frames])
            recs, _ = _run(eng, frames)  # uninterrupted: one dispatch serves every frame
            if resident:
                assert eng.info(pf.INFO_LAST_SHAPE) == pf.SHAPE_RESIDENT
                assert eng.info(pf.INFO_SERVER_DISPATCHES) == 1
                assert eng.info(pf.INFO_SERVER_FRAMES) == len(frames)
            else:
                assert eng.info(pf.INFO_LAST_SHAPE) == pf.SHAPE_FRAME2
            assert eng.info(pf.INFO_FUSED_FALLBACKS) == 0
            final = (eng.get_weights(), eng.get_particles(0), eng.get_particles(1))
            recs2, reads = _run(eng, frames, read_every=1)  # a read-back after every frame: a dispatch per frame
            if resident:
                assert eng.info(pf.INFO_SERVER_DISPATCHES) == 1 + len(frames)
            runs[resident] = (recs, final, recs2, reads)
        finally:
            eng.close()
    a, b = runs[True], runs[False]
    _same_records(a[0], b[0])
    _same_reads([a[1]], [b[1]])
    _same_records(a[2], b[2])
    _same_reads(a[3], b[3])
    assert any(r["resampled"] for r in a[0])


def test_resident_ring_rollover_and_table_growth():
    """300 frames (> kSrvSlots): the dispatch ends after its last slot and the next frame restarts it.  Blob
    counts growing from 8 to 120 make some frame's table exceed the server's LDS: restarted with more."""
    N = 5_000
    st = syn.make_stream(syn.StreamConfig("t", M=5, B=120, N=N, seed=9), 4)
    frames = _frames(st, 300, B_of=lambda f: 8 + (f * 112) // 299)
    res = {}
    for resident in (True, False):
        eng = _engine(N, st, pf.STATE_F32, resident)
        try:
            recs, _ = _run(eng, frames)
            if resident:
                d = eng.info(pf.INFO_SERVER_DISPATCHES)
                assert 2 <= d <= 8, d
                assert eng.info(pf.INFO_SERVER_FRAMES) == len(frames)
            res[resident] = (recs, eng.get_particles(1))
        finally:
            eng.close()
    _same_records(res[True][0], res[False][0])
    assert np.array_equal(res[True][1], res[False][1])


def test_resident_idle_gaps():
    """A gap past the host's restart bound (0.5 s) and one past the kernel's own idle exit (1 s)."""
    N = 20_000
    st = syn.make_stream(syn.StreamConfig("t", M=5, B=40, N=N, seed=3), 4)
    frames = _frames(st, 8)
    res = {}
    for resident in (True, False):
        eng = _engine(N, st, pf.STATE_F32, resident)
        try:
            recs, _ = _run(eng, frames, sleep_at={3: 0.7, 6: 1.3} if resident else None)
            if resident:
                assert eng.info(pf.INFO_SERVER_DISPATCHES) == 3
                assert eng.info(pf.INFO_FUSED_FALLBACKS) == 0
            res[resident] = (recs, eng.get_particles(1))
        finally:
            eng.close()
    _same_records(res[True][0], res[False][0])
    assert np.array_equal(res[True][1], res[False][1])


def test_resident_abandoned_frame_is_redone():
    """DIAG_ABANDON: every block gives up at the weighing barrier, the server ends, the host redoes the frame by
    two launches (the record a two-launch run gives) and one-launch frames stay off (FUSED_FALLBACKS = 1)."""
    N = 20_000
    st = syn.make_stream(syn.StreamConfig("t", M=5, B=40, N=N, seed=4), 3)
    frames = _frames(st, 3)
    eng = _engine(N, st, pf.STATE_F32, True)
    ref = _engine(N, st, pf.STATE_F32, False, fused=0)
    try:
        r0, _ = _run(eng, frames[:1])
        assert eng.info(pf.INFO_LAST_SHAPE) == pf.SHAPE_RESIDENT
        eng.set_option(pf.OPT_DIAG, pf.DIAG_ABANDON)
        t0 = time.time()
        r1, _ = _run(eng, frames[1:2])
        assert time.time() - t0 < 10
        assert eng.info(pf.INFO_FUSED_FALLBACKS) == 1
        assert eng.info(pf.INFO_LAST_SHAPE) == pf.SHAPE_TWO_LAUNCH
        eng.set_option(pf.OPT_DIAG, 0)
        r2, _ = _run(eng, frames[2:])
        assert eng.info(pf.INFO_LAST_SHAPE) == pf.SHAPE_TWO_LAUNCH  # one-launch frames off after the fallback
        rr, _ = _run(ref, frames)
        _same_records(r0 + r1 + r2, rr)
        assert np.array_equal(eng.get_particles(1), ref.get_particles(1))
    finally:
        eng.close()
        ref.close()


def test_resident_second_context_and_destroy():
    """Context A's server holds the device's one-launch slot: context B's frames run as two launches (guard
    skips) with the results B gives alone; A is destroyed with its server running; B then serves itself."""
    N = 20_000
    st = syn.make_stream(syn.StreamConfig("t", M=5, B=40, N=N, seed=6), 4)
    frames = _frames(st, 4)
    alone = _engine(N, st, pf.STATE_F32, False)
    try:
        ref_b, _ = _run(alone, frames)
    finally:
        alone.close()
    a = _engine(N, st, pf.STATE_F32, True)
    b = _engine(N, st, pf.STATE_F32, True)
    try:
        _run(a, frames[:1])
        assert a.info(pf.INFO_LAST_SHAPE) == pf.SHAPE_RESIDENT
        rb, _ = _run(b, frames[:2])
        assert b.info(pf.INFO_LAST_SHAPE) == pf.SHAPE_TWO_LAUNCH
        assert b.info(pf.INFO_GUARD_SKIPS) >= 2
        a.close()  # server still running
        rb2, _ = _run(b, frames[2:])
        assert b.info(pf.INFO_LAST_SHAPE) == pf.SHAPE_RESIDENT
        _same_records(rb + rb2, ref_b)
    finally:
        a.close()
        b.close()


def test_resident_kernel_stats():
    """PFMPE_OPT_TIMING with the server: each timed frame's device duration goes to K_FRAME."""
    N = 100_000
    st = syn.make_stream(syn.StreamConfig("t", M=5, B=50, N=N, seed=8), 4)
    eng = _engine(N, st, pf.STATE_F32, True)
    try:
        eng.set_option(pf.OPT_TIMING, 1)
        _run(eng, _frames(st, 10))
        ks = eng.kernel_stats()
        n, ms = ks["k_frame"] if "k_frame" in ks else ks[pf.K_FRAME]
        assert n == 10
        assert 0.005 < ms / n < 5.0, ms / n
    finally:
        eng.close()
