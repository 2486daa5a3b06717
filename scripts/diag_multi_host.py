"""Host-side split of a batch (pfmpe_step_multi, diagnostic): S streams of a config as one batch per frame, the C loop
pfmpe_step_multi_batch; prints wall time per batch and the leader's host timing (undocumented info keys 110-114):
entry -> first launch, the launches, last launch -> records, records -> return.

    python scripts/diag_multi_host.py [--config C4] [--S 2] [--steps 30]
"""
import argparse
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pf_monocular_pose_estimator_amd as pf  # noqa: E402
from pf_monocular_pose_estimator_amd import synthetic as syn  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C4")
ap.add_argument("--S", type=int, default=2)
ap.add_argument("--steps", type=int, default=30)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--diag", type=int, default=0)
a = ap.parse_args()
base = syn.CONFIGS[a.config]
state = pf.STATE_F16 if a.config == "C4" else pf.STATE_F32
n = a.steps + a.warmup
engs, frames = [], []
for s in range(a.S):
    st = syn.make_stream(syn.StreamConfig(base.name, M=base.M, B=base.B, N=base.N, heavy=base.heavy, seed=s), n)
    e = pf.Engine(device=0, max_particles=base.N, state_dtype=state)
    e.set_model(st.markers, st.K)
    e.set_params(pf.default_params())
    e.set_prior(st.prior(fast=True))
    e.stage_blob_bank([f.blobs for f in st.frames])
    if a.diag:
        e.set_option(99, a.diag)
    engs.append(e)
    frames.append([e.make_frame(f.current_pose, f.predicted_pose, f.prediction, B=len(f.blobs), bank_frame=f.index,
                                dt=f.dt, seed=(s << 32) + 17 + f.index, frame_idx=f.index) for f in st.frames])
lib = engs[0].lib
ctxs = (C.c_void_p * a.S)(*[e.ctx.value for e in engs])
ins = (pf.FrameIn * (a.S * n))(*[frames[s][f] for f in range(n) for s in range(a.S)])
outs = (pf.FrameOut * (a.S * n))()
fin, fout = C.sizeof(pf.FrameIn), C.sizeof(pf.FrameOut)
done = C.c_int()


def run(first, count):
    pin = C.cast(C.byref(ins, first * a.S * fin), C.POINTER(pf.FrameIn))
    pout = C.cast(C.byref(outs, first * a.S * fout), C.POINTER(pf.FrameOut))
    engs[0]._chk(lib.pfmpe_step_multi_batch(ctxs, a.S, pin, count, pout, C.byref(done)))


run(0, a.warmup)
k0 = [engs[0].info(k) for k in (110, 111, 112, 113, 114)]
t0 = time.perf_counter()
run(a.warmup, a.steps)
el = time.perf_counter() - t0
k1 = [engs[0].info(k) for k in (110, 111, 112, 113, 114)]
nb = k1[4] - k0[4]
parts = [(k1[i] - k0[i]) / max(nb, 1) / 1e3 for i in range(4)]
upd = sum(base.N * outs[i].iters for i in range(a.warmup * a.S, n * a.S))
print(f"{a.S} x {a.config}: {el * 1e6 / a.steps:.1f} us per batch, {upd / el / 1e9:.2f} G updates/s; host: entry->launch "
      f"{parts[0]:.2f} us, launches {parts[1]:.2f} us, launch->records {parts[2]:.2f} us, records->return {parts[3]:.2f} us "
      f"({nb} batches)")
# one stream alone, pfmpe_step_batch
e = engs[0]
prep = e.prepare_batch(frames[0][a.warmup:])
t0 = time.perf_counter()
o = e.run_batch(prep)
el1 = time.perf_counter() - t0
upd1 = sum(base.N * x.iters for x in o)
print(f"1 x {a.config} alone: {el1 * 1e6 / a.steps:.1f} us per frame, {upd1 / el1 / 1e9:.2f} G updates/s")
for e in engs:
    e.close()
