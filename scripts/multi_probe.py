#!/usr/bin/env python3
"""Batched-vs-solo probe of pfmpe_step_multi at large per-stream sizes.

S streams of N particles each run F frames twice: once as batches (pfmpe_step_multi, optionally split into G
concurrent batches on G host threads) and once stream by stream (pfmpe_step, two-launch shape).  Every record
field and a digest of every stream's resampled set must be identical.  Prints one line per frame and a final
verdict; exit status 0 only when everything matched.

    python scripts/multi_probe.py --S 2 --N 3000000 --state f16 --frames 2 [--groups 1]
"""
from __future__ import annotations

import argparse
import hashlib
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import pf_monocular_pose_estimator_amd as pf  # noqa: E402
from pf_monocular_pose_estimator_amd import synthetic as syn  # noqa: E402


def engine(N, st, state, fused):
    e = pf.Engine(device=0, max_particles=N, state_dtype=state)
    e.set_option(pf.OPT_FUSED, fused)
    e.set_model(st.markers, st.K)
    e.set_params(pf.default_params())
    e.set_prior(st.prior(N))
    e.stage_blob_bank([f.blobs for f in st.frames])
    return e


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--S", type=int, default=2)
    ap.add_argument("--N", type=int, default=3_000_000)
    ap.add_argument("--state", default="f16", choices=["f16", "f32", "f64"])
    ap.add_argument("--frames", type=int, default=2)
    ap.add_argument("--groups", type=int, default=1)
    ap.add_argument("--no-solo", action="store_true", help="batched run only (no comparison)")
    a = ap.parse_args()
    state = {"f16": pf.STATE_F16, "f32": pf.STATE_F32, "f64": pf.STATE_F64}[a.state]
    streams = [syn.make_stream(syn.StreamConfig("p", M=5, B=50, N=a.N, seed=s), a.frames) for s in range(a.S)]
    t0 = time.time()
    batch = [engine(a.N, st, state, 0) for st in streams]
    solo = [] if a.no_solo else [engine(a.N, st, state, 0) for st in streams]
    print(f"setup {time.time() - t0:.1f} s: {a.S} x {a.N} {a.state}, groups {a.groups}", flush=True)
    G = max(1, min(a.groups, a.S))
    parts = [list(range(a.S))[g::G] for g in range(G)]
    ok = True
    try:
        for f in range(a.frames):
            ins = {}
            for s, st in enumerate(streams):
                fr = st.frames[f]
                ins[s] = [e.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, B=len(fr.blobs),
                                       bank_frame=f, dt=fr.dt, seed=(s << 32) + 17 + f, frame_idx=f)
                          for e in ([batch[s]] + ([solo[s]] if solo else []))]
            outs = {}
            errs = []

            def run(part):
                try:
                    res = pf.Engine.step_multi([batch[s] for s in part], [ins[s][0] for s in part])
                    for s, o in zip(part, res):
                        outs[s] = o
                except Exception as ex:  # noqa: BLE001
                    errs.append(repr(ex))

            t1 = time.time()
            if G == 1:
                run(parts[0])
            else:
                th = [threading.Thread(target=run, args=(p,)) for p in parts]
                for t in th:
                    t.start()
                for t in th:
                    t.join()
            tb = time.time() - t1
            if errs:
                print("batched step failed:", errs, flush=True)
                return 1
            print(f"frame {f}: batch {tb * 1e3:.1f} ms, iters {[outs[s].iters for s in range(a.S)]}", flush=True)
            if not solo:
                continue
            for s in range(a.S):
                ro = solo[s].step(ins[s][1])
                da, db = outs[s].as_dict(), ro.as_dict()
                for k in da:
                    same = np.array_equal(da[k], db[k]) if isinstance(da[k], np.ndarray) else da[k] == db[k]
                    if not same:
                        ok = False
                        print(f"  stream {s} frame {f}: record field {k} differs: {da[k]} vs {db[k]}", flush=True)
                if da["resampled"]:
                    ha = hashlib.sha1(batch[s].get_particles(1).tobytes()).hexdigest()
                    hb = hashlib.sha1(solo[s].get_particles(1).tobytes()).hexdigest()
                    if ha != hb:
                        ok = False
                        print(f"  stream {s} frame {f}: resampled sets differ", flush=True)
            print(f"frame {f}: compared {a.S} streams, {'identical' if ok else 'MISMATCH'}", flush=True)
    finally:
        for e in batch + solo:
            e.close()
    print("PROBE", "OK" if ok else "MISMATCH", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
