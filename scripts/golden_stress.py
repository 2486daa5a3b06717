"""Diagnostic: replay one golden fixture through one frame shape many times in one process and report every
frame whose discrete outputs or counts differ from the fixture (first-mismatch details printed)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pf_monocular_pose_estimator_amd as pf  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "pf_c1_reference_rng"
fused = int(sys.argv[2]) if len(sys.argv) > 2 else 2
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 100
g = dict(np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                              name + ".npz")))
N = g["prior0"].shape[0]
INT_KEYS = ("iters", "kept_iter", "accepted", "resampled", "most_likely_idx", "winner_idx", "n_corr", "flag_fail")
bad = 0
for rep in range(reps):
    eng = pf.Engine(device=0, max_particles=N, max_blobs=int(g["B"].max()), state_dtype=pf.STATE_F64)
    eng.set_model(g["markers"], g["K"])
    prm = pf.default_params()
    prm.rng_mode = int(g["rng_mode"])
    eng.set_params(prm)
    eng.set_option(pf.OPT_RECORD_COUNTS, 1)
    eng.set_option(pf.OPT_FUSED, fused)
    eng.set_prior(g["prior0"])
    for f in range(len(g["seed"])):
        B = int(g["B"][f])
        fr = eng.make_frame(g["cur"][f], g["pred"][f], g["predm"][f], dt=float(g["dt"][f]), seed=int(g["seed"][f]),
                            frame_idx=int(g["frame_idx"][f]), blobs=g["blobs"][f][:B])
        out = eng.step(fr).as_dict()
        diff = [k for k in INT_KEYS if out[k] != g[k][f]]
        w = eng.get_weights()
        wd = float(np.max(np.abs(w - g["weights"][f])))
        cd = None
        if out["resampled"]:
            c = eng.get_counts()
            cd = np.nonzero(c != g["counts"][f])[0]
        if diff or wd > 1e-9 or (cd is not None and len(cd)):
            bad += 1
            if bad <= 3:
                print("MISMATCH rep", rep, "frame", f, "keys", diff, {k: (out[k], int(g[k][f])) for k in diff},
                      "max|dw|", wd, "count idx", None if cd is None else cd[:10].tolist(),
                      "gpu", None if cd is None else c[cd[:10]].tolist(), "gold",
                      None if cd is None else g["counts"][f][cd[:10]].tolist(),
                      "fallbacks", eng.info(pf.INFO_FUSED_FALLBACKS), "shape", eng.info(pf.INFO_LAST_SHAPE),
                      flush=True)
    eng.close()
    if rep % 20 == 0:
        print("rep", rep, "bad frames so far", bad, flush=True)
print("DONE reps", reps, "bad frames", bad)
