"""fp32 vs fp16 winners on a C2-shaped stream: per frame, pairs equality and GN-refined pose agreement."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn
from oracle import pforacle as orc
N = 50_000
st = syn.make_stream(syn.StreamConfig("t", M=5, B=50, N=N), 30)
runs = {}
for name, state in (("f32", pf.STATE_F32), ("f16", pf.STATE_F16)):
    eng = pf.Engine(0, N, state_dtype=state)
    eng.set_model(st.markers, st.K); eng.set_params(pf.default_params()); eng.set_prior(st.prior())
    runs[name] = [eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=fr.blobs,
                                          dt=fr.dt, seed=3 + fr.index, frame_idx=fr.index)).as_dict() for fr in st.frames]
    eng.close()
np.savez("gpurun_out/diag_gn.npz", **{f"{k}_{i}_{f}": np.asarray(o[f]) for k, v in runs.items() for i, o in enumerate(v)
                                       for f in ("winner_pose", "pairs")})
for i, (fr, a, b) in enumerate(zip(st.frames, runs["f32"], runs["f16"])):
    eq = np.array_equal(a["pairs"], b["pairs"])
    pa, _, ia = orc.optimise_pose(st.markers, st.K, fr.blobs, a["pairs"], a["winner_pose"])
    pb, _, ib = orc.optimise_pose(st.markers, st.K, fr.blobs, b["pairs"], b["winner_pose"])
    R1, R0 = syn.to44(pa)[:3, :3], syn.to44(pb)[:3, :3]
    ang = np.arccos(np.clip((np.trace(R1.T @ R0) - 1) / 2, -1, 1))
    print(i, "pairs_eq", eq, "n", len(a["pairs"]), len(b["pairs"]), "it", ia, ib, "dt %.2e" % np.abs(pa[[3, 7, 11]] - pb[[3, 7, 11]]).max(), "drot %.2e" % ang)
