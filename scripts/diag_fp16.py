"""fp16 vs fp32 state on one C2-shaped stream: raw winner and GN-refined translation error vs truth."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn
from oracle import pforacle as orc
N = 50_000
cfg = syn.StreamConfig("t", M=5, B=50, N=N)
st = syn.make_stream(cfg, 30)
for name, state in (("f32", pf.STATE_F32), ("f16", pf.STATE_F16)):
    eng = pf.Engine(0, N, state_dtype=state)
    eng.set_model(st.markers, st.K); eng.set_params(pf.default_params()); eng.set_prior(st.prior())
    raw, gn = [], []
    for fr in st.frames:
        out = eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=fr.blobs, dt=fr.dt,
                                      seed=3 + fr.index, frame_idx=fr.index)).as_dict()
        T = np.asarray(out["winner_pose"]).reshape(3, 4)
        raw.append(np.abs(T[:, 3] - fr.truth[:3, 3]).max())
        pg, _, _ = orc.optimise_pose(st.markers, st.K, fr.blobs, out["pairs"], out["winner_pose"])
        gn.append(np.abs(syn.to44(pg)[:3, 3] - fr.truth[:3, 3]).max())
    print(name, "raw max %.4f median %.4f | GN max %.5f median %.5f" % (max(raw), np.median(raw), max(gn), np.median(gn)))
    eng.close()
