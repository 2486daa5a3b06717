import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn
from oracle import pforacle as orc
N, M, B = 4099, 5, 50
cfg = syn.StreamConfig("t", M=M, B=B, N=N)
st = syn.make_stream(cfg, 3)
for rep in range(3):
    eng = pf.Engine(0, N, state_dtype=pf.STATE_F64)
    eng.set_model(st.markers, st.K); prm = pf.default_params(); prm.rng_mode = pf.RNG_REFERENCE; eng.set_params(prm)
    eng.set_prior(st.prior())
    prior = st.prior()
    for fr in st.frames:
        out = eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=fr.blobs, dt=fr.dt, seed=1000 + fr.index, frame_idx=fr.index)).as_dict()
        ref, arr = orc.pf_step(st.markers, st.K, orc.make_params(rng_mode=0), prior, fr.current_pose, fr.predicted_pose, fr.prediction, fr.blobs, dt=fr.dt, seed=1000 + fr.index, frame_idx=fr.index)
        proj = np.array([orc.project(st.K, out["winner_pose"], X) for X in st.markers])
        _, pairs_from_pose = orc.likelihood(proj, fr.blobs, 5.0, 4.0)
        print(rep, fr.index, "win", out["winner_idx"], ref["winner_idx"], "pose_eq", np.abs(out["winner_pose"]-ref["winner_pose"]).max(),
              "gpu", out["pairs"].tolist(), "ref", ref["pairs"].tolist(), "from_gpu_pose", pairs_from_pose.tolist())
        prior = arr["resampled"]
    eng.close()
