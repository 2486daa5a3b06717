"""Diagnostic: where do fp32 weights / counts differ from the fp64 oracle?"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn
from oracle import pforacle as orc

for (N, M, B, heavy) in [(20000, 5, 50, False), (8192, 12, 200, True)]:
    cfg = syn.StreamConfig("t", M=M, B=B, N=N, heavy=heavy)
    st = syn.make_stream(cfg, 2)
    for state in (pf.STATE_F32, pf.STATE_F64):
        eng = pf.Engine(0, N, state_dtype=state)
        eng.set_model(st.markers, st.K); prm = pf.default_params(); eng.set_params(prm)
        eng.set_option(pf.OPT_RECORD_COUNTS, 1)
        eng.set_prior(st.prior())
        for fr in st.frames:
            pr = eng.get_particles(1)
            out = eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=fr.blobs, dt=fr.dt, seed=50+fr.index, frame_idx=fr.index)).as_dict()
            w = eng.get_weights(); c = eng.get_counts().astype(int); prop = eng.get_particles(0)
            ref, arr = orc.pf_step(st.markers, st.K, orc.make_params(), pr, fr.current_pose, fr.predicted_pose, fr.prediction, fr.blobs, dt=fr.dt, seed=50+fr.index, frame_idx=fr.index)
            dw = np.abs(w - arr["weights"])
            big = np.where(dw > 1e-3)[0]
            cm = np.where(c != arr["counts"])[0]
            print(f"N={N} M={M} B={B} state={state} frame={fr.index}: S gpu={out['prob_sum']:.6f} ref={ref['prob_sum']:.6f} maxdw={dw.max():.3e} n(dw>1e-3)={len(big)} "
                  f"count_mismatch={len(cm)} first={cm[:5]} win={out['winner_idx']}/{ref['winner_idx']}")
            for i in big[:5]:
                print("   idx", i, "gpu", w[i], "ref", arr["weights"][i], "dpose", np.abs(prop[i]-arr["propagated"][i]).max())
            if len(cm):
                i0 = cm[0]
                cs_g = np.cumsum(w)/w.sum(); cs_r = np.cumsum(arr["weights"])/arr["weights"].sum()
                print("   cumsum diff at first mismatch", cs_g[i0]-cs_r[i0], "max cumsum diff", np.abs(cs_g-cs_r).max(), "1/N", 1/N)
        eng.close()
