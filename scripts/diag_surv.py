"""Diagnostic: fraction of particles (and of 64-lane waves) that receive resampling copies in a frame."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn

cfgname = sys.argv[1] if len(sys.argv) > 1 else "C3"
base = syn.CONFIGS[cfgname]
st = syn.make_stream(base, 12)
eng = pf.Engine(0, base.N)
eng.set_model(st.markers, st.K); eng.set_params(pf.default_params()); eng.set_prior(st.prior())
eng.set_option(pf.OPT_RECORD_COUNTS, 1)
for fr in st.frames:
    out = eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=fr.blobs, dt=fr.dt,
                                  seed=3, frame_idx=fr.index))
    cnt = eng.get_counts()
    n = len(cnt) // 64 * 64
    waves = (cnt[:n].reshape(-1, 64) > 0).any(axis=1)
    print(f"frame {fr.index}: iters {out.iters} surviving particles {np.mean(cnt > 0):.3f}  "
          f"waves with a survivor {waves.mean():.3f}  max copies {cnt.max()}")
eng.close()
