"""Per-frame look at the resampling kernel (k_resample_owners vs the block-per-256 k_resample): HIP-event time of
the resampling launch, the frame's iterations, the largest resample count and where it sits, the smallest weight.
  python scripts/diag_owners.py C5 60"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np

import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "C5"
n_frames = int(sys.argv[2]) if len(sys.argv) > 2 else 60
base = syn.CONFIGS[cfg_name]
cfg = syn.StreamConfig(base.name, M=base.M, B=base.B, N=base.N, heavy=base.heavy, seed=0)
st = syn.make_stream(cfg, n_frames)
state = pf.STATE_F16 if cfg_name == "C4" else pf.STATE_F32
res = {}
for diag in (0, pf.DIAG_BLOCK_RESAMPLE):
    eng = pf.Engine(device=0, max_particles=cfg.N, state_dtype=state)
    eng.set_model(st.markers, st.K)
    prm = pf.default_params()
    eng.set_params(prm)
    eng.set_prior(st.prior())
    eng.set_option(pf.OPT_DIAG, diag)
    eng.set_option(pf.OPT_RECORD_COUNTS, 1)
    eng.stage_blob_bank([f.blobs for f in st.frames])
    rows = []
    for f in st.frames:
        fr = eng.make_frame(f.current_pose, f.predicted_pose, f.prediction, B=len(f.blobs), bank_frame=f.index,
                            dt=f.dt, seed=17 + f.index, frame_idx=f.index)
        eng.reset_kernel_stats()
        eng.set_option(pf.OPT_TIMING, 1)
        t0 = time.perf_counter()
        o = eng.step(fr)
        t1 = time.perf_counter()
        eng.set_option(pf.OPT_TIMING, 0)
        ks = eng.kernel_stats()
        c = eng.get_counts() if o.resampled else np.zeros(1, np.int64)
        w = eng.get_weights()
        i = int(np.argmax(c))
        rows.append((f.index, o.iters, (t1 - t0) * 1e6, {k: round(v[1] * 1e3 / max(v[0], 1), 1) for k, v in ks.items() if v[0]},
                     int(c.max()), i, i // 256, float(w.min()), int((c > 64).sum())))
    eng.close()
    res[diag] = rows
for a, b in zip(res[0], res[pf.DIAG_BLOCK_RESAMPLE]):
    print(f"frame {a[0]:3d} it {a[1]:2d} | new {a[2]:7.1f} us {a[3].get('k_resample', 0):7.1f} | old {b[2]:7.1f} us "
          f"{b[3].get('k_resample', 0):7.1f} | maxcount {a[4]} at {a[5]} (block {a[6]}) wmin {a[7]:.3f} n>64 {a[8]}")
