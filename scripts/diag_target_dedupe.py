"""How many distinct stratified-target cells a resampling wave meets (diagnostic for k_resample_owners).

Particle i of a 256-particle block evaluates F(R_i) at target k_i = floor(R_i N) (count_targets_wave): one Philox
call.  Consecutive particles with the same k_i need the same target numerator, so a wave could evaluate only the
run heads.  This prints, per frame of a synthetic stream, the mean number of 64-lane evaluation passes a block
would need with that de-duplication (against 4 without it).

    python scripts/diag_target_dedupe.py [--config C4] [--frames 8]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pf_monocular_pose_estimator_amd as pf  # noqa: E402
from pf_monocular_pose_estimator_amd import synthetic as syn  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C4")
ap.add_argument("--frames", type=int, default=8)
a = ap.parse_args()
base = syn.CONFIGS[a.config]
state = pf.STATE_F16 if a.config == "C4" else pf.STATE_F32
st = syn.make_stream(syn.StreamConfig(base.name, M=base.M, B=base.B, N=base.N, heavy=base.heavy, seed=0), a.frames)
e = pf.Engine(device=0, max_particles=base.N, state_dtype=state)
e.set_model(st.markers, st.K)
e.set_params(pf.default_params())
e.set_prior(st.prior(fast=True))
N = base.N
for f in st.frames:
    o = e.step(e.make_frame(f.current_pose, f.predicted_pose, f.prediction, blobs=f.blobs, dt=f.dt,
                            seed=17 + f.index, frame_idx=f.index))
    if not o.accepted:
        print(f"frame {f.index}: not resampled")
        continue
    w = e.get_weights()
    c = np.maximum.accumulate(np.cumsum(w) / w.sum())
    k = np.floor(c * N).astype(np.int64)
    nb = (N + 255) // 256
    kp = np.concatenate([[-1], k[:-1]])
    head = k != kp
    head[::256] = True
    hp = np.zeros(nb * 256, bool)
    hp[:N] = head
    heads = hp.reshape(nb, 256).sum(1)
    passes = (heads + 63) // 64
    zero = (w == 0).mean()
    print(f"frame {f.index}: iters {o.iters}, weights 0: {zero:.3f}, heads/block {heads.mean():.1f}, "
          f"passes/block {passes.mean():.2f} (hist {np.bincount(passes, minlength=5)[:5].tolist()})", flush=True)
e.close()
