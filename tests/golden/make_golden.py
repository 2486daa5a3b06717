#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (inputs + expected outputs, .npz).

The reference cannot be built or run here (Eigen/OpenCV/ROS absent; it ships no tests or fixtures,
SURVEY.md §8c), so the expected outputs come from the CPU restatement oracle/pf_oracle.cpp, itself pinned
by the known-answer tests in tests/test_oracle_kat.py.  The fixtures freeze that pinned behaviour:
tests/test_golden.py re-derives them from the oracle on CPU (the oracle must not drift) and
tests/test_gpu_golden.py runs them through the HIP engine.

    python tests/golden/make_golden.py        # rewrites the .npz files next to this script
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import pforacle as orc  # noqa: E402
from pf_monocular_pose_estimator_amd import synthetic as syn  # noqa: E402

OUT_KEYS_I = ("iters", "kept_iter", "accepted", "resampled", "most_likely_idx", "winner_idx", "n_corr", "flag_fail")
OUT_KEYS_F = ("highest_prob", "prob_sum")


def likelihood_vectors(n_cases=300, seed=20261015):
    """Random projections/blobs around the gate, with duplicates, downgrades, B < M and B = 0 cases."""
    rng = np.random.default_rng(seed)
    rows = {"M": [], "B": [], "tol": [], "tol_pf": [], "proj": [], "blobs": [], "downgrade": [], "P": [],
            "npairs": [], "pairs": []}
    for c in range(n_cases):
        M = int(rng.integers(1, 13))
        B = int(rng.integers(0, 30)) if c % 7 else int(rng.integers(0, M + 1))
        tol, tol_pf = (5.0, 4.0) if c % 3 else (5.0, float(rng.choice([2.0, 4.0, 10.0])))
        proj = rng.uniform(0, 200, size=(M, 2))
        blobs = rng.uniform(0, 200, size=(B, 2))
        for i in range(min(B, M)):  # some blobs near projections, some shared
            if rng.random() < 0.7:
                j = int(rng.integers(0, M))
                blobs[i] = proj[j] + rng.normal(0, 2.0, size=2)
        dg = (rng.random(M) < 0.2).astype(np.uint8)
        P, pairs = orc.likelihood(proj, blobs, tol, tol_pf, dg)
        rows["M"].append(M); rows["B"].append(B); rows["tol"].append(tol); rows["tol_pf"].append(tol_pf)
        rows["proj"].append(np.pad(proj, ((0, 12 - M), (0, 0))))
        rows["blobs"].append(np.pad(blobs, ((0, 30 - B), (0, 0))))
        rows["downgrade"].append(np.pad(dg, (0, 12 - M)))
        rows["P"].append(P)
        rows["npairs"].append(len(pairs))
        rows["pairs"].append(np.pad(pairs, ((0, 12 - len(pairs)), (0, 0))).astype(np.uint32))
    return {k: np.array(v) for k, v in rows.items()}


def stream_fixture(name, M, B, N, heavy, n_frames, rng_mode, seed_base):
    cfg = syn.StreamConfig(name, M=M, B=B, N=N, heavy=heavy)
    st = syn.make_stream(cfg, n_frames)
    prior0 = st.prior()
    prm = orc.make_params(rng_mode=rng_mode)
    fx = {"markers": st.markers, "K": st.K, "prior0": prior0, "rng_mode": rng_mode,
          "cur": [], "pred": [], "predm": [], "dt": [], "seed": [], "frame_idx": [], "B": [], "blobs": [],
          "counts": [], "pairs": [], "winner_pose": [], "most_likely_pose": [], "weights": []}
    for k in OUT_KEYS_I + OUT_KEYS_F:
        fx[k] = []
    maxB = max(len(f.blobs) for f in st.frames)
    prior = prior0
    for f in st.frames:
        seed = seed_base + f.index
        out, arr = orc.pf_step(st.markers, st.K, prm, prior, f.current_pose, f.predicted_pose, f.prediction, f.blobs,
                               dt=f.dt, seed=seed, frame_idx=f.index)
        fx["cur"].append(f.current_pose); fx["pred"].append(f.predicted_pose); fx["predm"].append(f.prediction)
        fx["dt"].append(f.dt); fx["seed"].append(seed); fx["frame_idx"].append(f.index); fx["B"].append(len(f.blobs))
        fx["blobs"].append(np.pad(f.blobs, ((0, maxB - len(f.blobs)), (0, 0))))
        for k in OUT_KEYS_I + OUT_KEYS_F:
            fx[k].append(out[k])
        fx["pairs"].append(np.pad(out["pairs"], ((0, 16 - len(out["pairs"])), (0, 0))).astype(np.uint32))
        fx["winner_pose"].append(out["winner_pose"]); fx["most_likely_pose"].append(out["most_likely_pose"])
        fx["counts"].append(arr["counts"].astype(np.uint32))
        fx["weights"].append(arr["weights"])
        if out["resampled"]:
            prior = arr["resampled"]
    fx["final_prior"] = prior
    return {k: np.asarray(v) for k, v in fx.items()}


FIXTURES = {
    # C1 (BASELINE.json configs[0]): 5 LEDs, 20 blobs, 1000 particles, both RNG streams
    "pf_c1_reference_rng": dict(name="C1", M=5, B=20, N=1000, heavy=False, n_frames=4, rng_mode=orc.RNG_REFERENCE,
                                seed_base=101),
    "pf_c1_philox": dict(name="C1", M=5, B=20, N=1000, heavy=False, n_frames=4, rng_mode=orc.RNG_PHILOX,
                         seed_base=202),
    # C3 shape, small N: 12 LEDs, 200 blobs with heavy near/far outliers and an occluded LED
    "pf_m12_heavy_philox": dict(name="C3", M=12, B=200, N=257, heavy=True, n_frames=3, rng_mode=orc.RNG_PHILOX,
                                seed_base=303),
}


def main():
    np.savez_compressed(os.path.join(HERE, "likelihood_vectors.npz"), **likelihood_vectors())
    for name, kw in FIXTURES.items():
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **stream_fixture(**kw))
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)), "bytes")


if __name__ == "__main__":
    main()
