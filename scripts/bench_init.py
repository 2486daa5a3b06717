"""Benchmark of the brute-force P3P (re)initialisation (PE:1503-1786).

Prints one JSON line: the histogram stage (k_p3p_hist, the hot part: C(B,3) x P(M,3) P3P solves) at a
given (M, B) — device time from HIP events and wall time through the C-ABI — and the whole
pfmpe_initialise on a realistic track-loss frame, each beside the CPU oracle (oracle/init_oracle.cpp,
the reference's algorithm restated, 1 thread).
"""
import argparse
import json
import os
import sys
import time
from math import comb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import pf_monocular_pose_estimator_amd as pf  # noqa: E402
from pf_monocular_pose_estimator_amd import synthetic as syn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=5)
    ap.add_argument("--B", type=int, default=50)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cpu", type=int, default=1, help="time the CPU oracle too (0 = skip)")
    a = ap.parse_args()
    M, B = a.M, a.B
    blobs, _ = syn.init_blobs(M, B - M, seed=2, noise_px=0.3)
    eng = pf.Engine(device=0, max_particles=1000, state_dtype=pf.STATE_F64)
    eng.set_model(syn.markers_for(M), syn.K_README)
    eng.set_params(pf.default_params())
    for _ in range(2):
        eng.p3p_histogram(blobs)
    eng.set_option(pf.OPT_TIMING, 1)
    eng.reset_kernel_stats()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        h = eng.p3p_histogram(blobs)
    wall = (time.perf_counter() - t0) / a.reps
    n, ms = eng.kernel_stats()["k_p3p_hist"]
    dev = ms / max(n, 1) / 1e3
    items = comb(B, 3) * M * (M - 1) * (M - 2)
    res = {"metric": "P3P initialisation histogram: (3-blob combination x ordered 3-marker) P3P solves/s",
           "value": items / dev, "unit": "P3P solves/s", "config": {"M": M, "B": B, "items": items},
           "k_p3p_hist_us": dev * 1e6, "wall_us": wall * 1e6, "hist_total": int(h.sum()), "dtype": "f64"}
    # full initialise on a realistic frame (all markers + 3 outliers)
    fb, _ = syn.init_blobs(M, 3, seed=0)
    eng.reset_kernel_stats()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        out, _ = eng.initialise(fb, n_particles=1000)
    res["initialise_wall_us"] = (time.perf_counter() - t0) / a.reps * 1e6
    res["initialise_found"] = out["found"]
    if a.cpu:
        from oracle import pforacle as orc
        t0 = time.perf_counter()
        orc.init_histogram(syn.markers_for(M), syn.K_README, blobs)
        cpu = time.perf_counter() - t0
        t0 = time.perf_counter()
        orc.initialise(syn.markers_for(M), syn.K_README, fb, 1000)
        cpu_init = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": items / cpu, "unit": "P3P solves/s", "cores": 1, "kind": "port",
                               "histogram_s": cpu, "initialise_s": cpu_init,
                               "sample": f"one histogram at M={M}, B={B}; one initialise at M={M}, B={M + 3}"}
    print(json.dumps(res))
    eng.close()


if __name__ == "__main__":
    main()
