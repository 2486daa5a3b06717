"""ctypes binding of the CPU oracle (oracle/pf_oracle.cpp) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and only as
the checker / the timed CPU baseline.  The product (pf_monocular_pose_estimator_amd) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "libpforacle.so")

RNG_REFERENCE, RNG_PHILOX = 0, 1


class OrcParams(C.Structure):
    _fields_ = [
        ("tol", C.c_double), ("tol_pf", C.c_double),
        ("ang_min", C.c_double), ("ang_max", C.c_double),
        ("trans_min", C.c_double), ("trans_max", C.c_double),
        ("growth", C.c_double),
        ("max_iter", C.c_int), ("exit_cap", C.c_int), ("accept_cap", C.c_int), ("rng_mode", C.c_int),
        ("fast_search", C.c_int),
    ]


class OrcFrameIn(C.Structure):
    _fields_ = [
        ("current_pose", C.c_double * 12), ("predicted_pose", C.c_double * 12),
        ("prediction", C.c_double * 12), ("cam_move_inv", C.c_double * 12),
        ("blobs", C.POINTER(C.c_double)), ("B", C.c_int), ("it_since_init", C.c_int),
        ("dt", C.c_double), ("seed", C.c_uint64), ("frame_idx", C.c_uint64), ("force_iters", C.c_int),
    ]


class OrcFrameOut(C.Structure):
    _fields_ = [
        ("iters", C.c_int), ("kept_iter", C.c_int), ("most_likely_idx", C.c_int), ("accepted", C.c_int),
        ("resampled", C.c_int), ("winner_idx", C.c_int), ("n_corr", C.c_int), ("flag_fail", C.c_int),
        ("highest_prob", C.c_double), ("prob_sum", C.c_double),
        ("winner_pose", C.c_double * 12), ("most_likely_pose", C.c_double * 12),
        ("corr", C.c_uint * 64),
    ]

    def as_dict(self) -> dict:
        return {
            "iters": self.iters, "kept_iter": self.kept_iter, "most_likely_idx": self.most_likely_idx,
            "accepted": self.accepted, "resampled": self.resampled, "winner_idx": self.winner_idx,
            "n_corr": self.n_corr, "flag_fail": self.flag_fail, "highest_prob": self.highest_prob,
            "prob_sum": self.prob_sum, "winner_pose": np.array(self.winner_pose),
            "most_likely_pose": np.array(self.most_likely_pose),
            "pairs": np.array(self.corr[: 2 * self.n_corr], dtype=np.uint32).reshape(-1, 2),
        }


class OrcInitParams(C.Structure):
    _fields_ = [("tol", C.c_double), ("certainty_threshold", C.c_double), ("valid_corr_threshold", C.c_double),
                ("use_pf", C.c_int), ("max_candidates", C.c_int)]


class OrcInitOut(C.Structure):
    _fields_ = [("found", C.c_int), ("flag_fail", C.c_int), ("n_estimates", C.c_int), ("n_candidates", C.c_int),
                ("first_match", C.c_int), ("n_corr", C.c_int), ("corr", C.c_uint32 * 32),
                ("predicted_pose", C.c_double * 12), ("hist_total", C.c_uint64)]

    def as_dict(self) -> dict:
        return {"found": self.found, "flag_fail": self.flag_fail, "n_estimates": self.n_estimates,
                "n_candidates": self.n_candidates, "first_match": self.first_match,
                "pairs": np.array(self.corr[: 2 * self.n_corr], dtype=np.uint32).reshape(-1, 2),
                "predicted_pose": np.array(self.predicted_pose), "hist_total": self.hist_total}


class OrcDetectParams(C.Structure):
    _fields_ = [("threshold_value", C.c_int), ("gaussian_sigma", C.c_double), ("min_blob_area", C.c_double),
                ("max_blob_area", C.c_double), ("max_width_height_distortion", C.c_double),
                ("max_circular_distortion", C.c_double), ("active_markers", C.c_int), ("roi_x", C.c_int),
                ("roi_y", C.c_int), ("roi_w", C.c_int), ("roi_h", C.c_int)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    dp = C.POINTER(C.c_double)
    up = C.POINTER(C.c_uint)
    u8p = C.POINTER(C.c_uint8)
    lib.orc_likelihood.restype = C.c_double
    lib.orc_likelihood.argtypes = [C.c_int, C.c_int, dp, dp, C.c_double, C.c_double, u8p, up, C.POINTER(C.c_int)]
    lib.orc_likelihood_closed.restype = C.c_double
    lib.orc_likelihood_closed.argtypes = lib.orc_likelihood.argtypes
    lib.orc_project.restype = None
    lib.orc_project.argtypes = [dp, dp, dp, dp]
    lib.orc_philox4x32_10.restype = None
    lib.orc_philox4x32_10.argtypes = [C.POINTER(C.c_uint32)] * 3
    lib.orc_minstd_outputs.restype = None
    lib.orc_minstd_outputs.argtypes = [C.c_uint32, C.c_int, C.POINTER(C.c_uint32)]
    lib.orc_uniform_draws.restype = None
    lib.orc_uniform_draws.argtypes = [C.c_uint32, C.c_double, C.c_double, C.c_int, dp]
    lib.orc_pf_step.restype = C.c_int
    lib.orc_pf_step.argtypes = [C.c_int, C.c_int, dp, dp, u8p, C.POINTER(OrcParams), C.POINTER(OrcFrameIn), dp,
                                C.POINTER(OrcFrameOut), dp, dp, dp, C.POINTER(C.c_int), up]
    lib.orc_stratified_resample.restype = C.c_int
    lib.orc_pf_sample.argtypes = [C.c_int, C.POINTER(C.c_int), C.c_int, dp, dp, u8p, C.POINTER(OrcParams),
                                  C.POINTER(OrcFrameIn), C.c_int, dp, dp, dp]
    lib.orc_pf_sample.restype = C.c_int
    lib.orc_stratified_resample.argtypes = [C.c_int, dp, C.c_int, C.c_uint64, C.c_uint64, C.c_int, up,
                                            C.POINTER(C.c_int)]
    lib.orc_exp_map.restype = None
    lib.orc_exp_map.argtypes = [dp, dp]
    lib.orc_log_map.restype = None
    lib.orc_log_map.argtypes = [dp, dp]
    lib.orc_predict_pose.restype = None
    lib.orc_predict_pose.argtypes = [dp, dp, C.c_double, C.c_double, C.c_double, dp, dp]
    lib.orc_optimise_pose.restype = C.c_int
    lib.orc_optimise_pose.argtypes = [C.c_int, dp, dp, C.c_int, dp, up, C.c_int, dp, dp, dp]
    lib.orc_predict_roi.restype = C.c_int
    lib.orc_predict_roi.argtypes = [C.c_int, C.c_int, dp, dp, dp, dp, dp, dp, dp, C.c_int, C.c_int, C.c_int,
                                    C.POINTER(C.c_int), dp]
    u32p = C.POINTER(C.c_uint32)
    lib.orc_image_vectors.restype = C.c_int
    lib.orc_image_vectors.argtypes = [dp, C.c_int, dp, dp]
    lib.orc_p3p.restype = C.c_int
    lib.orc_p3p.argtypes = [dp, dp, dp]
    lib.orc_inverse44.restype = None
    lib.orc_inverse44.argtypes = [dp, dp]
    lib.orc_init_histogram.restype = C.c_int
    lib.orc_init_histogram.argtypes = [C.c_int, dp, dp, C.c_int, dp, C.c_double, u32p]
    lib.orc_init_histogram_bounds.restype = C.c_int
    lib.orc_init_histogram_bounds.argtypes = [C.c_int, dp, dp, C.c_int, dp, C.c_double, u32p, u32p, u32p,
                                              C.POINTER(C.c_int)]
    lib.orc_find_leds.restype = C.c_int
    lib.orc_find_leds.argtypes = [C.POINTER(C.c_uint8), C.c_int, C.c_int, C.c_int, C.POINTER(OrcDetectParams), dp, dp,
                                  C.c_int, C.POINTER(C.c_float), dp, dp, C.POINTER(C.c_uint8)]
    lib.orc_initialise.restype = C.c_int
    lib.orc_initialise.argtypes = [C.c_int, dp, dp, C.c_int, dp, C.POINTER(OrcInitParams), C.c_int, u32p, u32p,
                                   dp, C.POINTER(OrcInitOut)]
    _lib = lib
    return lib


def _d(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _p(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def likelihood(proj, blobs, tol, tol_pf, downgrade=None, closed=False):
    lib = load()
    proj = _d(proj).reshape(-1, 2)
    blobs = _d(blobs).reshape(-1, 2)
    M, B = proj.shape[0], blobs.shape[0]
    pairs = np.zeros(2 * max(M, 1), dtype=np.uint32)
    n = C.c_int()
    dg = None
    if downgrade is not None:
        dga = np.ascontiguousarray(downgrade, dtype=np.uint8)
        dg = dga.ctypes.data_as(C.POINTER(C.c_uint8))
    fn = lib.orc_likelihood_closed if closed else lib.orc_likelihood
    P = fn(M, B, _p(proj), _p(blobs) if B else C.POINTER(C.c_double)(), tol, tol_pf, dg,
           pairs.ctypes.data_as(C.POINTER(C.c_uint)), C.byref(n))
    return P, pairs[: 2 * n.value].reshape(-1, 2)


def project(K, pose12, X):
    out = np.zeros(2)
    load().orc_project(_p(_d(K).reshape(9)), _p(_d(pose12).reshape(12)), _p(_d(X).reshape(3)), _p(out))
    return out


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    load().orc_philox4x32_10(c, k, o)
    return list(o)


def minstd_outputs(seed, n):
    o = (C.c_uint32 * n)()
    load().orc_minstd_outputs(seed, n, o)
    return list(o)


def uniform_draws(seed, a, b, n):
    o = np.zeros(n)
    load().orc_uniform_draws(seed, a, b, n, _p(o))
    return o


def make_params(tol=5.0, tol_pf=4.0, ang=(-0.015, 0.015), trans=(-0.035, 0.035), growth=0.025,
                max_iter=80, exit_cap=5, accept_cap=3, rng_mode=RNG_PHILOX, fast_search=0) -> OrcParams:
    """fast_search=1: the resampler's cumulative search by binary search (identical results, O(N log N);
    for long closed-loop tests at 100k particles).  0 keeps the reference's O(N^2) scan (cpu_baseline)."""
    return OrcParams(tol, tol_pf, ang[0], ang[1], trans[0], trans[1], growth, max_iter, exit_cap, accept_cap,
                     rng_mode, fast_search)


def pf_step(markers, K, params: OrcParams, prior, current_pose, predicted_pose, prediction, blobs,
            it_since_init=2, dt=0.02, seed=1, frame_idx=0, force_iters=0, cam_move_inv=None, downgrade=None,
            want_arrays=True):
    """One reference PF step.  Returns (out_dict, arrays) where arrays holds propagated / weights /
    resampled / resample_idx / counts (None if want_arrays is False)."""
    lib = load()
    m = _d(markers).reshape(-1, 3)
    M = m.shape[0]
    prior = _d(prior).reshape(-1, 12)
    N = prior.shape[0]
    b = _d(blobs).reshape(-1, 2)
    fi = OrcFrameIn()
    fi.current_pose[:] = list(_d(current_pose).reshape(12))
    fi.predicted_pose[:] = list(_d(predicted_pose).reshape(12))
    fi.prediction[:] = list(_d(prediction).reshape(12))
    fi.cam_move_inv[:] = list(np.eye(4)[:3].reshape(12) if cam_move_inv is None else _d(cam_move_inv).reshape(12))
    fi.blobs = _p(b)
    fi.B = b.shape[0]
    fi.it_since_init = it_since_init
    fi.dt = dt
    fi.seed = seed
    fi.frame_idx = frame_idx
    fi.force_iters = force_iters
    out = OrcFrameOut()
    dg = None
    if downgrade is not None:
        dga = np.ascontiguousarray(downgrade, dtype=np.uint8)
        dg = dga.ctypes.data_as(C.POINTER(C.c_uint8))
    arrays = None
    null_d = C.POINTER(C.c_double)()
    if want_arrays:
        arrays = {
            "propagated": np.zeros((N, 12)), "weights": np.zeros(N), "resampled": np.zeros((N, 12)),
            "resample_idx": np.full(N, -1, dtype=np.int32), "counts": np.zeros(N, dtype=np.uint32),
        }
        rc = lib.orc_pf_step(N, M, _p(m), _p(_d(K).reshape(9)), dg, C.byref(params), C.byref(fi), _p(prior),
                             C.byref(out), _p(arrays["propagated"]), _p(arrays["weights"]),
                             _p(arrays["resampled"]), arrays["resample_idx"].ctypes.data_as(C.POINTER(C.c_int)),
                             arrays["counts"].ctypes.data_as(C.POINTER(C.c_uint)))
    else:
        rc = lib.orc_pf_step(N, M, _p(m), _p(_d(K).reshape(9)), dg, C.byref(params), C.byref(fi), _p(prior),
                             C.byref(out), null_d, null_d, null_d, C.POINTER(C.c_int)(), C.POINTER(C.c_uint)())
    if rc != 0:
        raise RuntimeError(f"orc_pf_step failed: {rc}")
    return out.as_dict(), arrays


def pf_sample(markers, K, params: OrcParams, idx, prior_rows, current_pose, predicted_pose, prediction, blobs, iter_,
              it_since_init=2, dt=0.02, seed=1, frame_idx=0, cam_move_inv=None, downgrade=None):
    """Particles idx of PF iteration iter_ alone (Philox stream), each from its prior pose prior_rows[s]:
    (propagated poses, literal weights) of orc_pf_sample."""
    lib = load()
    m = _d(markers).reshape(-1, 3)
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    pr = _d(prior_rows).reshape(-1, 12)
    assert pr.shape[0] == idx.shape[0]
    b = _d(blobs).reshape(-1, 2)
    fi = OrcFrameIn()
    fi.current_pose[:] = list(_d(current_pose).reshape(12))
    fi.predicted_pose[:] = list(_d(predicted_pose).reshape(12))
    fi.prediction[:] = list(_d(prediction).reshape(12))
    fi.cam_move_inv[:] = list(np.eye(4)[:3].reshape(12) if cam_move_inv is None else _d(cam_move_inv).reshape(12))
    fi.blobs = _p(b)
    fi.B = b.shape[0]
    fi.it_since_init = it_since_init
    fi.dt = dt
    fi.seed = seed
    fi.frame_idx = frame_idx
    dg = None
    if downgrade is not None:
        dga = np.ascontiguousarray(downgrade, dtype=np.uint8)
        dg = dga.ctypes.data_as(C.POINTER(C.c_uint8))
    prop = np.zeros((idx.shape[0], 12))
    w = np.zeros(idx.shape[0])
    rc = lib.orc_pf_sample(int(idx.shape[0]), idx.ctypes.data_as(C.POINTER(C.c_int)), m.shape[0], _p(m),
                           _p(_d(K).reshape(9)), dg, C.byref(params), C.byref(fi), int(iter_), _p(pr), _p(prop), _p(w))
    if rc != 0:
        raise RuntimeError(f"orc_pf_sample failed: {rc}")
    return prop, w


def stratified_resample(weights, rng_mode, seed, frame_idx, iters):
    """PE:627-682 alone on the given raw weights -> (counts, idx)."""
    w = _d(weights)
    N = w.size
    counts = np.zeros(N, dtype=np.uint32)
    idx = np.zeros(N, dtype=np.int32)
    load().orc_stratified_resample(N, _p(w), rng_mode, seed, frame_idx, iters,
                                   counts.ctypes.data_as(C.POINTER(C.c_uint)), idx.ctypes.data_as(C.POINTER(C.c_int)))
    return counts, idx


def exp_map(twist):
    out = np.zeros(12)
    load().orc_exp_map(_p(_d(twist)), _p(out))
    return out


def log_map(pose12):
    out = np.zeros(6)
    load().orc_log_map(_p(_d(pose12).reshape(12)), _p(out))
    return out


def predict_pose(prev12, cur12, t_prev, t_cur, t_pred):
    pm = np.zeros(12)
    pp = np.zeros(12)
    load().orc_predict_pose(_p(_d(prev12).reshape(12)), _p(_d(cur12).reshape(12)), t_prev, t_cur, t_pred,
                            _p(pm), _p(pp))
    return pm, pp


def optimise_pose(markers, K, blobs, pairs, pose12):
    m = _d(markers).reshape(-1, 3)
    b = _d(blobs).reshape(-1, 2)
    pr = np.ascontiguousarray(pairs, dtype=np.uint32).reshape(-1)
    out = np.zeros(12)
    cov = np.zeros(36)
    it = load().orc_optimise_pose(m.shape[0], _p(m), _p(_d(K).reshape(9)), b.shape[0], _p(b),
                                  pr.ctypes.data_as(C.POINTER(C.c_uint)), pr.size // 2, _p(_d(pose12).reshape(12)),
                                  _p(out), _p(cov))
    return out, cov.reshape(6, 6), it


def predict_roi(markers, K, D, prior, cam_move_inv, prediction, predicted_pose, image_w, image_h, border):
    """predictMarkerPositionsInImage + determineROI (PE:1036-1053, led_detector.cpp:217-414) ->
    (roi [x, y, w, h], bbox [x_min, x_max, y_min, y_max])."""
    m = _d(markers).reshape(-1, 3)
    pr = _d(prior).reshape(-1, 12)
    roi = (C.c_int * 4)()
    bbox = np.zeros(4)
    load().orc_predict_roi(pr.shape[0], m.shape[0], _p(m), _p(_d(K).reshape(9)), _p(_d(D).reshape(5)), _p(pr),
                           _p(_d(cam_move_inv).reshape(12)), _p(_d(prediction).reshape(12)),
                           _p(_d(predicted_pose).reshape(12)), image_w, image_h, border, roi, _p(bbox))
    return list(roi), bbox


# ------------------------------------------------------------------ brute-force P3P initialisation
def image_vectors(K, blobs):
    b = _d(blobs).reshape(-1, 2)
    out = np.zeros((b.shape[0], 3))
    load().orc_image_vectors(_p(_d(K).reshape(9)), b.shape[0], _p(b), _p(out))
    return out


def p3p(feature_vectors, world_points):
    """P3P::computePoses on rows = the three unit feature vectors / world points -> (rc, 4 x 12)."""
    sol = np.zeros((4, 12))
    rc = load().orc_p3p(_p(_d(feature_vectors).reshape(9)), _p(_d(world_points).reshape(9)), _p(sol))
    return rc, sol


def inverse44(sol12):
    out = np.zeros(16)
    load().orc_inverse44(_p(_d(sol12).reshape(12)), _p(out))
    return out.reshape(4, 4)


def init_histogram(markers, K, blobs, tol=5.0):
    m = _d(markers).reshape(-1, 3)
    b = _d(blobs).reshape(-1, 2)
    h = np.zeros((b.shape[0], m.shape[0]), dtype=np.uint32)
    rc = load().orc_init_histogram(m.shape[0], _p(m), _p(_d(K).reshape(9)), b.shape[0], _p(b), tol,
                                   h.ctypes.data_as(C.POINTER(C.c_uint32)))
    if rc != 0:
        raise ValueError("orc_init_histogram: bad sizes")
    return h


def init_histogram_bounds(markers, K, blobs, tol=5.0):
    """(hist, lo, hi, unbounded): the reference histogram and the band any ulp-level reimplementation must
    land in (fragile decisions: repeated-solution skip between near-equal roots, the tol gate, ties)."""
    m = _d(markers).reshape(-1, 3)
    b = _d(blobs).reshape(-1, 2)
    hs = [np.zeros((b.shape[0], m.shape[0]), dtype=np.uint32) for _ in range(3)]
    ub = C.c_int()
    u32 = C.POINTER(C.c_uint32)
    rc = load().orc_init_histogram_bounds(m.shape[0], _p(m), _p(_d(K).reshape(9)), b.shape[0], _p(b), tol,
                                          *[h.ctypes.data_as(u32) for h in hs], C.byref(ub))
    if rc != 0:
        raise ValueError("orc_init_histogram_bounds: bad sizes")
    return hs[0], hs[1], hs[2], ub.value


def initialise(markers, K, blobs, n_particles, particles=None, tol=5.0, certainty_threshold=1.0,
               valid_corr_threshold=0.5, use_pf=True, max_candidates=65536, hist=None):
    """PoseEstimator::initialise (PE:1503-1786) -> (out dict, hist (B x M), particles (N x 12)).
    `particles` is PoseParticle before the call (default: identity poses); `hist` overrides the
    histogram stage."""
    m = _d(markers).reshape(-1, 3)
    b = _d(blobs).reshape(-1, 2)
    M, B = m.shape[0], b.shape[0]
    if particles is None:
        particles = np.tile(np.eye(4)[:3].reshape(12), (n_particles, 1))
    pp = np.array(_d(particles).reshape(n_particles, 12))
    hout = np.zeros((B, M), dtype=np.uint32)
    hin = None
    if hist is not None:
        hin = np.ascontiguousarray(hist, dtype=np.uint32).reshape(B, M)
    prm = OrcInitParams(tol, certainty_threshold, valid_corr_threshold, 1 if use_pf else 0, max_candidates)
    out = OrcInitOut()
    u32 = C.POINTER(C.c_uint32)
    rc = load().orc_initialise(M, _p(m), _p(_d(K).reshape(9)), B, _p(b), C.byref(prm), n_particles,
                               hin.ctypes.data_as(u32) if hin is not None else u32(), hout.ctypes.data_as(u32),
                               _p(pp), C.byref(out))
    if rc != 0:
        raise RuntimeError(f"orc_initialise failed: {rc}")
    return out.as_dict(), hout, pp


# ------------------------------------------------------------------ LED detector (LEDDetector::findLeds)
def find_leds(image, K, D, threshold_value=240, gaussian_sigma=0.6, min_blob_area=20, max_blob_area=160,
              max_width_height_distortion=0.7, max_circular_distortion=0.7, active_markers=True, roi=None,
              max_out=1024, want_mask=False):
    """-> (undistorted B x 2, distorted B x 2 float32, areas B, mask or None)."""
    img = np.ascontiguousarray(image, dtype=np.uint8)
    h, w = img.shape
    rx, ry, rw, rh = roi if roi is not None else (0, 0, w, h)
    prm = OrcDetectParams(threshold_value, gaussian_sigma, min_blob_area, max_blob_area, max_width_height_distortion,
                          max_circular_distortion, 1 if active_markers else 0, rx, ry, rw, rh)
    und = np.zeros((max_out, 2))
    dist = np.zeros((max_out, 2), dtype=np.float32)
    areas = np.zeros(max_out)
    mask = np.zeros((rh, rw), dtype=np.uint8) if want_mask else None
    n = load().orc_find_leds(img.ctypes.data_as(C.POINTER(C.c_uint8)), w, h, img.strides[0], C.byref(prm),
                             _p(_d(K).reshape(9)), _p(_d(D).reshape(5)), max_out,
                             dist.ctypes.data_as(C.POINTER(C.c_float)), _p(und), _p(areas),
                             mask.ctypes.data_as(C.POINTER(C.c_uint8)) if want_mask else None)
    if n < 0:
        raise ValueError("orc_find_leds: bad arguments")
    n = min(n, max_out)
    return und[:n], dist[:n], areas[:n], mask
