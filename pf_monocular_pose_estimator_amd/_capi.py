"""ctypes binding of the C-ABI in include/pfmpe.h (libpfmpe.so, built in-tree by __graft_entry__.build()).

This is the same boundary a reference-side maintainer would bind; it loads ONLY the
HIP-built product library and raises if it is missing — there is no CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpfmpe.so")

MAX_MARKERS = 16
MAX_BLOBS = 1024

OK, E_ARG, E_HIP, E_CAP, E_STATE = 0, -1, -2, -3, -4
STATE_F32, STATE_F64, STATE_F16 = 0, 1, 2
RNG_REFERENCE, RNG_PHILOX = 0, 1
FLAG_ACCEPTED, FLAG_REINIT = 1, 4
OPT_RECORD_COUNTS, OPT_PRUNE, OPT_TIMING, OPT_FUSED, OPT_KEEP_PROPAGATED = 1, 2, 3, 4, 5
OPT_WAIT_BOUND_US, OPT_FUSED_REARM, OPT_MULTI_MAX_BLOCKS = 6, 7, 8
OPT_DIAG = 99  # undocumented diagnostic switches (csrc/pf_kernels.hpp kDiag*)
DIAG_LAG_LOADS, DIAG_ABANDON, DIAG_NO_STREAM, DIAG_FORCE_STREAM, DIAG_SERIAL_TOP = 64, 128, 512, 1024, 2048
DIAG_NO_PK, DIAG_CORRUPT_DESC, DIAG_NO_DEFER, DIAG_BLOCK_RESAMPLE, DIAG_MIN_SIDE = 4096, 8192, 16384, 32768, 65536
DIAG_ABANDON_FINISH = 131072
OPT_DEFER_RESAMPLE = 9
SHAPE_TWO_LAUNCH, SHAPE_FRAME, SHAPE_FRAME2 = 0, 1, 2
INFO_FUSED, INFO_FUSED_FALLBACKS, INFO_LAST_SHAPE, INFO_GUARD_SKIPS, INFO_N, INFO_LAST_WEIGH_PASS = 1, 2, 3, 4, 5, 6
INFO_LAST_GRID, INFO_LAST_RESAMPLE = 7, 8
WEIGH_BLOCKS, WEIGH_STREAM, WEIGH_PK = 0, 1, 2
RESAMPLE_BLOCKS, RESAMPLE_OWNERS = 0, 1
K_PROPAGATE, K_RESAMPLE, K_AUX, K_FRAME, K_ROI, K_FINAL, K_P3P_HIST, K_P3P_CHECK, K_DETECT, K_COUNT = range(10)

# every symbol include/pfmpe.h declares (tests check the .so exports all of them)
EXPORTED_SYMBOLS = (
    "pfmpe_create", "pfmpe_destroy", "pfmpe_last_error", "pfmpe_abi_version",
    "pfmpe_set_model", "pfmpe_set_params", "pfmpe_default_params", "pfmpe_set_prior",
    "pfmpe_step", "pfmpe_step_batch", "pfmpe_step_multi", "pfmpe_step_multi_batch", "pfmpe_get_particles", "pfmpe_get_weights", "pfmpe_get_counts",
    "pfmpe_set_option", "pfmpe_stage_blob_bank", "pfmpe_get_kernel_stats",
    "pfmpe_reset_kernel_stats", "pfmpe_kernel_name", "pfmpe_host_ref_uniform", "pfmpe_host_philox",
    "pfmpe_predict_roi", "pfmpe_default_init_params", "pfmpe_p3p_histogram", "pfmpe_initialise",
    "pfmpe_parse_marker_yaml", "pfmpe_default_launch_config", "pfmpe_parse_launch", "pfmpe_parse_camera_info",
    "pfmpe_write_blob_stream", "pfmpe_read_blob_stream", "pfmpe_stage_blob_stream",
    "pfmpe_default_detect_params", "pfmpe_stage_image", "pfmpe_find_leds", "pfmpe_get_info",
)


class Params(C.Structure):
    _fields_ = [
        ("tol", C.c_double), ("tol_pf", C.c_double),
        ("ang_min", C.c_double), ("ang_max", C.c_double),
        ("trans_min", C.c_double), ("trans_max", C.c_double),
        ("growth", C.c_double),
        ("max_iter", C.c_int32), ("exit_cap", C.c_int32), ("accept_cap", C.c_int32),
        ("rng_mode", C.c_int32),
    ]


class FrameIn(C.Structure):
    _fields_ = [
        ("current_pose", C.c_double * 12), ("predicted_pose", C.c_double * 12),
        ("prediction", C.c_double * 12), ("cam_move_inv", C.c_double * 12),
        ("blobs", C.POINTER(C.c_double)), ("B", C.c_int32), ("bank_frame", C.c_int32),
        ("it_since_init", C.c_int32), ("force_iters", C.c_int32),
        ("dt", C.c_double), ("seed", C.c_uint64), ("frame_idx", C.c_uint64),
    ]


class RoiIn(C.Structure):
    _fields_ = [
        ("cam_move_inv", C.c_double * 12), ("prediction", C.c_double * 12), ("predicted_pose", C.c_double * 12),
        ("D", C.c_double * 5), ("image_w", C.c_int32), ("image_h", C.c_int32), ("border", C.c_int32),
        ("pad", C.c_int32),
    ]


class RoiOut(C.Structure):
    _fields_ = [("x", C.c_int32), ("y", C.c_int32), ("width", C.c_int32), ("height", C.c_int32),
                ("bbox", C.c_double * 4)]


class InitParams(C.Structure):
    _fields_ = [("certainty_threshold", C.c_double), ("valid_corr_threshold", C.c_double),
                ("n_particles", C.c_int32), ("max_candidates", C.c_int32)]


class InitOut(C.Structure):
    _fields_ = [("found", C.c_int32), ("flag_fail", C.c_int32), ("n_estimates", C.c_int32),
                ("n_candidates", C.c_int32), ("first_match", C.c_int32), ("n_corr", C.c_int32),
                ("corr", C.c_uint32 * (2 * MAX_MARKERS)), ("predicted_pose", C.c_double * 12),
                ("hist_total", C.c_uint64)]

    def as_dict(self) -> dict:
        return {"found": self.found, "flag_fail": self.flag_fail, "n_estimates": self.n_estimates,
                "n_candidates": self.n_candidates, "first_match": self.first_match,
                "pairs": np.array(self.corr[: 2 * self.n_corr], dtype=np.uint32).reshape(-1, 2),
                "predicted_pose": np.array(self.predicted_pose), "hist_total": self.hist_total}


class DetectParams(C.Structure):
    _fields_ = [("threshold_value", C.c_int32), ("active_markers", C.c_int32), ("gaussian_sigma", C.c_double),
                ("min_blob_area", C.c_double), ("max_blob_area", C.c_double),
                ("max_width_height_distortion", C.c_double), ("max_circular_distortion", C.c_double),
                ("D", C.c_double * 5), ("roi_x", C.c_int32), ("roi_y", C.c_int32), ("roi_w", C.c_int32),
                ("roi_h", C.c_int32)]


class DetectOut(C.Structure):
    _fields_ = [("n", C.c_int32), ("n_components", C.c_int32), ("overflow", C.c_int32), ("pad", C.c_int32)]


class LaunchConfig(C.Structure):
    _fields_ = [("pf", Params), ("init", InitParams), ("num_objects", C.c_int32),
                ("markers_per_object", C.c_int32 * 4), ("use_particle_filter", C.c_int32),
                ("downgrade", C.c_uint8 * MAX_MARKERS)]


class FrameOut(C.Structure):
    _fields_ = [
        ("iters", C.c_int32), ("kept_iter", C.c_int32), ("most_likely_idx", C.c_int32),
        ("accepted", C.c_int32), ("resampled", C.c_int32), ("winner_idx", C.c_int32),
        ("n_corr", C.c_int32), ("flag_fail", C.c_int32),
        ("highest_prob", C.c_double), ("prob_sum", C.c_double),
        ("winner_pose", C.c_double * 12), ("most_likely_pose", C.c_double * 12),
        ("corr", C.c_uint32 * (2 * MAX_MARKERS)),
    ]

    def pairs(self) -> np.ndarray:
        return np.array(self.corr[: 2 * self.n_corr], dtype=np.uint32).reshape(-1, 2)

    def as_dict(self) -> dict:
        return {
            "iters": self.iters, "kept_iter": self.kept_iter, "most_likely_idx": self.most_likely_idx,
            "accepted": self.accepted, "resampled": self.resampled, "winner_idx": self.winner_idx,
            "n_corr": self.n_corr, "flag_fail": self.flag_fail, "highest_prob": self.highest_prob,
            "prob_sum": self.prob_sum, "winner_pose": np.array(self.winner_pose),
            "most_likely_pose": np.array(self.most_likely_pose), "pairs": self.pairs(),
        }


_lib = None


def load() -> C.CDLL:
    """Load libpfmpe.so (raises if it has not been built: the product has no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build the HIP engine first (python -c 'import __graft_entry__ as g; g.build()')"
        )
    lib = C.CDLL(os.environ.get("PFMPE_LIB_OVERRIDE") or LIB_PATH)  # override: A/B builds of the same ABI
    P, I, D, U64, I64 = C.c_void_p, C.c_int, C.c_double, C.c_uint64, C.c_int64
    dp = C.POINTER(C.c_double)
    sig = {
        "pfmpe_create": (I, [C.POINTER(P), I, I, I, I, I]),
        "pfmpe_destroy": (None, [P]),
        "pfmpe_last_error": (C.c_char_p, [P]),
        "pfmpe_abi_version": (I, []),
        "pfmpe_set_model": (I, [P, dp, I, dp, C.POINTER(C.c_uint8)]),
        "pfmpe_set_params": (I, [P, C.POINTER(Params)]),
        "pfmpe_default_params": (None, [C.POINTER(Params)]),
        "pfmpe_set_prior": (I, [P, dp, I]),
        "pfmpe_step": (I, [P, C.POINTER(FrameIn), C.POINTER(FrameOut)]),
        "pfmpe_step_batch": (I, [P, C.POINTER(FrameIn), I, C.POINTER(FrameOut), C.POINTER(I)]),
        "pfmpe_step_multi": (I, [C.POINTER(P), I, C.POINTER(FrameIn), C.POINTER(FrameOut)]),
        "pfmpe_step_multi_batch": (I, [C.POINTER(P), I, C.POINTER(FrameIn), I, C.POINTER(FrameOut), C.POINTER(I)]),
        "pfmpe_get_particles": (I, [P, I, dp]),
        "pfmpe_get_weights": (I, [P, dp]),
        "pfmpe_get_counts": (I, [P, C.POINTER(C.c_uint32)]),
        "pfmpe_set_option": (I, [P, I, I64]),
        "pfmpe_get_info": (I, [P, I, C.POINTER(I64)]),
        "pfmpe_stage_blob_bank": (I, [P, dp, C.POINTER(C.c_int32), I]),
        "pfmpe_get_kernel_stats": (I, [P, I, C.POINTER(I64), dp]),
        "pfmpe_reset_kernel_stats": (I, [P]),
        "pfmpe_kernel_name": (C.c_char_p, [I]),
        "pfmpe_host_ref_uniform": (D, [C.c_uint32, U64, D, D]),
        "pfmpe_host_philox": (None, [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
        "pfmpe_predict_roi": (I, [P, C.POINTER(RoiIn), C.POINTER(RoiOut)]),
        "pfmpe_default_init_params": (None, [C.POINTER(InitParams)]),
        "pfmpe_p3p_histogram": (I, [P, dp, I, C.POINTER(C.c_uint32)]),
        "pfmpe_initialise": (I, [P, dp, I, C.POINTER(InitParams), C.POINTER(InitOut), C.POINTER(C.c_uint32)]),
        "pfmpe_parse_marker_yaml": (I, [C.c_char_p, dp, I]),
        "pfmpe_default_launch_config": (None, [C.POINTER(LaunchConfig)]),
        "pfmpe_parse_launch": (I, [C.c_char_p, C.POINTER(LaunchConfig)]),
        "pfmpe_parse_camera_info": (I, [C.c_char_p, dp, dp, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
        "pfmpe_write_blob_stream": (I, [C.c_char_p, dp, dp, C.POINTER(C.c_int32), I]),
        "pfmpe_read_blob_stream": (I, [C.c_char_p, dp, dp, C.POINTER(C.c_int32), I, I64, C.POINTER(I),
                                       C.POINTER(I64)]),
        "pfmpe_stage_blob_stream": (I, [P, C.c_char_p, C.POINTER(I)]),
        "pfmpe_default_detect_params": (None, [C.POINTER(DetectParams)]),
        "pfmpe_stage_image": (I, [P, C.POINTER(C.c_uint8), I, I, I]),
        "pfmpe_find_leds": (I, [P, C.POINTER(C.c_uint8), I, I, I, C.POINTER(DetectParams), dp,
                                C.POINTER(C.c_float), I, C.POINTER(DetectOut)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def default_params() -> Params:
    p = Params()
    load().pfmpe_default_params(C.byref(p))
    return p


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class PFError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"pfmpe error {code}: {msg}")
        self.code = code


class Engine:
    """One PF context (one camera stream / tracked object) on one HIP device."""

    def __init__(self, device: int = 0, max_particles: int = 1000, max_markers: int = MAX_MARKERS,
                 max_blobs: int = MAX_BLOBS, state_dtype: int = STATE_F32):
        self.lib = load()
        self.ctx = C.c_void_p()
        rc = self.lib.pfmpe_create(C.byref(self.ctx), device, max_particles, max_markers, max_blobs, state_dtype)
        if rc != OK:
            raise PFError(rc, "pfmpe_create failed (no HIP device?)")
        self.state_dtype = state_dtype
        self.max_particles = max_particles
        self.N = 0
        self.M = 0

    def close(self):
        if self.ctx:
            self.lib.pfmpe_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc: int):
        if rc != OK:
            raise PFError(rc, self.lib.pfmpe_last_error(self.ctx).decode())

    def set_model(self, markers: np.ndarray, K: np.ndarray, downgrade=None):
        m = np.ascontiguousarray(markers, dtype=np.float64).reshape(-1, 3)
        k = np.ascontiguousarray(K, dtype=np.float64).reshape(9)
        dg = None
        if downgrade is not None:
            dga = np.ascontiguousarray(downgrade, dtype=np.uint8)
            dg = dga.ctypes.data_as(C.POINTER(C.c_uint8))
        self._chk(self.lib.pfmpe_set_model(self.ctx, _dptr(m), m.shape[0], _dptr(k), dg))
        self.M = m.shape[0]

    def set_params(self, params: Params):
        self._chk(self.lib.pfmpe_set_params(self.ctx, C.byref(params)))

    def set_option(self, opt: int, value: int):
        self._chk(self.lib.pfmpe_set_option(self.ctx, opt, int(value)))

    def info(self, key: int) -> int:
        v = C.c_int64()
        self._chk(self.lib.pfmpe_get_info(self.ctx, key, C.byref(v)))
        return v.value

    def last_error(self) -> str:
        return self.lib.pfmpe_last_error(self.ctx).decode()

    def set_prior(self, poses: np.ndarray):
        p = np.ascontiguousarray(poses, dtype=np.float64).reshape(-1, 12)
        self._chk(self.lib.pfmpe_set_prior(self.ctx, _dptr(p), p.shape[0]))
        self.N = p.shape[0]

    def stage_blob_bank(self, frames):
        offs = np.zeros(len(frames) + 1, dtype=np.int32)
        for i, f in enumerate(frames):
            offs[i + 1] = offs[i] + len(f)
        allb = np.ascontiguousarray(np.concatenate([np.asarray(f, np.float64).reshape(-1, 2) for f in frames]
                                                   + [np.zeros((0, 2))]), dtype=np.float64)
        self._bank_keep = allb
        self._chk(self.lib.pfmpe_stage_blob_bank(self.ctx, _dptr(allb), offs.ctypes.data_as(C.POINTER(C.c_int32)),
                                                 len(frames)))

    @staticmethod
    def make_frame(current_pose, predicted_pose, prediction, blobs=None, B=None, cam_move_inv=None,
                   it_since_init=2, dt=0.02, seed=1, frame_idx=0, force_iters=0, bank_frame=-1):
        fi = FrameIn()
        fi.current_pose[:] = list(np.asarray(current_pose, np.float64).reshape(12))
        fi.predicted_pose[:] = list(np.asarray(predicted_pose, np.float64).reshape(12))
        fi.prediction[:] = list(np.asarray(prediction, np.float64).reshape(12))
        cm = np.eye(4)[:3].reshape(12) if cam_move_inv is None else np.asarray(cam_move_inv, np.float64).reshape(12)
        fi.cam_move_inv[:] = list(cm)
        keep = None
        if blobs is not None:
            keep = np.ascontiguousarray(blobs, dtype=np.float64).reshape(-1, 2)
            fi.blobs = _dptr(keep)
            fi.B = keep.shape[0]
        else:
            fi.blobs = C.POINTER(C.c_double)()
            fi.B = int(B or 0)
        fi.bank_frame = bank_frame
        fi.it_since_init = it_since_init
        fi.force_iters = force_iters
        fi.dt = dt
        fi.seed = seed
        fi.frame_idx = frame_idx
        fi._keep = keep  # keep the blob buffer alive with the struct
        return fi

    def step(self, frame: FrameIn) -> FrameOut:
        out = FrameOut()
        self._chk(self.lib.pfmpe_step(self.ctx, C.byref(frame), C.byref(out)))
        return out

    def step_batch(self, frames) -> list:
        """Frames (a list of FrameIn) run back to back in C, each blocking on its own record; returns a list."""
        return list(self.run_batch(self.prepare_batch(frames)))

    @staticmethod
    def prepare_batch(frames):
        """The input and output arrays of a step_batch call, built ahead of it (a timed loop then contains only
        the C call: building 20 ctypes frames cost the driver's 20-frame bench line ~1-2 us per frame)."""
        n = len(frames)
        return n, (FrameIn * n)(*frames), (FrameOut * n)()

    def run_batch(self, prepared):
        """pfmpe_step_batch over prepare_batch's arrays; returns prepare_batch's output array itself (a ctypes
        FrameOut array, not a copy): a second run over the same prepared arrays overwrites it (the bench's timed loop
        reuses them on purpose)."""
        n, arr_in, arr_out = prepared
        done = C.c_int()
        self._chk(self.lib.pfmpe_step_batch(self.ctx, arr_in, n, arr_out, C.byref(done)))
        return arr_out

    @staticmethod
    def step_multi(engines, frames) -> list:
        """One frame of each engine (independent camera streams / objects) as ONE batch on the device
        (pfmpe_step_multi): frames[s] belongs to engines[s]; outputs and state equal per-engine step()."""
        S = len(engines)
        if S != len(frames) or S == 0:
            raise ValueError("step_multi: one frame per engine")
        ctxs = (C.c_void_p * S)(*[e.ctx.value for e in engines])
        arr_in = (FrameIn * S)(*frames)
        arr_out = (FrameOut * S)()
        engines[0]._chk(engines[0].lib.pfmpe_step_multi(ctxs, S, arr_in, arr_out))
        return list(arr_out)

    def predict_roi(self, prediction, predicted_pose, D, image_w, image_h, border, cam_move_inv=None) -> dict:
        """Region of interest for the next detection (PE:396-412): {"roi": [x, y, w, h], "bbox": [...]}."""
        ri = RoiIn()
        cm = np.eye(4)[:3].reshape(12) if cam_move_inv is None else np.asarray(cam_move_inv, np.float64).reshape(12)
        ri.cam_move_inv[:] = list(cm)
        ri.prediction[:] = list(np.asarray(prediction, np.float64).reshape(12))
        ri.predicted_pose[:] = list(np.asarray(predicted_pose, np.float64).reshape(12))
        ri.D[:] = list(np.asarray(D, np.float64).reshape(5))
        ri.image_w, ri.image_h, ri.border = int(image_w), int(image_h), int(border)
        ro = RoiOut()
        self._chk(self.lib.pfmpe_predict_roi(self.ctx, C.byref(ri), C.byref(ro)))
        return {"roi": [ro.x, ro.y, ro.width, ro.height], "bbox": np.array(list(ro.bbox))}

    def p3p_histogram(self, blobs) -> np.ndarray:
        """Stage 1 of initialise (PE:1526-1716): the B x M correspondence histogram (uint32)."""
        b = np.ascontiguousarray(blobs, dtype=np.float64).reshape(-1, 2)
        h = np.zeros((b.shape[0], self.M), dtype=np.uint32)
        self._chk(self.lib.pfmpe_p3p_histogram(self.ctx, _dptr(b), b.shape[0], h.ctypes.data_as(C.POINTER(C.c_uint32))))
        return h

    def initialise(self, blobs, n_particles=0, certainty_threshold=1.0, valid_corr_threshold=0.5,
                   max_candidates=1 << 20):
        """PoseEstimator::initialise (PE:1503-1786) -> (out dict, histogram).  On success the context's
        particle set is the seeded PoseParticle set (self.N = n_particles)."""
        b = np.ascontiguousarray(blobs, dtype=np.float64).reshape(-1, 2)
        ip = InitParams()
        self.lib.pfmpe_default_init_params(C.byref(ip))
        ip.certainty_threshold = certainty_threshold
        ip.valid_corr_threshold = valid_corr_threshold
        ip.n_particles = int(n_particles)
        ip.max_candidates = int(max_candidates)
        out = InitOut()
        h = np.zeros((b.shape[0], self.M), dtype=np.uint32)
        self._chk(self.lib.pfmpe_initialise(self.ctx, _dptr(b), b.shape[0], C.byref(ip), C.byref(out),
                                            h.ctypes.data_as(C.POINTER(C.c_uint32))))
        d = out.as_dict()
        if d["found"]:
            self.N = int(n_particles) if n_particles else (self.N or self.max_particles)
        return d, h

    def stage_image(self, image: np.ndarray):
        img = np.ascontiguousarray(image, dtype=np.uint8)
        self._chk(self.lib.pfmpe_stage_image(self.ctx, img.ctypes.data_as(C.POINTER(C.c_uint8)), img.shape[1],
                                             img.shape[0], img.strides[0]))
        self._img_shape = img.shape

    def find_leds(self, image=None, D=None, roi=None, max_out=MAX_BLOBS, **kw):
        """LEDDetector::findLeds (led_detector.cpp:46-215) on the device -> (undistorted B x 2,
        distorted B x 2 float32, info).  image None: the staged image.  kw: DetectParams fields."""
        p = DetectParams()
        self.lib.pfmpe_default_detect_params(C.byref(p))
        if D is not None:
            p.D[:] = list(np.asarray(D, np.float64).reshape(5))
        if roi is not None:
            p.roi_x, p.roi_y, p.roi_w, p.roi_h = [int(v) for v in roi]
        for k, v in kw.items():
            setattr(p, k, v)
        blobs = np.zeros((max(max_out, 1), 2))
        dist = np.zeros((max(max_out, 1), 2), dtype=np.float32)
        out = DetectOut()
        if image is not None:
            img = np.ascontiguousarray(image, dtype=np.uint8)
            ip, (h, w), pitch = img.ctypes.data_as(C.POINTER(C.c_uint8)), img.shape, img.strides[0]
        else:
            ip, (h, w) = C.POINTER(C.c_uint8)(), self._img_shape
            pitch = w
        self._chk(self.lib.pfmpe_find_leds(self.ctx, ip, w, h, pitch, C.byref(p), _dptr(blobs),
                                           dist.ctypes.data_as(C.POINTER(C.c_float)), max_out, C.byref(out)))
        n = min(out.n, max_out)
        return blobs[:n].copy(), dist[:n].copy(), {"n": out.n, "n_components": out.n_components,
                                                    "overflow": out.overflow}

    def stage_blob_stream(self, path) -> int:
        """Stage every frame of a PFMB stream file in the device blob bank; returns the frame count."""
        n = C.c_int()
        self._chk(self.lib.pfmpe_stage_blob_stream(self.ctx, _enc(path), C.byref(n)))
        return n.value

    def get_particles(self, which: int) -> np.ndarray:
        out = np.empty((self.N, 12), dtype=np.float64)
        self._chk(self.lib.pfmpe_get_particles(self.ctx, which, _dptr(out)))
        return out

    def get_weights(self) -> np.ndarray:
        out = np.empty(self.N, dtype=np.float64)
        self._chk(self.lib.pfmpe_get_weights(self.ctx, _dptr(out)))
        return out

    def get_counts(self) -> np.ndarray:
        out = np.empty(self.N, dtype=np.uint32)
        self._chk(self.lib.pfmpe_get_counts(self.ctx, out.ctypes.data_as(C.POINTER(C.c_uint32))))
        return out

    def kernel_stats(self) -> dict:
        res = {}
        for k in range(K_COUNT):
            n = C.c_int64()
            ms = C.c_double()
            self._chk(self.lib.pfmpe_get_kernel_stats(self.ctx, k, C.byref(n), C.byref(ms)))
            res[self.lib.pfmpe_kernel_name(k).decode()] = (n.value, ms.value)
        return res

    def reset_kernel_stats(self):
        self._chk(self.lib.pfmpe_reset_kernel_stats(self.ctx))


def _enc(x):
    return x.encode() if isinstance(x, str) else x


def parse_marker_yaml(text) -> np.ndarray:
    """Marker positions (M x 3) from the reference's marker YAML (README.md:95-117)."""
    lib = load()
    n = lib.pfmpe_parse_marker_yaml(_enc(text), None, 0)
    if n < 0:
        raise PFError(n, "malformed marker YAML")
    out = np.zeros((n, 3))
    lib.pfmpe_parse_marker_yaml(_enc(text), _dptr(out), n)
    return out


def parse_launch(text) -> LaunchConfig:
    """PF / init / marker-split parameters of a ROS launch file (pf_mpe/launch/<name>.launch)."""
    lib = load()
    cfg = LaunchConfig()
    lib.pfmpe_default_launch_config(C.byref(cfg))
    n = lib.pfmpe_parse_launch(_enc(text), C.byref(cfg))
    if n < 0:
        raise PFError(n, "malformed launch text")
    cfg.n_known = n
    return cfg


def parse_camera_info(text) -> dict:
    """K (3x3), D (5), width, height from a sensor_msgs/CameraInfo echo (README.md:127-143)."""
    K = np.zeros(9)
    D = np.zeros(5)
    w, h = C.c_int32(), C.c_int32()
    m = load().pfmpe_parse_camera_info(_enc(text), _dptr(K), _dptr(D), C.byref(w), C.byref(h))
    if m < 0:
        raise PFError(m, "malformed camera_info")
    return {"K": K.reshape(3, 3), "D": D, "width": w.value, "height": h.value, "found": m}


def write_blob_stream(path, frames, timestamps=None):
    """Recorded detections (a list of B_f x 2 arrays, undistorted px) -> the PFMB stream file."""
    offs = np.zeros(len(frames) + 1, dtype=np.int32)
    for i, f in enumerate(frames):
        offs[i + 1] = offs[i] + len(f)
    allb = np.ascontiguousarray(np.concatenate([np.asarray(f, np.float64).reshape(-1, 2) for f in frames]
                                               + [np.zeros((0, 2))]), dtype=np.float64)
    ts = np.ascontiguousarray(np.zeros(len(frames)) if timestamps is None else timestamps, dtype=np.float64)
    rc = load().pfmpe_write_blob_stream(_enc(path), _dptr(ts), _dptr(allb), offs.ctypes.data_as(C.POINTER(C.c_int32)),
                                        len(frames))
    if rc != OK:
        raise PFError(rc, f"cannot write {path}")


def read_blob_stream(path):
    """PFMB stream file -> (timestamps, list of B_f x 2 arrays)."""
    lib = load()
    nf, nb = C.c_int(), C.c_int64()
    rc = lib.pfmpe_read_blob_stream(_enc(path), None, None, None, 0, 0, C.byref(nf), C.byref(nb))
    if rc != OK:
        raise PFError(rc, f"cannot read {path}")
    ts = np.zeros(nf.value)
    bl = np.zeros((max(nb.value, 1), 2))
    off = np.zeros(nf.value + 1, dtype=np.int32)
    rc = lib.pfmpe_read_blob_stream(_enc(path), _dptr(ts), _dptr(bl), off.ctypes.data_as(C.POINTER(C.c_int32)), nf.value,
                                    nb.value, C.byref(nf), C.byref(nb))
    if rc != OK:
        raise PFError(rc, f"cannot read {path}")
    return ts, [bl[off[i]:off[i + 1]].copy() for i in range(nf.value)]


def host_ref_uniform(seed: int, j: int, a: float, b: float) -> float:
    return load().pfmpe_host_ref_uniform(seed, j, a, b)


def host_philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    load().pfmpe_host_philox(c, k, o)
    return list(o)
