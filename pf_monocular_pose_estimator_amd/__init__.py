"""pf_monocular_pose_estimator_amd — MI355X-native particle-filter pose engine.

The hot path of ObiRobotics/pf_monocular_pose_estimator (the PF step of PoseEstimator::estimateBodyPose,
pf_mpe_lib/src/pose_estimator.cpp:475-733) as hand-written HIP for gfx950 behind the C-ABI in
include/pfmpe.h.  This package holds the in-tree built library (libpfmpe.so), its ctypes binding
(`_capi`), and the synthetic stream generator used by tests and bench.py.
"""
from ._capi import (  # noqa: F401
    Engine, FrameIn, FrameOut, Params, PFError, default_params, load, host_philox, host_ref_uniform,
    STATE_F32, STATE_F64, STATE_F16, RNG_REFERENCE, RNG_PHILOX, FLAG_ACCEPTED, FLAG_REINIT,
    OPT_RECORD_COUNTS, OPT_PRUNE, OPT_TIMING, OPT_FUSED, OPT_KEEP_PROPAGATED, K_FRAME, K_ROI, K_FINAL, MAX_MARKERS, MAX_BLOBS, LIB_PATH,
    OPT_WAIT_BOUND_US, OPT_FUSED_REARM, OPT_MULTI_MAX_BLOCKS, OPT_DIAG, DIAG_LAG_LOADS, DIAG_ABANDON, DIAG_NO_STREAM, DIAG_FORCE_STREAM,
    DIAG_SERIAL_TOP, DIAG_NO_PK, DIAG_CORRUPT_DESC, DIAG_NO_DEFER, DIAG_BLOCK_RESAMPLE, DIAG_MIN_SIDE, DIAG_ABANDON_FINISH, OPT_DEFER_RESAMPLE, OK, E_ARG, E_HIP, E_CAP, E_STATE,
    SHAPE_TWO_LAUNCH, SHAPE_FRAME, SHAPE_FRAME2, INFO_FUSED, INFO_FUSED_FALLBACKS, INFO_LAST_SHAPE,
    INFO_GUARD_SKIPS, INFO_N, INFO_LAST_WEIGH_PASS, INFO_LAST_GRID, INFO_LAST_RESAMPLE, RESAMPLE_BLOCKS, RESAMPLE_OWNERS, WEIGH_BLOCKS, WEIGH_STREAM, WEIGH_PK,
)

__all__ = [
    "Engine", "FrameIn", "FrameOut", "Params", "PFError", "default_params", "load",
    "STATE_F32", "STATE_F64", "RNG_REFERENCE", "RNG_PHILOX",
]
