"""GPU: the frame shape the engine actually runs.

A one-launch frame needs every block resident at once; a kernel whose registers grow past the residency
rule (csrc/pfmpe_ctx.hpp frame_fused: at most 2 blocks per CU, one below the occupancy answer) silently
takes the two-launch path, which is correct but slower.  These tests pin the shape at the sizes the
bench and the scale configs use, for every state precision: the default (k_frame2) and the tree frame
must run as ONE launch up to 512 blocks, and the two-launch path above.
"""
import pytest

import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn

pytestmark = pytest.mark.gpu

STATE = {"f32": pf.STATE_F32, "f64": pf.STATE_F64, "f16": pf.STATE_F16}


def run_frames(N, state, fused, frames=3):
    base = syn.CONFIGS["C2"]
    cfg = syn.StreamConfig(base.name, M=base.M, B=base.B, N=N, heavy=base.heavy)
    st = syn.make_stream(cfg, frames)
    eng = pf.Engine(device=0, max_particles=N, state_dtype=STATE[state])
    try:
        eng.set_option(pf.OPT_FUSED, fused)
        eng.set_model(st.markers, st.K)
        eng.set_params(pf.default_params())
        eng.set_prior(st.prior())
        eng.set_option(pf.OPT_TIMING, 1)  # every frame bracketed: the per-kernel launch counts
        eng.reset_kernel_stats()
        for fr in st.frames:
            eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=fr.blobs, dt=fr.dt,
                                    seed=3, frame_idx=fr.index))
        return {k: v[0] for k, v in eng.kernel_stats().items()}
    finally:
        eng.close()


@pytest.mark.parametrize("state", ["f32", "f64", "f16"])
@pytest.mark.parametrize("fused", [2, 1])
@pytest.mark.parametrize("N", [100000, 131072])  # 391 blocks (C2) and the 512-block limit
def test_one_launch_frame(N, state, fused):
    n = run_frames(N, state, fused)
    if fused == 1 and state == "f64":
        # the fp64 tree frame holds more registers than 3 waves per SIMD allow: above 256 blocks it runs
        # as two launches (the default flat frame does not)
        assert n["k_frame"] == 0 and n["k_propagate_weigh"] >= 3, n
        return
    assert n["k_frame"] >= 3, n
    assert n["k_propagate_weigh"] == 0 and n["k_resample"] == 0, n


@pytest.mark.parametrize("N", [200000])
def test_two_launch_beyond_residency(N):
    n = run_frames(N, "f32", 2, frames=2)
    assert n["k_frame"] == 0, n
    assert n["k_propagate_weigh"] >= 2 and n["k_resample"] >= 2, n
