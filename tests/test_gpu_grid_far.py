"""The blob cell grid at far-out image coordinates.

The device finds a marker's cell as fma(u, inv_c, ox) in fp32; the table lists every blob within tolq + 0.01 px
of a cell, so the rounding of that cell coordinate must stay well inside 0.01 px.  build_blob_table_host bounds
it (2^-23 (|gx0| inv_c + ncx + 1) cells of cs px) and builds no grid when the bound exceeds 0.0025 px; the frame
then takes the exact x-bucket search.  Here the principal point is moved so that markers and blobs sit around
1e4 px (bound below the limit: the grid serves) and around 2e5 px (above it: the x-buckets serve), and the
pruned search must give exactly the brute-force scan's weights and records either way."""
import numpy as np
import pytest

import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn
from test_gpu_parity import make_engine

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("offset,grid", [(1.0e4, 1), (2.0e5, 0)])
def test_far_coordinates_prune_equals_brute_force(offset, grid):
    N = 50_000
    st = syn.make_stream(syn.StreamConfig("t", M=5, B=50, N=N), 2)
    K = np.array(st.K, dtype=np.float64).reshape(3, 3).copy()
    K[0, 2] += offset
    K[1, 2] += offset
    runs = []
    for prune in (True, False):
        eng = make_engine(N, st.markers, K, pf.STATE_F32, pf.RNG_PHILOX, prune=prune, fused=0)
        try:
            eng.set_prior(st.prior(fast=True))
            recs = []
            for f, fr in enumerate(st.frames):
                blobs = np.asarray(fr.blobs, dtype=np.float64) + offset  # u = fx x/z + cx: the same shift
                out = eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=blobs,
                                              dt=fr.dt, seed=31 + f, frame_idx=f)).as_dict()
                recs.append((out, eng.get_weights(), eng.info(pf.INFO_LAST_GRID)))
            runs.append(recs)
        finally:
            eng.close()
    pruned, brute = runs
    assert [g for _, _, g in pruned] == [grid] * len(st.frames), [g for _, _, g in pruned]
    assert any(o["accepted"] for o, _, _ in pruned)  # the markers do match blobs at these coordinates
    for (a, wa, _), (b, wb, _) in zip(pruned, brute):
        for k, v in a.items():
            assert np.array_equal(np.asarray(v), np.asarray(b[k])), k
        assert np.array_equal(wa, wb)
