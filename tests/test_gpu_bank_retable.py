"""A staged blob bank follows tol_PF: its tables' cell grids are built for the tol_PF current at
staging, so pfmpe_set_params rebuilds them when tol_PF changes.  A bank staged before a wider tol_PF must
still search its grid (PFMPE_INFO_LAST_GRID) and give the records of host-supplied blobs, whose table is
built per frame with the current parameters."""
import numpy as np
import pytest

import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn
from test_gpu_parity import make_engine

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("state", [pf.STATE_F32, pf.STATE_F16])
def test_bank_rebuilt_when_tol_pf_widens(state):
    N = 20_000
    st = syn.make_stream(syn.StreamConfig("t", M=5, B=50, N=N), 3)
    runs = []
    for use_bank in (True, False):
        eng = make_engine(N, st.markers, st.K, state, pf.RNG_PHILOX, fused=0)
        try:
            if use_bank:
                eng.stage_blob_bank([f.blobs for f in st.frames])  # staged with the default tol_PF
            prm = pf.default_params()
            prm.rng_mode = pf.RNG_PHILOX
            prm.tol_pf = 2.0 * prm.tol_pf  # wider window: the staged grids no longer cover it
            eng.set_params(prm)
            eng.set_prior(st.prior(fast=True))
            recs, grids = [], []
            for f, fr in enumerate(st.frames):
                kw = {"B": len(fr.blobs), "bank_frame": f} if use_bank else {"blobs": fr.blobs}
                out = eng.step(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, dt=fr.dt,
                                              seed=77 + f, frame_idx=f, **kw)).as_dict()
                recs.append((out, eng.get_weights()))
                grids.append(eng.info(pf.INFO_LAST_GRID))
            runs.append((recs, grids))
        finally:
            eng.close()
    (bank, gb), (host, gh) = runs
    assert gb == [1] * len(st.frames) and gh == [1] * len(st.frames), (gb, gh)
    for (a, wa), (b, wb) in zip(bank, host):
        for k, v in a.items():
            assert np.array_equal(np.asarray(v), np.asarray(b[k])), k
        assert np.array_equal(wa, wb)
