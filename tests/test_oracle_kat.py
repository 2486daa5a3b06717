"""Known-answer tests that pin the CPU oracle (the reference ships no tests or fixtures).

Each KAT is derived from the reference source:
  * calculateEstimationProbability  pf_mpe_lib/src/pose_estimator.cpp:2385-2445 (SURVEY §8c KATs i-x)
  * std::default_random_engine      minstd_rand0, the C++ standard's [rand.predef] check value
  * Philox4x32-10                   published Random123 known-answer vectors
"""
import numpy as np
import pytest

from oracle import pforacle as orc

TOL, TOL_PF = 5.0, 4.0


def proj_exact(M=5, seed=0):
    rng = np.random.default_rng(seed)
    return rng.uniform([50, 50], [700, 430], size=(M, 2))


@pytest.mark.parametrize("closed", [False, True])
def test_kat_i_exact_pose_scores_M_times_M_plus_1(closed):
    p = proj_exact()
    P, pairs = orc.likelihood(p, p.copy(), TOL, TOL_PF, closed=closed)
    assert P == 5 * 6
    assert sorted(pairs[:, 0].tolist()) == [1, 2, 3, 4, 5]
    assert (pairs[:, 0] == pairs[:, 1]).all()


@pytest.mark.parametrize("closed", [False, True])
@pytest.mark.parametrize("d", [0.0, 0.5, 1.7, 3.999])
def test_kat_ii_offset_marker_term(d, closed):
    p = proj_exact()
    b = p.copy()
    b[2, 0] += d
    P, _ = orc.likelihood(p, b, TOL, TOL_PF, closed=closed)
    expect = 4 * (5 + 1.0) + (5 + ((TOL - d) / TOL) ** 2)
    assert P == pytest.approx(expect, abs=1e-12)


@pytest.mark.parametrize("closed", [False, True])
def test_kat_iii_beyond_gate_dropped(closed):
    p = proj_exact()
    b = p.copy()
    b[3, 1] += TOL_PF + 1e-6
    P, pairs = orc.likelihood(p, b, TOL, TOL_PF, closed=closed)
    assert P == pytest.approx(4 * 6.0)
    assert 4 not in pairs[:, 0]


@pytest.mark.parametrize("closed", [False, True])
def test_kat_iv_self_occlusion_penalties(closed):
    p = proj_exact()
    # markers 1 and 2 project onto one blob: one penalty 3
    far = np.array([[5000.0, 5000.0], [6000.0, 6000.0]])  # keep B = 5 so the cap min(B, M) stays 5
    b = np.vstack([np.delete(p.copy(), 1, axis=0), far[:1]])
    pp = p.copy()
    pp[1] = p[0]
    P, _ = orc.likelihood(pp, b, TOL, TOL_PF, closed=closed)
    assert P == pytest.approx(5 * 6.0 - 3)
    # three markers on one blob: penalties 3 + 6
    pp[2] = p[0]
    b2 = np.vstack([np.delete(p.copy(), [1, 2], axis=0), far])
    P2, _ = orc.likelihood(pp, b2, TOL, TOL_PF, closed=closed)
    assert P2 == pytest.approx(5 * 6.0 - 3 - 6)
    # with B = 4 blobs only min(B, M) = 4 extractions happen (PE:2409)
    P3, pairs3 = orc.likelihood(pp[:5], np.delete(p.copy(), 1, axis=0), TOL, TOL_PF, closed=closed)
    assert len(pairs3) == 4


@pytest.mark.parametrize("closed", [False, True])
def test_kat_v_downgrade(closed):
    p = proj_exact()
    dg = np.array([0, 1, 0, 0, 1], np.uint8)
    P, _ = orc.likelihood(p, p.copy(), TOL, TOL_PF, downgrade=dg, closed=closed)
    assert P == pytest.approx(30 - 4)


@pytest.mark.parametrize("closed", [False, True])
def test_kat_vi_fewer_blobs_caps_accepted(closed):
    p = proj_exact()
    P, pairs = orc.likelihood(p, p[:3].copy(), TOL, TOL_PF, closed=closed)
    assert len(pairs) == 3
    assert P == pytest.approx(3 * 6.0)


@pytest.mark.parametrize("closed", [False, True])
def test_kat_vii_tol_pf_above_tol(closed):
    p = proj_exact()
    b = p.copy()
    b[0, 0] += 8.0  # d = 8 > tol = 5 but <= tol_pf = 10 (cfg default): term grows again
    P, _ = orc.likelihood(p, b, TOL, 10.0, closed=closed)
    assert P == pytest.approx(4 * 6.0 + 5 + ((5 - 8) / 5) ** 2)


def test_kat_viii_behind_camera_mirrors():
    K = np.array([[400.0, 0, 300], [0, 400, 200], [0, 0, 1]])
    pose = np.eye(4)[:3].reshape(12)
    uv_front = orc.project(K, pose, [0.1, 0.05, 2.0])
    uv_back = orc.project(K, pose, [-0.1, -0.05, -2.0])
    assert np.allclose(uv_front, uv_back)  # no z>0 cull (PE:1032)


def test_kat_nan_at_origin_breaks_immediately():
    p = proj_exact()
    p[0] = [np.nan, np.nan]
    P, pairs = orc.likelihood(p, p.copy(), TOL, TOL_PF)
    Pc, _ = orc.likelihood(p, p.copy(), TOL, TOL_PF, closed=True)
    assert P == 0.0 and Pc == 0.0 and len(pairs) == 0


def test_literal_equals_closed_form_random():
    rng = np.random.default_rng(3)
    for trial in range(400):
        M = int(rng.integers(1, 13))
        B = int(rng.integers(0, 40))
        proj = rng.uniform(0, 60, size=(M, 2))
        blobs = rng.uniform(0, 60, size=(B, 2))
        if B and trial % 3 == 0:  # force exact ties and shared blobs
            blobs[: min(B, M)] = np.round(proj[: min(B, M)])
            proj = np.round(proj)
        dg = rng.integers(0, 2, size=M).astype(np.uint8)
        tol_pf = float(rng.choice([2.0, 4.0, 10.0]))
        a = orc.likelihood(proj, blobs, TOL, tol_pf, downgrade=dg)
        b = orc.likelihood(proj, blobs, TOL, tol_pf, downgrade=dg, closed=True)
        assert a[0] == b[0], (trial, a, b)
        assert np.array_equal(a[1], b[1]), (trial, a, b)


def test_minstd_rand0_standard_check_value():
    # [rand.predef]: the 10000th consecutive invocation of a default-constructed minstd_rand0
    # produces 1043618065
    assert orc.minstd_outputs(1, 10000)[-1] == 1043618065
    assert orc.minstd_outputs(1, 3) == [16807, 282475249, 1622650073]


@pytest.mark.parametrize("ctr,key,expect", [
    ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
    ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
    ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
     [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
])
def test_philox_published_vectors(ctr, key, expect):
    assert orc.philox(ctr, key) == expect


def test_uniform_draw_two_engine_outputs():
    """generate_canonical consumes two engine outputs per double (bits/random.tcc:3348-3376)."""
    g = orc.minstd_outputs(42, 4)
    u = orc.uniform_draws(42, 0.0, 1.0, 2)
    R = 2147483646.0
    expect0 = ((g[0] - 1) + (g[1] - 1) * R) / 4611686009837453312.0
    assert u[0] == expect0
    assert u[1] == ((g[2] - 1) + (g[3] - 1) * R) / 4611686009837453312.0
