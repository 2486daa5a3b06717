"""GPU parity of the LED detector (pfmpe_find_leds; LEDDetector::findLeds, led_detector.cpp:46-215,
SURVEY.md §8f row 4) against the CPU restatement (oracle/detect_oracle.cpp).  The pipeline is integer
(threshold, blur, labelling, border following) up to the polygon moments (exact double sums of small
integers) and the same-order double undistortion, so the bar is exact: same detections, same order,
identical float centres and double undistorted positions."""
import numpy as np
import pytest

import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn
from oracle import pforacle as orc

pytestmark = pytest.mark.gpu
K, D = syn.K_README, syn.D_README


def engine():
    eng = pf.Engine(device=0, max_particles=1000)
    eng.set_model(syn.markers_for(5), K)
    return eng


def compare(eng, img, **kw):
    und, dist, info = eng.find_leds(img, D=D, **kw)
    okw = dict(kw)
    if "active_markers" in okw:
        okw["active_markers"] = bool(okw["active_markers"])
    u_ref, d_ref, _, _ = orc.find_leds(img, K, D, **okw)
    assert info["overflow"] == 0
    assert und.shape == u_ref.shape, (und.shape, u_ref.shape)
    np.testing.assert_array_equal(dist, d_ref)
    np.testing.assert_array_equal(und, u_ref)
    return und


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_full_image_matches_oracle(seed):
    eng = engine()
    T = syn.truth_pose(0.3 + 0.2 * seed)
    img, ideal = syn.led_image(T, syn.markers_for(5), seed=seed, n_false=2 + seed)
    und = compare(eng, img)
    for p in ideal:
        assert np.min(np.hypot(*(und - p).T)) < 0.3
    eng.close()


def test_roi_sigma_and_filters_match_oracle():
    eng = engine()
    img, ideal = syn.led_image(syn.truth_pose(0.5), syn.markers_for(5), seed=5, radius=4.5, noise=120)
    x0, y0 = int(ideal[:, 0].min()) - 25, int(ideal[:, 1].min()) - 20
    roi = (x0, y0, int(ideal[:, 0].max()) + 25 - x0, int(ideal[:, 1].max()) + 20 - y0)
    compare(eng, img, roi=roi)
    compare(eng, img, roi=roi, gaussian_sigma=1.3, min_blob_area=10.0, max_blob_area=400.0)
    compare(eng, img, threshold_value=100)  # background noise passes: many small components
    eng.close()


def test_passive_markers_and_staged_image():
    eng = engine()
    img, _ = syn.led_image(syn.truth_pose(0.7), syn.markers_for(5), seed=7)
    inv = np.ascontiguousarray(255 - img)
    compare(eng, inv, threshold_value=14, active_markers=0)
    eng.stage_image(img)
    und, dist, info = eng.find_leds(None, D=D)
    u_ref, d_ref, _, _ = orc.find_leds(img, K, D)
    np.testing.assert_array_equal(und, u_ref)
    eng.close()


def test_detections_drive_the_pf():
    """Detector output (image_points_) feeds the PF step exactly like synthetic blobs would."""
    M, N = 5, 4096
    T = syn.truth_pose(0.5)
    img, ideal = syn.led_image(T, syn.markers_for(M), seed=11, n_false=2)
    eng = pf.Engine(device=0, max_particles=N)
    eng.set_model(syn.markers_for(M), K)
    eng.set_params(pf.default_params())
    blobs, _, _ = eng.find_leds(img, D=D)
    eng.set_prior(syn.initial_prior(T, N))
    T12 = syn.to12(T)
    out = eng.step(eng.make_frame(T12, T12, np.eye(4)[:3].reshape(12), blobs=blobs, seed=1)).as_dict()
    assert out["accepted"] == 1 and out["n_corr"] == M
    eng.close()
