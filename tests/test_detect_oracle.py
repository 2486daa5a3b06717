"""CPU checks of the LED-detector restatement (oracle/detect_oracle.cpp; LEDDetector::findLeds,
pf_mpe_lib/src/led_detector.cpp:46-215).  OpenCV is absent and the reference ships no fixtures: parity
unpinned; these are known-answer checks derived from OpenCV 2.4's documented arithmetic and geometry."""
import numpy as np

from pf_monocular_pose_estimator_amd import synthetic as syn
from oracle import pforacle as orc

K, D = syn.K_README, syn.D_README


def test_single_pixel_blur_support():
    """A 255 pixel through the [1, 42, 170, 42, 1]/256 x 2 kernel (sigma 0.6, 8 fraction bits): nonzero where
    (255 k_i k_j + 2^15) >> 16 >= 1, i.e. the 3x3 block and (+-2, 0), (0, +-2)."""
    img = np.zeros((21, 21), np.uint8)
    img[10, 10] = 255
    _, _, _, mask = orc.find_leds(img, K, D, min_blob_area=0, max_blob_area=1e9, max_width_height_distortion=10,
                                  max_circular_distortion=1e9, want_mask=True)
    ys, xs = np.nonzero(mask)
    got = sorted(zip((ys - 10).tolist(), (xs - 10).tolist()))
    want = sorted([(dy, dx) for dy in (-1, 0, 1) for dx in (-1, 0, 1)] + [(-2, 0), (2, 0), (0, -2), (0, 2)])
    assert got == want


def test_threshold_is_strict_and_frame_is_cleared():
    img = np.zeros((30, 30), np.uint8)
    img[10:15, 10:15] = 240  # not > 240: nothing survives THRESH_TOZERO
    _, _, _, mask = orc.find_leds(img, K, D, want_mask=True)
    assert mask.sum() == 0
    img[:, 0] = 255  # the 1-pixel frame is zeroed before findContours
    _, _, _, mask = orc.find_leds(img, K, D, want_mask=True)
    assert mask[:, 0].sum() == 0 and mask[:, 1].sum() > 0


def test_square_blob_centre_and_area():
    img = np.zeros((40, 50), np.uint8)
    img[12:19, 20:27] = 255  # 7 x 7 square centred on (23, 15)
    und, dist, areas, _ = orc.find_leds(img, K, D, min_blob_area=0, max_blob_area=1e9)
    assert len(dist) == 1
    np.testing.assert_allclose(dist[0], [23.0, 15.0], atol=1e-6)  # symmetric contour
    assert 7 * 7 < areas[0] < 11 * 11


def test_synthetic_leds_found_at_their_projections():
    T = syn.truth_pose(0.5)
    img, ideal = syn.led_image(T, syn.markers_for(5), seed=1)
    und, dist, areas, _ = orc.find_leds(img, K, D)
    assert len(und) == 8  # 5 LEDs + 3 distractor discs; the bar fails the aspect filter
    for p in ideal:
        assert np.min(np.hypot(*(und - p).T)) < 0.3
    # findContours order: reverse raster order of each contour's first pixel (bottom blobs first)
    top = [np.floor(d[1] - 4) for d in dist]
    assert all(a >= b - 1 for a, b in zip(top, top[1:]))


def test_roi_offsets_and_passive_markers():
    T = syn.truth_pose(0.5)
    img, ideal = syn.led_image(T, syn.markers_for(5), seed=2, n_false=0)
    x0, y0 = int(ideal[:, 0].min()) - 30, int(ideal[:, 1].min()) - 30
    roi = (x0, y0, int(ideal[:, 0].max()) + 30 - x0, int(ideal[:, 1].max()) + 30 - y0)
    und_full, _, _, _ = orc.find_leds(img, K, D)
    und_roi, _, _, _ = orc.find_leds(img, K, D, roi=roi)
    # same contours; the centre is float(ROI-relative centroid) + float(offset) (LD:94): float rounding only
    np.testing.assert_allclose(np.sort(und_full, axis=0), np.sort(und_roi, axis=0), rtol=0, atol=1e-4)
    inv = 255 - img  # dark markers on a bright background: THRESH_BINARY_INV with the mirrored threshold
    und_inv, _, _, _ = orc.find_leds(inv, K, D, threshold_value=14, active_markers=False)
    assert len(und_inv) == 5
