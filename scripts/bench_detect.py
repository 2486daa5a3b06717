"""Benchmark of the LED detector (led_detector.cpp:46-215): pfmpe_find_leds on a
device-resident 752x480 camera image (staged once: a camera DMA would land it there), full-image ROI and a
tracking-size ROI, against the CPU restatement (oracle/detect_oracle.cpp, 1 thread).  One JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import pf_monocular_pose_estimator_amd as pf  # noqa: E402
from pf_monocular_pose_estimator_amd import synthetic as syn  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    T = syn.truth_pose(0.5)
    img, ideal = syn.led_image(T, syn.markers_for(5), seed=1)
    eng = pf.Engine(device=0, max_particles=1000)
    eng.set_model(syn.markers_for(5), syn.K_README)
    eng.stage_image(img)
    x0, y0 = int(ideal[:, 0].min()) - 30, int(ideal[:, 1].min()) - 30
    roi = (x0, y0, int(ideal[:, 0].max()) + 30 - x0, int(ideal[:, 1].max()) + 30 - y0)
    res = {"metric": "LED detector frames/s (threshold + blur + contours + moments + undistort)", "unit": "frames/s",
           "image": [int(img.shape[1]), int(img.shape[0])], "roi_tracking": list(roi)}
    for name, r in (("full", None), ("roi", roi)):
        for _ in range(5):
            eng.find_leds(None, D=syn.D_README, roi=r)
        eng.set_option(pf.OPT_TIMING, 1)
        eng.reset_kernel_stats()
        t0 = time.perf_counter()
        for _ in range(reps):
            und, _, info = eng.find_leds(None, D=syn.D_README, roi=r)
        wall = (time.perf_counter() - t0) / reps
        n, ms = eng.kernel_stats()["k_det (detector pipeline)"]
        eng.set_option(pf.OPT_TIMING, 0)
        res[name] = {"wall_us": wall * 1e6, "device_us": ms / max(n, 1) * 1e3, "detections": int(len(und)),
                     "components": info["n_components"]}
    from oracle import pforacle as orc
    for name, r in (("full", None), ("roi", roi)):
        t0 = time.perf_counter()
        k = 5
        for _ in range(k):
            orc.find_leds(img, syn.K_README, syn.D_README, roi=r)
        res[name]["cpu_us"] = (time.perf_counter() - t0) / k * 1e6
    res["value"] = 1e6 / res["full"]["wall_us"]
    res["cpu_baseline"] = {"value": 1e6 / res["full"]["cpu_us"], "unit": "frames/s", "cores": 1, "kind": "port",
                           "sample": "5 full 752x480 frames, oracle/detect_oracle.cpp"}
    print(json.dumps(res))
    eng.close()


if __name__ == "__main__":
    main()
