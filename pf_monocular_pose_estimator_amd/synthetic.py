"""Synthetic camera streams for the PF step: README intrinsics and markers, a smooth
6-DoF trajectory at 50 fps, undistorted blob lists with noise, occlusions and outliers.

There are no recorded bags in the reference tree, so every benchmark and end-to-end test
input is generated here from fixed seeds.  Outlier recipes mimic the reference's fault injection
(LEDDetector::occludeDetections / insertFalseDetections, pf_mpe_lib/src/led_detector.cpp:417-488).
Blob coordinates are rounded to float32 because the reference's detector hands over cv::Point2f
(led_detector.cpp:192-209).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

# README.md:137-141 (mvBlueFOX 752x480 plumb_bob calibration)
IMAGE_W, IMAGE_H = 752, 480
K_README = np.array([[475.4220992391843, 0.0, 378.1094270899403],
                     [0.0, 475.6638941565314, 236.6226272309063],
                     [0.0, 0.0, 1.0]])
D_README = np.array([-0.2987656130625547, 0.090512327786479, 0.0006983134447049677, 0.0004069824038616868, 0.0])

# README.md:102-117 marker_positions (5 LEDs)
MARKERS_5 = np.array([[0.0, 0.0, 0.0], [0.004, -0.188, 0.039], [0.228, -0.140, 0.0],
                      [0.264, 0.124, 0.0], [0.076, 0.128, 0.005]])
# pf_mpe/marker_positions/demo_marker_positions.yaml:4-15 (4 LEDs)
MARKERS_DEMO = np.array([[0.0714197, 0.0800214, 0.0622611], [0.0400755, -0.0912328, 0.0317064],
                         [-0.0647293, -0.0879977, 0.0830852], [-0.0558663, -0.0165446, 0.053473]])


def markers_12() -> np.ndarray:
    """12 LEDs: the 5 README LEDs + the 4 demo LEDs + 3 drawn with default_rng(12) in [-0.15, 0.3]^3
    with >= 3 cm separation (there is no 12-LED file in the reference tree)."""
    pts = [p for p in MARKERS_5] + [p for p in MARKERS_DEMO]
    rng = np.random.default_rng(12)
    while len(pts) < 12:
        c = rng.uniform(-0.15, 0.3, size=3)
        if min(np.linalg.norm(c - p) for p in pts) >= 0.03:
            pts.append(c)
    return np.array(pts)


# ------------------------------------------------------------------------------------------ SE(3)
def rot_x(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])


def rot_y(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def rot_z(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def to12(T: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(T, np.float64)[:3, :4].reshape(12))


def to44(p12) -> np.ndarray:
    T = np.eye(4)
    T[:3, :4] = np.asarray(p12, np.float64).reshape(3, 4)
    return T


def skew(w):
    return np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])


def se3_exp(xi) -> np.ndarray:
    """Twist (upsilon, omega) -> 4x4 (same closed form as PoseEstimator::exponentialMap, PE:2194)."""
    ups, om = np.asarray(xi[:3], float), np.asarray(xi[3:], float)
    th = np.linalg.norm(om)
    O = skew(om)
    if th == 0:
        R, V = np.eye(3), np.eye(3)
    else:
        R = np.eye(3) + O / th * np.sin(th) + O @ O / th**2 * (1 - np.cos(th))
        V = np.eye(3) + (1 - np.cos(th)) / th**2 * O + (th - np.sin(th)) / th**3 * O @ O
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = V @ ups
    return T


def se3_log(T) -> np.ndarray:
    R, t = T[:3, :3], T[:3, 3]
    c = np.clip((np.trace(R) - 1) / 2, -1, 1)
    phi = np.arccos(c)
    if phi < 1e-12:
        W = np.zeros((3, 3))
    else:
        W = (R - R.T) / (2 * np.sin(phi)) * phi
    w = np.array([W[2, 1], W[0, 2], W[1, 0]])
    wn = np.linalg.norm(w)
    if wn < 1e-12:
        Ainv = np.eye(3)
    else:
        Ainv = np.eye(3) - W / 2 + (2 * np.sin(wn) - wn * (1 + np.cos(wn))) / (2 * wn**2 * np.sin(wn)) * W @ W
    return np.concatenate([Ainv @ t, w])


def rigid_inv(T):
    Ti = np.eye(4)
    Ti[:3, :3] = T[:3, :3].T
    Ti[:3, 3] = -T[:3, :3].T @ T[:3, 3]
    return Ti


def project(K, T, X) -> np.ndarray:
    """Pinhole projection of object points X (M x 3) through T (camera<-object) and K (PE:1017)."""
    Xc = (T[:3, :3] @ np.asarray(X).T).T + T[:3, 3]
    p = (K @ Xc.T).T
    return p[:, :2] / p[:, 2:3]


# ------------------------------------------------------------------------------------ trajectory
def truth_pose(t: float) -> np.ndarray:
    """Smooth bounded 6-DoF motion in front of the camera (speed ~0.3-0.5 m/s, ~0.2-0.4 rad/s)."""
    T = np.eye(4)
    T[:3, :3] = rot_z(0.3 + 0.3 * np.sin(0.8 * t)) @ rot_y(0.2 * np.sin(0.6 * t)) @ rot_x(0.1 + 0.2 * np.sin(0.7 * t))
    T[:3, 3] = [0.05 + 0.25 * np.sin(1.3 * t) - 0.1, -0.02 + 0.15 * np.sin(1.7 * t) - 0.05, 2.0 + 0.3 * np.sin(0.9 * t)]
    return T


@dataclass
class StreamConfig:
    name: str
    M: int
    B: int
    N: int
    heavy: bool = False          # C3 recipe: occlusion + 50% near-blob outliers
    noise_px: float = 0.3
    dt: float = 0.02             # 50 fps (pf_mpe/launch/LaunchIrchelExperiments.launch:40)
    seed: int = 0


CONFIGS = {
    "C1": StreamConfig("C1", M=5, B=20, N=1000),
    "C2": StreamConfig("C2", M=5, B=50, N=100_000),
    "C3": StreamConfig("C3", M=12, B=200, N=1_000_000, heavy=True),
    "C4": StreamConfig("C4", M=5, B=50, N=10_000_000),
    # BASELINE.json configs[4]: 8 independent camera streams x 1M particles, one stream per GPU (the
    # per-rank workload of `bench.py --gpus N`; stream seed = rank)
    "C5": StreamConfig("C5", M=5, B=50, N=1_000_000),
}


def markers_for(M: int) -> np.ndarray:
    if M == 5:
        return MARKERS_5.copy()
    if M == 12:
        return markers_12()
    if M <= 5:
        return MARKERS_5[:M].copy()
    return markers_12()[:M].copy()


def blobs_for_frame(cfg: StreamConfig, T: np.ndarray, frame: int, markers: np.ndarray) -> np.ndarray:
    rng = np.random.default_rng(1000 + frame + 7919 * cfg.seed)
    true_px = project(K_README, T, markers) + rng.normal(0.0, cfg.noise_px, size=(len(markers), 2))
    blobs = list(true_px)
    if cfg.heavy and len(blobs) > 0:
        blobs.pop(int(rng.integers(0, len(blobs))))  # one occlusion (led_detector.cpp:432-451)
    n_out = max(0, cfg.B - len(blobs))
    if cfg.heavy:
        n_near = n_out // 2
        for _ in range(n_near):  # 1-5 px from a random true blob (led_detector.cpp:475-484)
            base = true_px[int(rng.integers(0, len(true_px)))]
            off = rng.integers(1, 6, size=2) * rng.choice([-1, 1], size=2)
            blobs.append(base + off)
        n_out -= n_near
    for _ in range(n_out):
        blobs.append(np.array([rng.uniform(0, IMAGE_W), rng.uniform(0, IMAGE_H)]))
    blobs = np.array(blobs[: cfg.B]) if len(blobs) else np.zeros((0, 2))
    rng.shuffle(blobs)
    return blobs.astype(np.float32).astype(np.float64)


def initial_prior(T: np.ndarray, N: int, seed: int = 7, ang=0.015, trans=0.035) -> np.ndarray:
    """Truth (+) U(+-ang rad, +-trans m) per particle."""
    rng = np.random.default_rng(seed)
    a = rng.uniform(-ang, ang, size=(N, 3))
    d = rng.uniform(-trans, trans, size=(N, 3))
    out = np.empty((N, 12))
    R0, t0 = T[:3, :3], T[:3, 3]
    for n in range(N):
        R = R0 @ rot_z(a[n, 2]) @ rot_y(a[n, 1]) @ rot_x(a[n, 0])
        out[n, [0, 1, 2]] = R[0]
        out[n, [4, 5, 6]] = R[1]
        out[n, [8, 9, 10]] = R[2]
        out[n, [3, 7, 11]] = t0 + d[n]
    return out


def initial_prior_fast(T: np.ndarray, N: int, seed: int = 7, ang=0.015, trans=0.035) -> np.ndarray:
    """Vectorised initial_prior for large N (identical distribution, different float order)."""
    rng = np.random.default_rng(seed)
    a = rng.uniform(-ang, ang, size=(N, 3))
    d = rng.uniform(-trans, trans, size=(N, 3))
    cx, sx = np.cos(a[:, 0]), np.sin(a[:, 0])
    cy, sy = np.cos(a[:, 1]), np.sin(a[:, 1])
    cz, sz = np.cos(a[:, 2]), np.sin(a[:, 2])
    Rz = np.zeros((N, 3, 3)); Rz[:, 0, 0] = cz; Rz[:, 0, 1] = -sz; Rz[:, 1, 0] = sz; Rz[:, 1, 1] = cz; Rz[:, 2, 2] = 1
    Ry = np.zeros((N, 3, 3)); Ry[:, 0, 0] = cy; Ry[:, 0, 2] = sy; Ry[:, 2, 0] = -sy; Ry[:, 2, 2] = cy; Ry[:, 1, 1] = 1
    Rx = np.zeros((N, 3, 3)); Rx[:, 1, 1] = cx; Rx[:, 1, 2] = -sx; Rx[:, 2, 1] = sx; Rx[:, 2, 2] = cx; Rx[:, 0, 0] = 1
    R = T[:3, :3][None] @ Rz @ Ry @ Rx
    out = np.empty((N, 3, 4))
    out[:, :, :3] = R
    out[:, :, 3] = T[:3, 3][None] + d
    return out.reshape(N, 12)


@dataclass
class Frame:
    index: int
    time: float
    truth: np.ndarray          # 4x4
    current_pose: np.ndarray   # 12 (previous frame's estimate; here truth of the previous frame)
    predicted_pose: np.ndarray # 12
    prediction: np.ndarray     # 12
    blobs: np.ndarray          # B x 2
    dt: float


@dataclass
class Stream:
    cfg: StreamConfig
    markers: np.ndarray
    K: np.ndarray
    frames: list = field(default_factory=list)

    def prior(self, N=None, fast=None) -> np.ndarray:
        N = N or self.cfg.N
        # the prior is last frame's resampled set: centred on the previous pose of frame 0
        T0 = to44(self.frames[0].current_pose) if self.frames else truth_pose(0.0)
        if fast or N > 20000:
            return initial_prior_fast(T0, N)
        return initial_prior(T0, N)


def make_stream(cfg: StreamConfig, n_frames: int, t0: float = 0.5) -> Stream:
    """Per-frame host inputs as the tracker would produce them: current_pose = previous estimate
    (truth of the previous frame), prediction = constant-velocity extrapolation from the two previous
    estimates (predictPose, PE:995-1010), predicted = current * prediction."""
    markers = markers_for(cfg.M)
    st = Stream(cfg, markers, K_README.copy())
    dt = cfg.dt
    for f in range(n_frames):
        t = t0 + (f + 1) * dt
        T = truth_pose(t)
        Tc = truth_pose(t - dt)
        Tp = truth_pose(t - 2 * dt)
        delta = se3_log(rigid_inv(Tp) @ Tc) / dt * dt
        Pm = se3_exp(delta)
        st.frames.append(Frame(f, t, T, to12(Tc), to12(Tc @ Pm), to12(Pm), blobs_for_frame(cfg, T, f, markers), dt))
    return st


def init_blobs(M: int = 5, n_out: int = 3, seed: int = 0, noise_px: float = 0.0, t: float = 0.5,
               near: int = 0):
    """Detections of a track-loss frame for the brute-force initialisation (PE:1503): every marker at
    truth_pose(t) (+ N(0, noise_px)), `near` outliers 1-5 px from true blobs, `n_out` uniform outliers,
    shuffled and rounded through float32 like detector output.  Returns (blobs B x 2, truth 4x4)."""
    rng = np.random.default_rng(5000 + seed)
    T = truth_pose(t)
    markers = markers_for(M)
    px = project(K_README, T, markers) + (rng.normal(0.0, noise_px, size=(M, 2)) if noise_px > 0 else 0.0)
    blobs = list(px)
    for _ in range(near):
        base = px[int(rng.integers(0, M))]
        blobs.append(base + rng.integers(1, 6, size=2) * rng.choice([-1, 1], size=2))
    for _ in range(n_out):
        blobs.append(np.array([rng.uniform(0, IMAGE_W), rng.uniform(0, IMAGE_H)]))
    blobs = np.array(blobs)
    rng.shuffle(blobs)
    return blobs.astype(np.float32).astype(np.float64), T


def distort_px(K, D, uv: np.ndarray) -> np.ndarray:
    """plumb_bob distortion of ideal pixel positions (what the camera sees)."""
    k1, k2, p1, p2, k3 = D
    x = (uv[:, 0] - K[0, 2]) / K[0, 0]
    y = (uv[:, 1] - K[1, 2]) / K[1, 1]
    r2 = x * x + y * y
    rad = 1 + k1 * r2 + k2 * r2 * r2 + k3 * r2 ** 3
    xd = x * rad + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * rad + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    return np.stack([xd * K[0, 0] + K[0, 2], yd * K[1, 1] + K[1, 2]], axis=1)


def led_image(T: np.ndarray, markers: np.ndarray, seed: int = 0, radius: float = 3.2, n_false: int = 3,
              W: int = IMAGE_W, H: int = IMAGE_H, noise: int = 60):
    """An 8-bit camera image of the LED object at pose T (LEDDetector::findLeds input, led_detector.cpp:46):
    saturated discs (radius px, soft 1-px edge) at the DISTORTED projections of the markers, `n_false`
    bright distractors (discs and an elongated bar), uniform background noise.  Returns (image H x W
    uint8, ideal undistorted projections M x 2)."""
    rng = np.random.default_rng(9000 + seed)
    img = rng.integers(0, noise + 1, size=(H, W)).astype(np.float64)
    ideal = project(K_README, T, markers)
    centres = list(distort_px(K_README, D_README, ideal))
    while len(centres) < len(ideal) + n_false:  # distractors >= 20 px from every LED (no merged blobs)
        c = np.array([rng.uniform(20, W - 20), rng.uniform(20, H - 20)])
        if min(np.hypot(*(c - q)) for q in centres) >= 20:
            centres.append(c)
    yy, xx = np.mgrid[0:H, 0:W]
    for i, (cx, cy) in enumerate(centres):
        d = np.hypot(xx - cx, yy - cy)
        spot = np.clip(radius + 1.0 - d, 0.0, 1.0) * 255.0
        img = np.maximum(img, spot)
    if n_false:
        for _ in range(100):
            x0, y0 = int(rng.uniform(40, W - 80)), int(rng.uniform(40, H - 40))
            if min(np.hypot(*(np.array([x0 + 15, y0 + 1]) - q)) for q in centres) >= 35:
                break
        img[y0:y0 + 3, x0:x0 + 30] = 255.0  # elongated: fails the aspect filter
    return np.clip(np.rint(img), 0, 255).astype(np.uint8), ideal
