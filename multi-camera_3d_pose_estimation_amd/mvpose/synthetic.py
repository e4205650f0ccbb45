"""Seeded synthetic multi-camera workloads (SURVEY.md §8(d) "Synthetic inputs").

There is no network and no recorded video on the GPU box, so every bench and
parity test draws its inputs from here:

* camera rigs: K with fx=fy=1000, cx=640, cy=360 for 1280x720 frames
  (reference examples/calibration_settings.yaml:1-2); camera 0 is the world
  origin (R=I, T=0, as setup_camera_configuration.py:392-393 writes it); the
  others sit on a circle around the subject, looking at it; Brown-Conrady
  distortion drawn from the ranges in SURVEY §8(d);
* poses: 17-joint COCO skeleton with the segment lengths of reference
  examples/body_part_lengths.yaml, root random walk, per-joint jitter;
* 2D keypoints: forward projection with the reference's own distortion model
  (pose_refinement.py:147-161) + N(0, 1 px) noise, confidence U(0.3, 1.0), in
  the reference layout (T, 17, 3, V) float32 (pose_estimation.py:135).

World units are cm (the reference's calibration units).
"""
from __future__ import annotations

import numpy as np
from scipy.signal import lfilter

FRAME_W, FRAME_H = 1280, 720
N_JOINTS = 17

# COCO joint template (cm, y down, z toward the cameras), pelvis at the origin.
_TEMPLATE = np.array([
    [0.0, -80.0, -8.0],    # 0 nose
    [-3.0, -83.0, -6.0],   # 1 left_eye
    [3.0, -83.0, -6.0],    # 2 right_eye
    [-7.0, -81.0, 0.0],    # 3 left_ear
    [7.0, -81.0, 0.0],     # 4 right_ear
    [-23.0, -54.0, 0.0],   # 5 left_shoulder
    [23.0, -54.0, 0.0],    # 6 right_shoulder
    [-25.0, -16.0, 0.0],   # 7 left_elbow
    [25.0, -16.0, 0.0],    # 8 right_elbow
    [-26.0, 11.0, 0.0],    # 9 left_wrist
    [26.0, 11.0, 0.0],     # 10 right_wrist
    [-15.5, 0.0, 0.0],     # 11 left_hip
    [15.5, 0.0, 0.0],      # 12 right_hip
    [-15.5, 51.0, 0.0],    # 13 left_knee
    [15.5, 51.0, 0.0],     # 14 right_knee
    [-15.5, 91.0, 0.0],    # 15 left_ankle
    [15.5, 91.0, 0.0],     # 16 right_ankle
])

SUBJECT_CENTER = np.array([0.0, 0.0, 350.0])


def _look_at(pos, target):
    z = target - pos
    z = z / np.linalg.norm(z)
    up = np.array([0.0, 1.0, 0.0])
    x = np.cross(up, z)
    x = x / np.linalg.norm(x)
    y = np.cross(z, x)
    R = np.stack([x, y, z])  # world -> camera rows
    T = -R @ pos
    return R, T.reshape(3, 1)


def make_rig(n_cams: int, seed: int = 0, distortion: bool = True):
    """Returns a list of dicts {K (3,3), R (3,3), T (3,1), dist (1,5)} float64."""
    rng = np.random.default_rng(seed)
    cams = []
    for v in range(n_cams):
        K = np.array([[1000.0, 0.0, 640.0], [0.0, 1000.0, 360.0], [0.0, 0.0, 1.0]])
        if v == 0:
            R, T = np.eye(3), np.zeros((3, 1))
        else:
            th = np.deg2rad(35.0 * v + rng.uniform(-5.0, 5.0))
            pos = SUBJECT_CENTER + 300.0 * np.array([np.sin(th), rng.uniform(-0.15, 0.15), -np.cos(th)])
            R, T = _look_at(pos, SUBJECT_CENTER)
        if distortion:
            dist = np.array([[rng.uniform(-0.1, 0.1), rng.uniform(-0.05, 0.05),
                              rng.uniform(-1e-3, 1e-3), rng.uniform(-1e-3, 1e-3),
                              rng.uniform(-0.02, 0.02)]])
        else:
            dist = np.zeros((1, 5))
        cams.append({"K": K, "R": R, "T": T, "dist": dist})
    return cams


def make_poses(n_frames: int, seed: int = 0, jitter: float = 5.0):
    """(T, 17, 3) float64 world-space poses (cm)."""
    rng = np.random.default_rng(seed)
    # mean-reverting (AR(1)) root walk: stays within ~+-40 cm of the subject centre
    # for any sequence length, so long benches keep the same geometry
    steps = rng.normal(0.0, 2.0, (n_frames, 3)) * np.array([1.0, 0.2, 1.0])
    root = SUBJECT_CENTER + lfilter([1.0], [1.0, -0.98], steps, axis=0)
    yaw = lfilter([1.0], [1.0, -0.995], rng.normal(0.0, 0.02, n_frames))
    out = np.empty((n_frames, N_JOINTS, 3))
    for t in range(n_frames):
        c, s = np.cos(yaw[t]), np.sin(yaw[t])
        Ry = np.array([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]])
        out[t] = _TEMPLATE @ Ry.T + root[t] + rng.normal(0.0, jitter, (N_JOINTS, 3))
    return out


def project(points, cam, distortion: bool = True):
    """Reference forward model (pose_refinement.py:94-179) in fp64 numpy.
    points (..., 3) -> (..., 2) pixels."""
    X = np.asarray(points, dtype=np.float64)
    pc = X @ cam["R"].T + cam["T"].reshape(3)
    x = pc[..., 0] / pc[..., 2]
    y = pc[..., 1] / pc[..., 2]
    if distortion:
        k1, k2, p1, p2, k3 = cam["dist"].ravel()
        r2 = x * x + y * y
        radial = 1 + k1 * r2 + k2 * r2 ** 2 + k3 * r2 ** 3
        xd = x * radial + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
        yd = y * radial + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
        x, y = xd, yd
    K = cam["K"]
    u = K[0, 0] * x + K[0, 1] * y + K[0, 2]
    v = K[1, 1] * y + K[1, 2]
    return np.stack([u, v], axis=-1)


def make_kpts_2d(poses, cams, seed: int = 0, noise_px: float = 1.0, conf_range=(0.3, 1.0)):
    """(T, 17, 3, V) float32 in the reference layout (pose_estimation.py:135)."""
    rng = np.random.default_rng(seed)
    T, J, _ = poses.shape
    V = len(cams)
    out = np.empty((T, J, 3, V), np.float32)
    for v, cam in enumerate(cams):
        uv = project(poses, cam) + rng.normal(0.0, noise_px, (T, J, 2))
        out[:, :, 0, v] = uv[..., 0]
        out[:, :, 1, v] = uv[..., 1]
        out[:, :, 2, v] = rng.uniform(conf_range[0], conf_range[1], (T, J))
    return out


def reference_camera_params(cams):
    """{idx: [K, R, T, dist]} — the structure utils.get_params_from_name returns
    (reference utils.py:807-828) and get_pose_3D consumes."""
    return {i: [c["K"], c["R"], c["T"], c["dist"]] for i, c in enumerate(cams)}


def make_frames(n: int, seed: int = 0, h: int = FRAME_H, w: int = FRAME_W):
    """(n, H, W, 3) uint8 uniform random frames."""
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, (n, h, w, 3), dtype=np.uint8)


# ------------------------------------------------------------- rendered people --
# Colour per COCO joint pair (nose alone): a joint and its left / right partner share a
# colour and the subject's LEFT joint is the one further right in the image (a frontal
# person), so the flip test's left/right swap is consistent with what the picture shows.
_PAIR_COLORS = np.array([[230, 40, 40], [40, 220, 40], [50, 80, 240], [235, 225, 40], [225, 50, 220],
                         [40, 220, 225], [245, 245, 245], [245, 140, 30], [140, 60, 200]], np.uint8)
_PAIR_OF_JOINT = np.array([0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8])
HEATMAP_OFFSET = (0.0, 0.25)   # sub-cell (x, y) position of the rendered joints on the heatmap grid


def _whole_image_heatmap_to_image(h: int, w: int):
    """(scale, offset) of the whole-image crop's heatmap -> image map (mmpose restore:
    kp / input_size * scale + center - scale / 2 with kp = 4 * heatmap cell)."""
    sw, sh = 1.25 * w, 1.25 * h
    sw, sh = (sw, sw / 0.75) if sw > sh * 0.75 else (sh * 0.75, sh)
    return np.array([sw / 48.0, sh / 64.0]), np.array([w / 2.0 - sw / 2.0, h / 2.0 - sh / 2.0])


def skeleton_layout(rng, h: int = FRAME_H, w: int = FRAME_W, min_dist: float = 3.0):
    """17 joint positions on the heatmap grid of the whole-image crop (cells + HEATMAP_OFFSET),
    inside the frame, pairwise >= min_dist cells apart, each left joint 2-7 cells to the
    image right of its right partner."""
    k, off = _whole_image_heatmap_to_image(h, w)
    lo = np.ceil((np.array([40.0, 40.0]) - off) / k).astype(int)
    hi = np.floor((np.array([w - 40.0, h - 40.0]) - off) / k).astype(int)
    for _ in range(1000):
        pts = np.zeros((N_JOINTS, 2))
        placed = []
        ok = True
        for j in [0] + list(range(2, N_JOINTS, 2)):      # the nose, then each right joint with its left partner
            for _try in range(200):
                p = rng.integers(lo, hi + 1).astype(float)
                cand = [p]
                if j > 0:
                    q = p + np.array([rng.integers(2, 8), rng.integers(-2, 3)])
                    if not ((lo <= q).all() and (q <= hi).all()):
                        continue
                    cand.append(q)
                if all(np.hypot(*(c - d)) >= min_dist for c in cand for d in placed):
                    break
            else:
                ok = False
                break
            placed += cand
            if j == 0:
                pts[0] = p
            else:
                pts[j], pts[j - 1] = p, cand[1]              # right joint j, left joint j - 1 (to its image right)
        if ok:
            return pts + np.array(HEATMAP_OFFSET)
    raise RuntimeError("skeleton_layout: no layout found")


def make_skeleton_frames(n: int, seed: int = 0, h: int = FRAME_H, w: int = FRAME_W, radius: float = 0.9):
    """(frames (n, H, W, 3) uint8, joints (n, 17, 2) heatmap-grid cells of the whole-image crop):
    dark noisy backgrounds with one coloured disc per COCO joint (radius in heatmap cells), laid
    out by skeleton_layout.  The test / training input for weights with trained-model-like
    peaked heatmaps (tools/train_peaked_hrnet.py, tests/test_e2e_parity_gpu.py)."""
    rng = np.random.default_rng(seed)
    k, off = _whole_image_heatmap_to_image(h, w)
    frames = np.empty((n, h, w, 3), np.uint8)
    joints = np.empty((n, N_JOINTS, 2))
    ys, xs = np.mgrid[0:h, 0:w].astype(np.float32)
    for i in range(n):
        base = rng.integers(20, 90, 3).astype(np.int16)
        img = (base + rng.integers(-10, 11, (h, w, 3), dtype=np.int16)).astype(np.uint8)   # 10..99: no clipping
        cells = skeleton_layout(rng, h, w)
        # the crop samples pixel centres: heatmap position c <-> image coordinate c * k + off
        centers = cells * k + off
        r = radius * k[0]
        for j in range(N_JOINTS):
            cx, cy = centers[j]
            x0, x1 = int(max(0, cx - r - 1)), int(min(w, cx + r + 2))
            y0, y1 = int(max(0, cy - r - 1)), int(min(h, cy + r + 2))
            m = (xs[y0:y1, x0:x1] - cx) ** 2 + (ys[y0:y1, x0:x1] - cy) ** 2 <= r * r
            col = np.clip(_PAIR_COLORS[_PAIR_OF_JOINT[j]].astype(np.int16) + rng.integers(-8, 9, 3), 0, 255)
            img[y0:y1, x0:x1][m] = col.astype(np.uint8)
        frames[i] = img
        joints[i] = cells
    return frames, joints
