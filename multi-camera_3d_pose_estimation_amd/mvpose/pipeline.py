"""Multi-view 2D -> 3D pipeline on one GPU: the reference's
estimate_pose_from_video / run_pose_est / get_pose_2D / get_pose_3D loop
(pose_estimation.py:157-327) for a whole batch of synchronised frames at once.

process(frames (T, V, H, W, 3) uint8 on GPU) returns, device-resident:
    kpts_2d     (T, 17, 3, V) float32   [x, y, score] per camera   (pose_estimation.py:135)
    heatmaps_2d (T, V, 17, 6) float64   [mx, my, vxx, vxy, vxy, vyy] (mmpose_pose_estimation.py:208-210)
    kpts_3d     (T, 17, 3)    float32   triangulated                 (pose_estimation.py:319-322)

process(..., overlap_moments=True) computes heatmaps_2d on a side stream beside the
next batch's backbone (triangulation reads only kpts_2d); call wait(out) before reading
heatmaps_2d on the current stream.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops
from .estimator import BatchPoseEstimator
from .hrnet import N_JOINTS


class MultiViewPipeline:
    def __init__(self, camera_params, estimator: BatchPoseEstimator | None = None, camera_indices=(0, 1),
                 mode: int = ops.TRI_REFERENCE, device="cuda", detector=None, bbox_thr: float = 0.3,
                 tri_solver: str = "tolerance", **estimator_kw):
        """camera_params: {camera key: [K, R, T, dist]} (utils.get_params_from_name order),
        keys 0..V-1 as the reference assumes (pose_estimation.py:276-280).
        detector: an mvpose.rtmdet.RTMDetector run on every camera-frame before the crops
        (PoseEstimator.predict, mmpose_pose_estimation.py:234-250: its first person box with
        score > bbox_thr, else the whole image), or None (whole-image crops).
        tri_solver: "tolerance" (default: MVP_TRI_TOLERANCE, <= 1e-4 world units against
        OpenCV's rounding sequence, bit-identical on almost every point) or "reference_compat"
        (OpenCV 4.9's fp64 rounding sequence, QR + inverse iteration with the Jacobi
        restatement where that has not converged)."""
        if tri_solver not in ("tolerance", "reference_compat"):
            raise ValueError(f"tri_solver {tri_solver!r}: 'tolerance' or 'reference_compat'")
        self.tri_solver = tri_solver
        self.detector = detector
        self.bbox_thr = bbox_thr
        self._best = None
        self.device = torch.device(device)
        self.n_views = len(camera_params)
        self.cams = torch.tensor(ops.pack_cameras(camera_params), device=self.device)
        self.camera_indices = list(camera_indices)
        self.mode = mode
        self.estimator = estimator or BatchPoseEstimator(device=device, **estimator_kw)

    @property
    def max_frames(self) -> int:
        return self.estimator.max_frames // self.n_views

    def process(self, frames: torch.Tensor, out: dict | None = None, overlap_moments: bool = False,
                bboxes=None) -> dict:
        """bboxes: None (the detector's boxes, or whole-image crops without one), host (T, V, 4)
        xyxy person boxes (NaN row = none), or device rows (T, V, >=4) f32 used as given."""
        T, V = frames.shape[:2]
        if V != self.n_views:
            raise ValueError(f"frames carry {V} views, pipeline has {self.n_views} cameras")
        flat = frames.reshape(T * V, *frames.shape[2:])
        if out is None:
            out = {}
        if "kpts_2d" not in out or tuple(out["kpts_2d"].shape) != (T, N_JOINTS, 3, V):
            out["kpts_2d"] = torch.empty((T, N_JOINTS, 3, V), dtype=torch.float32, device=self.device)
            out.pop("kpts_3d", None)
        thr = None
        if bboxes is None and self.detector is not None:
            bb, thr = self.detect(flat), self.bbox_thr       # device rows: no host round trip
        elif isinstance(bboxes, torch.Tensor) and bboxes.is_cuda:
            bb = bboxes.reshape(T * V, -1)
        else:
            bb = None if bboxes is None else np.asarray(bboxes, np.float64).reshape(T * V, 4)
        r = self.estimator.run(flat, n_views=V, kpts_tkv=out["kpts_2d"], overlap_moments=overlap_moments, bboxes=bb,
                               bbox_thr=thr)
        out["heatmaps_2d"] = r["gaussians"].reshape(T, V, N_JOINTS, 6)
        if r["moments_done"] is not None:
            out["moments_done"] = r["moments_done"]
        else:
            out.pop("moments_done", None)
        out["kpts_3d"] = ops.triangulate(out["kpts_2d"], self.cams, self.camera_indices, mode=self.mode,
                                         out=out.get("kpts_3d"), tolerance=self.tri_solver == "tolerance")
        return out

    def detect(self, flat: torch.Tensor) -> torch.Tensor:
        """(T*V, H, W, 3) camera-frames -> the detector's per-frame best rows (T*V, 6) f32 on the
        device {x1, y1, x2, y2, score, prior}; BatchPoseEstimator.run applies score > bbox_thr
        and derives the crops there (mvp_bbox_geometry)."""
        n = flat.shape[0]
        if self._best is None or self._best.shape[0] < n:
            self._best = torch.empty((n, 6), dtype=torch.float32, device=self.device)
        mb = self.detector.max_batch
        for i in range(0, n, mb):
            self.detector.detect(flat[i:i + mb], best_out=self._best[i:min(n, i + mb)])
        return self._best[:n]

    @staticmethod
    def wait(out: dict) -> None:
        """Order the current stream after an overlapped process()'s heatmaps_2d."""
        BatchPoseEstimator.wait_moments(out)

    def process_stream(self, frames: torch.Tensor, bboxes=None) -> dict:
        """Arbitrary-length sequence (T, V, H, W, 3): chunked to the estimator's batch."""
        T = frames.shape[0]
        step = self.max_frames
        parts = [self.process(frames[t:t + step], bboxes=None if bboxes is None else bboxes[t:t + step])
                 for t in range(0, T, step)]
        return {k: torch.cat([p[k] for p in parts]) for k in parts[0]}
