"""GPU drop-ins for the reference's utils.py functions on the hot path.

* ``triangulate_points(kpts_2d, cmtx1, dist1, R1, T1, cmtx2, dist2, R2, T2)``
  (utils.py:1277-1336): cv.undistortPoints x 2 + cv.triangulatePoints +
  cv.convertPointsFromHomogeneous for any leading shape (..., 2 cameras, 2) -> (..., 3),
  as ONE mvp_triangulate launch (OpenCV 4.9 numerics restated in fp64, f32 out).
* the calibration readers (utils.py:750-828) and the frame loader (:849-909) the
  pipeline uses, re-exported from mvpose.geometry / mvpose.pose_estimation.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops
from .geometry import (get_params_from_name, projection_matrix as calculate_projection_matrix,  # noqa: F401
                       read_camera_parameters, read_rotation_translation)
from .pose_estimation import load_frames  # noqa: F401


def to_numpy(arr):
    """utils.py:1272-1273."""
    return arr if isinstance(arr, np.ndarray) else np.asarray(arr.detach().cpu() if torch.is_tensor(arr) else arr)


def triangulate_points(kpts_2d, cmtx1, dist1, R1, T1, cmtx2, dist2, R2, T2, device=None):
    """kpts_2d (..., 2, 2): [camera][x, y] -> (..., 3) numpy in the keypoints' precision, as
    OpenCV keeps it: float64 keypoints (the extrinsic branch's samples, pose_refinement.py:811)
    stay float64 end to end (mvp_triangulate_points_f64), anything else is taken as float32
    (the pipeline's keypoint dtype).  Camera 1's rows of the DLT system come first, as in
    cv.triangulatePoints(P1, P2, ...)."""
    k_in = np.asarray(to_numpy(kpts_2d))
    dev = torch.device(device if device is not None else "cuda")
    cams = ops.pack_cameras([[to_numpy(cmtx1), to_numpy(R1), to_numpy(T1), to_numpy(dist1)],
                             [to_numpy(cmtx2), to_numpy(R2), to_numpy(T2), to_numpy(dist2)]])
    if k_in.dtype == np.float64:
        if k_in.shape[-2:] != (2, 2):
            raise ValueError(f"kpts_2d must have shape (..., 2, 2), got {k_in.shape}")
        if k_in.size == 0:
            return np.zeros(k_in.shape[:-2] + (3,), np.float64)
        out = ops.triangulate_points_f64(torch.from_numpy(np.ascontiguousarray(k_in)).to(dev),
                                         torch.from_numpy(cams).to(dev))
        return out.cpu().numpy()
    k = k_in.astype(np.float32)
    if k.shape[-2:] != (2, 2):
        raise ValueError(f"kpts_2d must have shape (..., 2, 2), got {k.shape}")
    lead = k.shape[:-2]
    flat = k.reshape(-1, 2, 2)
    n = flat.shape[0]
    # the kernel's reference layout (n, 3, V): rows x, y, confidence; equal confidences keep
    # the camera order [0, 1] (np.argsort of a tie), i.e. (cmtx1, ...) first
    kt = np.empty((n, 3, 2), np.float32)
    kt[:, 0, :] = flat[:, :, 0]
    kt[:, 1, :] = flat[:, :, 1]
    kt[:, 2, :] = 1.0
    if n == 0:
        return np.zeros(lead + (3,), np.float32)
    out = ops.triangulate(torch.from_numpy(kt).to(dev), torch.from_numpy(cams).to(dev), [0, 1])
    return out.cpu().numpy().reshape(lead + (3,))
