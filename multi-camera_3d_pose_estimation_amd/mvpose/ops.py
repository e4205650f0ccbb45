"""torch-tensor front of the libmvpose C-ABI.

Device tensors are handed over as raw pointers with the current HIP stream;
the library enqueues stream-ordered kernels.  Shapes and dtypes are checked
here before any launch (the kernels assume them).
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np
import torch

from . import _lib
from ._lib import call

CAM_DOUBLES = 40
TRI_REFERENCE = 0
TRI_ALL_VIEWS = 1
TRI_EXACT_JACOBI = 0x10  # mode flag: exact Jacobi SVD for every point (mvpose.h)
TRI_TOLERANCE = 0x20     # mode flag: throughput solver validated to <= 1e-4 world units (mvpose.h)


def _stream(device=None) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _ptr(t: torch.Tensor) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())


def _require(t: torch.Tensor, dtype, name: str):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name} must live on the GPU (no CPU fallback)")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def pack_camera(K, R, T, dist) -> np.ndarray:
    """One MVP_CAM_DOUBLES record: [K | dist | R | T | P | pad] with
    P = np.dot(K, hstack(R, T)) exactly as reference utils.py:1318-1319 — in the parameters'
    own dtype (float32 camera tensors give the reference a float32 P, e.g. the extrinsic
    branch's decomposed parameters, pose_refinement.py:808-811), stored as float64."""
    P = np.dot(np.asarray(K), np.hstack((np.asarray(R), np.asarray(T).reshape(-1, 1))))
    K = np.asarray(K, dtype=np.float64).reshape(3, 3)
    R = np.asarray(R, dtype=np.float64).reshape(3, 3)
    T = np.asarray(T, dtype=np.float64).reshape(3, 1)
    d = np.zeros(5)
    dd = np.asarray(dist, dtype=np.float64).ravel()
    d[: min(5, dd.size)] = dd[:5]
    if dd.size > 5 and np.any(dd[5:] != 0):
        raise ValueError("only the 5-coefficient Brown-Conrady model is supported (reference calibration)")
    rec = np.zeros(CAM_DOUBLES)
    rec[0:9] = K.ravel()
    rec[9:14] = d
    rec[14:23] = R.ravel()
    rec[23:26] = T.ravel()
    rec[26:38] = np.asarray(P, dtype=np.float64).ravel()
    return rec


def pack_cameras(camera_params) -> np.ndarray:
    """camera_params: {idx: [K, R, T, dist]} (utils.get_params_from_name order) or a
    list of such lists, ordered by camera key.  Returns (n, 40) float64."""
    if isinstance(camera_params, dict):
        items = [camera_params[k] for k in camera_params]
    else:
        items = list(camera_params)
    return np.stack([pack_camera(K, R, T, dist) for (K, R, T, dist) in items])


def triangulate(kpts: torch.Tensor, cams: torch.Tensor, cam_idx: Sequence[int] = (0, 1),
                mode: int = TRI_REFERENCE, out: torch.Tensor | None = None,
                return_xyzw: bool = False, exact: bool = False, tolerance: bool = False):
    """kpts (..., 3, V) float32 on GPU (reference layout) -> (..., 3) float32.

    cams: (n_cams, 40) float64 on GPU (pack_cameras).  Every solver returns the exact path's
    float32 bits (OpenCV 4.9's rounding sequence restated).  Default: QR + inverse iteration,
    the Jacobi restatement where that has not converged or is not certified; exact=True: the
    JacobiSVDImpl_ restatement for every point; tolerance=True: the throughput solver
    (MVP_TRI_TOLERANCE, reference mode with two listed cameras), certified per point, the
    exact path by a second launch where it is not.  The certification bound is empirical (its
    rounding-floor constants were fitted on 1.4 M synthetic and random points, with margin; see
    include/mvpose.h MVP_TRI_TOLERANCE): pass exact=True where a proof of bit-identity is
    required.  return_xyzw: the float64 null vectors
    (diagnostic; bit-identical to the exact path's only where that path solved the point —
    every point in tolerance mode)."""
    if exact and tolerance:
        raise ValueError("exact and tolerance exclude each other")
    if exact:
        mode = int(mode) | TRI_EXACT_JACOBI
    if tolerance:
        mode = int(mode) | TRI_TOLERANCE
    _require(kpts, torch.float32, "kpts")
    _require(cams, torch.float64, "cams")
    if kpts.dim() < 2 or kpts.shape[-2] != 3:
        raise ValueError(f"kpts must be (..., 3, V), got {tuple(kpts.shape)}")
    if cams.dim() != 2 or cams.shape[1] != CAM_DOUBLES:
        raise ValueError(f"cams must be (n_cams, {CAM_DOUBLES}), got {tuple(cams.shape)}")
    V = kpts.shape[-1]
    lead = tuple(kpts.shape[:-2])
    n = int(np.prod(lead)) if lead else 1
    if out is None:
        out = torch.empty(lead + (3,), dtype=torch.float32, device=kpts.device)
    else:
        _require(out, torch.float32, "out")
        if tuple(out.shape) != lead + (3,):
            raise ValueError("out has the wrong shape")
    xyzw = torch.empty(lead + (4,), dtype=torch.float64, device=kpts.device) if return_xyzw else None
    ci = (ctypes.c_int * len(cam_idx))(*[int(c) for c in cam_idx])
    call("mvp_triangulate", _ptr(kpts), n, V, _ptr(cams), cams.shape[0], ci, len(cam_idx), int(mode),
         _ptr(out), _ptr(xyzw) if xyzw is not None else None, _stream(kpts.device))
    return (out, xyzw) if return_xyzw else out


def triangulate_fallback_total(device=None) -> int:
    """Points the MVP_TRI_TOLERANCE solver has re-solved on the exact path on the current stream
    so far (mvp_triangulate_fallback_total; synchronises the stream)."""
    out = ctypes.c_ulonglong(0)
    call("mvp_triangulate_fallback_total", _stream(device), ctypes.byref(out))
    return int(out.value)


def triangulate_points_f64(kpts: torch.Tensor, cams: torch.Tensor, return_xyzw: bool = False):
    """utils.triangulate_points on float64 keypoints (mvp_triangulate_points_f64): kpts
    (..., 2, 2) float64 [view][x, y] on GPU, cams (2, 40) float64 (camera 1, camera 2) ->
    (..., 3) float64, OpenCV's CV_64F semantics end to end."""
    _require(kpts, torch.float64, "kpts")
    _require(cams, torch.float64, "cams")
    if kpts.dim() < 2 or tuple(kpts.shape[-2:]) != (2, 2):
        raise ValueError(f"kpts must be (..., 2, 2), got {tuple(kpts.shape)}")
    if tuple(cams.shape) != (2, CAM_DOUBLES):
        raise ValueError(f"cams must be (2, {CAM_DOUBLES}), got {tuple(cams.shape)}")
    lead = tuple(kpts.shape[:-2])
    n = int(np.prod(lead)) if lead else 1
    out = torch.empty(lead + (3,), dtype=torch.float64, device=kpts.device)
    xyzw = torch.empty(lead + (4,), dtype=torch.float64, device=kpts.device) if return_xyzw else None
    call("mvp_triangulate_points_f64", _ptr(kpts), n, _ptr(cams), _ptr(out),
         _ptr(xyzw) if xyzw is not None else None, _stream(kpts.device))
    return (out, xyzw) if return_xyzw else out
