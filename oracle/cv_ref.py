"""ORACLE (test infrastructure only) — OpenCV-4.9-semantics triangulation.

Python front of oracle/cv_calib3d.c plus a restatement of the reference's
triangulation orchestration:

* ``undistort_points`` / ``triangulate_points_cv`` / ``convert_points_from_homogeneous``
  mirror cv2.undistortPoints / cv2.triangulatePoints /
  cv2.convertPointsFromHomogeneous (signatures and dtypes) so they can be
  plugged into a stub ``cv2`` module when importing the reference.
* ``triangulate_points`` restates reference utils.py:1277-1336.
* ``get_pose_3D`` restates reference pose_estimation.py:11-65 (camera
  selection quirks included: top-2 by confidence in ASCENDING order, camera
  parameters keyed by selection position, dead NaN check).
* ``triangulate_all_views`` is the V>2 extension (BASELINE config 3): one
  2V x 4 DLT per point through the same Jacobi SVD.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def _load():
    global _lib
    if _lib is not None:
        return _lib
    src = os.path.join(_HERE, "cv_calib3d.c")
    if not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    lib = ctypes.CDLL(_SO)
    f32p = ctypes.POINTER(ctypes.c_float)
    f64p = ctypes.POINTER(ctypes.c_double)
    lib.orc_undistort_points_f32.argtypes = [f32p, ctypes.c_int64, f64p, f64p, ctypes.c_int, f32p]
    lib.orc_jacobi_svd.argtypes = [f64p, ctypes.c_int, ctypes.c_int, f64p, f64p]
    lib.orc_triangulate_nview.argtypes = [f64p, ctypes.c_int, f32p, ctypes.c_int64, f32p, f64p]
    lib.orc_from_homogeneous_f32.argtypes = [f32p, ctypes.c_int64, f32p]
    lib.orc_undistort_points_f64.argtypes = [f64p, ctypes.c_int64, f64p, f64p, ctypes.c_int, f64p]
    lib.orc_triangulate_nview_f64.argtypes = [f64p, ctypes.c_int, f64p, ctypes.c_int64, f64p]
    lib.orc_from_homogeneous_f64.argtypes = [f64p, ctypes.c_int64, f64p]
    lib.orc_hypot_check.argtypes = [f64p, f64p, ctypes.c_int64]
    lib.orc_hypot_check.restype = ctypes.c_int64
    _lib = lib
    return lib


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


# --------------------------------------------------------------------------
# cv2-compatible leaf functions (OpenCV 4.9 semantics, f32 in -> f32 out)
# --------------------------------------------------------------------------
def undistort_points(src, cameraMatrix, distCoeffs, R=None, P=None):
    """cv2.undistortPoints(src, K, dist, R=None, P=K) for the case the reference
    uses (utils.py:1314-1315).  src: (N,1,2) float32 (the pipeline's keypoints) or float64
    (the extrinsic branch's samples, pose_refinement.py:811); returns the same dtype (OpenCV
    writes into the source's depth)."""
    lib = _load()
    src = np.asarray(src)
    assert src.dtype in (np.float32, np.float64), "reference feeds float32 or float64 keypoints"
    assert R is None, "reference passes R=None"
    K = np.ascontiguousarray(np.asarray(cameraMatrix, dtype=np.float64).reshape(3, 3))
    if P is not None:
        assert np.array_equal(np.asarray(P, dtype=np.float64).reshape(3, 3), K), "reference passes P=K"
    else:
        raise NotImplementedError("P=None (normalised output) is not on the reference path")
    d = np.ascontiguousarray(np.asarray(distCoeffs, dtype=np.float64).ravel())
    pts = np.ascontiguousarray(src.reshape(-1, 2))
    out = np.empty_like(pts)
    if src.dtype == np.float64:
        lib.orc_undistort_points_f64(_p(pts, ctypes.c_double), pts.shape[0], _p(K, ctypes.c_double),
                                     _p(d, ctypes.c_double), int(d.size), _p(out, ctypes.c_double))
        return out.reshape(src.shape)
    lib.orc_undistort_points_f32(_p(pts, ctypes.c_float), pts.shape[0], _p(K, ctypes.c_double),
                                 _p(d, ctypes.c_double), int(d.size), _p(out, ctypes.c_float))
    return out.reshape(src.shape)


def triangulate_points_cv(P1, P2, x1, x2, return_f64=False):
    """cv2.triangulatePoints(P1, P2, x1 (2,N), x2 (2,N)) -> (4,N) in x1's dtype (f32 or f64)."""
    return triangulate_nview_cv([P1, P2], [x1, x2], return_f64=return_f64)


def triangulate_nview_cv(Ps, xs, return_f64=False):
    lib = _load()
    nv = len(Ps)
    Ps = np.ascontiguousarray(np.stack([np.asarray(P, dtype=np.float64).reshape(3, 4) for P in Ps]))
    xs = [np.asarray(x) for x in xs]
    n = xs[0].shape[1]
    if all(x.dtype == np.float64 for x in xs):
        X = np.ascontiguousarray(np.stack([x.T for x in xs]))  # (nv, n, 2)
        out64 = np.empty((4, n), np.float64)
        lib.orc_triangulate_nview_f64(_p(Ps, ctypes.c_double), nv, _p(X, ctypes.c_double), n,
                                      _p(out64, ctypes.c_double))
        return out64
    assert all(x.dtype == np.float32 for x in xs)
    X = np.ascontiguousarray(np.stack([x.T for x in xs]).astype(np.float32))  # (nv, n, 2)
    out = np.empty((4, n), np.float32)
    out64 = np.empty((4, n), np.float64)
    lib.orc_triangulate_nview(_p(Ps, ctypes.c_double), nv, _p(X, ctypes.c_float), n,
                              _p(out, ctypes.c_float), _p(out64, ctypes.c_double))
    return (out, out64) if return_f64 else out


def convert_points_from_homogeneous(src):
    """cv2.convertPointsFromHomogeneous on (N,4) float32 -> (N,1,3) float32 (float64 -> float64)."""
    lib = _load()
    if np.asarray(src).dtype == np.float64:
        src = np.ascontiguousarray(np.asarray(src).reshape(-1, 4))
        out = np.empty((src.shape[0], 3), np.float64)
        lib.orc_from_homogeneous_f64(_p(src, ctypes.c_double), src.shape[0], _p(out, ctypes.c_double))
        return out.reshape(-1, 1, 3)
    src = np.ascontiguousarray(np.asarray(src, dtype=np.float32).reshape(-1, 4))
    out = np.empty((src.shape[0], 3), np.float32)
    lib.orc_from_homogeneous_f32(_p(src, ctypes.c_float), src.shape[0], _p(out, ctypes.c_float))
    return out.reshape(-1, 1, 3)


def hypot_restatement_mismatches(x, y):
    """Pairs where glibc's hypot restated (the device exact path's text) differs from libm's."""
    lib = _load()
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    return int(lib.orc_hypot_check(_p(x, ctypes.c_double), _p(y, ctypes.c_double), x.size))


def jacobi_svd(A):
    """cv::SVD::compute(A) restated (lapack.cpp JacobiSVDImpl_): returns (w, Vt)."""
    lib = _load()
    A = np.asarray(A, dtype=np.float64)
    m, n = A.shape
    At = np.ascontiguousarray(A.T)
    w = np.empty(n)
    Vt = np.empty((n, n))
    lib.orc_jacobi_svd(_p(At, ctypes.c_double), m, n, _p(w, ctypes.c_double), _p(Vt, ctypes.c_double))
    return w, Vt


# --------------------------------------------------------------------------
# Reference orchestration restated
# --------------------------------------------------------------------------
def projection_matrix(K, R, T):
    """P = K [R|T] exactly as utils.py:1318-1319 computes it: np.dot in the parameters' own
    dtype (fp64 calibration files; float32 torch parameters in the extrinsic branch)."""
    K = np.asarray(K)
    R = np.asarray(R)
    T = np.asarray(T)
    return np.dot(K, np.hstack((R, T.reshape(-1, 1))))


def triangulate_points(kpts_2d, cmtx1, dist1, R1, T1, cmtx2, dist2, R2, T2):
    """Restates reference utils.triangulate_points (utils.py:1277-1336)."""
    kpts_2d = np.asarray(kpts_2d)
    shape = list(kpts_2d.shape[:-2])
    kpts_2d = kpts_2d.reshape([-1, 2, 2])
    n_pts = kpts_2d.shape[0]
    u1 = undistort_points(kpts_2d[:, 0, :][:, None, :], cmtx1, dist1, None, cmtx1)[:, 0, :]
    u2 = undistort_points(kpts_2d[:, 1, :][:, None, :], cmtx2, dist2, None, cmtx2)[:, 0, :]
    P1 = projection_matrix(cmtx1, R1, T1)
    P2 = projection_matrix(cmtx2, R2, T2)
    chunks = []
    start = 0
    for stop in range(512, n_pts + 512, 512):  # utils.py:1322-1328 (512-point chunks)
        stop = min(stop, n_pts)
        chunks.append(triangulate_points_cv(P1, P2, u1[start:stop].T, u2[start:stop].T))
        start = stop
    X4 = np.concatenate(chunks, -1)
    X3 = convert_points_from_homogeneous(X4.T)
    return X3.reshape(shape + [3])


def select_top2(conf):
    """np.argsort(conf)[-2:] for a short 1-D array (pose_estimation.py:36): stable
    ascending order (numpy's insertion sort for n < 16), NaN sorted last."""
    conf = np.asarray(conf)
    return np.argsort(conf, kind="stable")[-2:]


def get_pose_3D(camera_params, all_kpts_2d, world_trans_rot=None, camera_indices=None,
                ignore_nonlinear_distortions=False):
    """Restates reference pose_estimation.get_pose_3D (pose_estimation.py:11-65).

    camera_params: {key: [K, R, T, dist]} (utils.get_params_from_name order).
    all_kpts_2d: (T, J, 3, V) float32.  Returns (T, J, 3) float32.
    """
    cp = {}
    for key, (K, R, T, dist) in camera_params.items():  # :15-18 reorder to (K, dist, R, T)
        d = np.asarray(dist) * 0 if ignore_nonlinear_distortions else np.asarray(dist)
        cp[key] = [K, d, R, T]
    keys = list(cp.keys())
    if camera_indices is None:
        camera_indices = keys
    index_positions = [keys.index(ci) for ci in camera_indices]
    out = []
    for kpts_2d in all_kpts_2d:
        frame = []
        for i in range(kpts_2d.shape[0]):
            slice_2d = kpts_2d[i, :, index_positions].T  # (3, n_cam)
            if slice_2d.shape[0] == 3:
                top = select_top2(slice_2d[2, :])
            else:
                top = np.array([0, 1])
            top_points = slice_2d[:2, top].T  # (2, 2)
            p0 = cp[top[0]]  # NOTE: keyed by selection position (reference quirk)
            p1 = cp[top[1]]
            frame.append(triangulate_points(top_points, *(p0 + p1)))
        out.append(np.array(frame).reshape((kpts_2d.shape[0], 3)))
    out = np.array(out)
    if world_trans_rot is not None:
        R_W0, _ = world_trans_rot
        out = np.einsum("ij,tpj->tpi", np.linalg.inv(R_W0), out)
    return out


def triangulate_all_views(cams, all_kpts_2d, camera_indices):
    """Extension (BASELINE config 3): all listed views in one 2V x 4 DLT per point,
    same undistortion and SVD semantics.  cams: list of (K, R, T, dist)."""
    all_kpts_2d = np.asarray(all_kpts_2d, dtype=np.float32)
    T, J = all_kpts_2d.shape[:2]
    n = T * J
    Ps, xs = [], []
    for c in camera_indices:
        K, R, Tt, dist = cams[c]
        pts = np.ascontiguousarray(all_kpts_2d[:, :, :2, c].reshape(n, 1, 2))
        xs.append(undistort_points(pts, K, dist, None, K)[:, 0, :].T)
        Ps.append(projection_matrix(K, R, Tt))
    X4 = triangulate_nview_cv(Ps, xs)
    return convert_points_from_homogeneous(X4.T).reshape(T, J, 3)
