"""Host-side geometry and calibration I/O for the hot path.

* Calibration files exactly as the reference writes and reads them
  (utils.save_camera_intrinsics / read_camera_parameters, utils.py:204-233 /
  750-770; save_extrinsic_calibration_parameters / read_rotation_translation,
  utils.py:720-793; get_params_from_name, utils.py:807-828; camera_names.pkl,
  setup_camera_configuration.py:34-106 / pose_estimation.py:265-270).
* mmpose top-down crop geometry for the reference's whole-image bbox fallback
  (mmpose_pose_estimation.py:246-253): bbox -> center/scale (padding 1.25),
  aspect-ratio fix, get_warp_matrix (via cv2.getAffineTransform's 6x6 system),
  and the inverse map cv2.warpAffine applies internally.
"""
from __future__ import annotations

import io
import os
import pickle

import numpy as np

INPUT_SIZE = (192, 256)     # (w, h) of the HRNet-W32 256x192 crop
HEATMAP_SIZE = (48, 64)     # (w, h)
BBOX_PADDING = 1.25


# ----------------------------------------------------------------- calibration
def _read_rows(lines, start, n):
    return [[float(v) for v in lines[start + i].split()] for i in range(n)]


def read_camera_parameters(camera_name, params_dir=""):
    """intrinsic_camera_parameters/<name>.dat: 'intrinsic:' + 3 rows, 'distortion:' + 1 row."""
    params_dir = params_dir or os.getcwd()
    with open(os.path.join(params_dir, camera_name + ".dat")) as f:
        lines = f.read().splitlines()
    return np.array(_read_rows(lines, 1, 3)), np.array(_read_rows(lines, 5, 1))


def read_rotation_translation(camera_name, params_dir=""):
    """extrinsic_camera_parameters/rot_trans_<name>.dat: 'R:' + 3 rows, 'T:' + 3 rows."""
    params_dir = params_dir or os.getcwd()
    with open(os.path.join(params_dir, "rot_trans_" + camera_name + ".dat")) as f:
        lines = f.read().splitlines()
    return np.array(_read_rows(lines, 1, 3)), np.array(_read_rows(lines, 5, 3))


def write_camera_parameters(camera_name, K, dist, params_dir):
    os.makedirs(params_dir, exist_ok=True)
    with open(os.path.join(params_dir, camera_name + ".dat"), "w") as f:
        f.write("intrinsic:\n")
        for row in np.asarray(K):
            f.write("".join(str(v) + " " for v in row) + "\n")
        f.write("distortion:\n")
        f.write("".join(str(v) + " " for v in np.asarray(dist).reshape(1, -1)[0]) + "\n")


def write_rotation_translation(camera_name, R, T, params_dir):
    os.makedirs(params_dir, exist_ok=True)
    with open(os.path.join(params_dir, "rot_trans_" + camera_name + ".dat"), "w") as f:
        f.write("R:\n")
        for row in np.asarray(R):
            f.write("".join(str(v) + " " for v in row) + "\n")
        f.write("T:\n")
        for row in np.asarray(T).reshape(3, -1):
            f.write("".join(str(v) + " " for v in row) + "\n")


def projection_matrix(K, R, T):
    """P = K [R|T] (utils.calculate_projection_matrix, utils.py:803-805)."""
    return np.asarray(K, np.float64) @ np.hstack((np.asarray(R, np.float64), np.asarray(T, np.float64).reshape(3, 1)))


def get_params_from_name(camera_name, intrinsic_params_dir="", extrinsic_params_dir=""):
    """Returns (P, [K, R, T, dist]) like utils.get_params_from_name; missing files
    are reported and left as None (the reference prints and continues)."""
    intrinsic_params_dir = intrinsic_params_dir or os.path.join(os.getcwd(), "intrinsic_camera_parameters")
    extrinsic_params_dir = extrinsic_params_dir or os.path.join(os.getcwd(), "extrinsic_camera_parameters")
    K = dist = R = T = P = None
    try:
        K, dist = read_camera_parameters(camera_name, intrinsic_params_dir)
    except (OSError, ValueError, IndexError) as e:
        print(f"failed to load {camera_name} intrinsic params ({e})")
    try:
        R, T = read_rotation_translation(camera_name, extrinsic_params_dir)
    except (OSError, ValueError, IndexError) as e:
        print(f"failed to load {camera_name} extrinsic params ({e})")
    if K is not None and R is not None:
        P = projection_matrix(K, R, T)
    return P, [K, R, T, dist]


class _CameraNamesUnpickler(pickle.Unpickler):
    """camera_names.pkl holds ({index: name}, origin_name): builtins only."""

    def find_class(self, module, name):
        raise pickle.UnpicklingError(f"camera_names.pkl may only hold dict/str/int, found {module}.{name}")


def load_camera_names(extrinsic_params_dir):
    with open(os.path.join(extrinsic_params_dir, "camera_names.pkl"), "rb") as f:
        return _CameraNamesUnpickler(io.BytesIO(f.read())).load()


def save_camera_names(extrinsic_params_dir, index_name, origin_name):
    os.makedirs(extrinsic_params_dir, exist_ok=True)
    with open(os.path.join(extrinsic_params_dir, "camera_names.pkl"), "wb") as f:
        pickle.dump((dict(index_name), origin_name), f)


# ------------------------------------------------------------ top-down crops
def bbox_center_scale(bbox_xyxy, padding=BBOX_PADDING):
    x1, y1, x2, y2 = [float(np.float32(v)) for v in bbox_xyxy]
    center = (np.array([x1 + x2, y1 + y2], np.float32) * 0.5).astype(np.float32)
    scale = (np.array([x2 - x1, y2 - y1], np.float32) * padding).astype(np.float32)
    return center, scale


def fix_aspect_ratio(scale, aspect_ratio):
    w, h = float(scale[0]), float(scale[1])
    return np.array([w, w / aspect_ratio] if w > h * aspect_ratio else [h * aspect_ratio, h], np.float32)


def lu_solve_batch(A, b):
    """cv::solve(DECOMP_LU) for N m x m systems at once: OpenCV's hal::LU64f (LUImpl,
    modules/core/src/matrix_decomp.cpp) — the pivot is the first row with the largest
    |a| of the column, d = -1 / pivot, rows updated a += (a_ji·d)·a_i, back substitution
    s -= a_ik·b_k then s / a_ii; a pivot below 100·DBL_EPSILON = failure = zeros.  numpy
    elementwise fp64 (no FMA), so the roundings are OpenCV's; mvp_bbox_geometry does the
    same on the device.  A (N, m, m), b (N, m) float64 -> (N, m)."""
    a = np.array(A, np.float64, copy=True)
    x = np.array(b, np.float64, copy=True)
    n, m = x.shape
    rows = np.arange(n)
    bad = np.zeros(n, bool)
    for i in range(m):
        k = i + np.argmax(np.abs(a[:, i:, i]), axis=1)      # first maximum = OpenCV's strict '>' scan
        bad |= np.abs(a[rows, k, i]) < 100 * np.finfo(np.float64).eps
        ai, ak = a[rows, i].copy(), a[rows, k].copy()
        a[rows, i], a[rows, k] = ak, ai
        xi, xk = x[rows, i].copy(), x[rows, k].copy()
        x[rows, i], x[rows, k] = xk, xi
        with np.errstate(divide="ignore", invalid="ignore"):
            d = -1.0 / a[:, i, i]
            for j in range(i + 1, m):
                alpha = a[:, j, i] * d
                a[:, j, i + 1:] += alpha[:, None] * a[:, i, i + 1:]
                x[:, j] += alpha * x[:, i]
    with np.errstate(divide="ignore", invalid="ignore"):
        for i in range(m - 1, -1, -1):
            s = x[:, i].copy()
            for c in range(i + 1, m):
                s -= a[:, i, c] * x[:, c]
            x[:, i] = s / a[:, i, i]
    x[bad] = 0.0
    return x


def _affine_system(src, dst):
    """cv2.getAffineTransform's 6x6 system for N point triples: src, dst (N, 3, 2) f32."""
    s = np.asarray(src, np.float32).astype(np.float64)
    d = np.asarray(dst, np.float32).astype(np.float64)
    n = s.shape[0]
    A = np.zeros((n, 6, 6))
    b = np.zeros((n, 6))
    for i in range(3):
        A[:, 2 * i, 0], A[:, 2 * i, 1], A[:, 2 * i, 2] = s[:, i, 0], s[:, i, 1], 1.0
        A[:, 2 * i + 1, 3], A[:, 2 * i + 1, 4], A[:, 2 * i + 1, 5] = s[:, i, 0], s[:, i, 1], 1.0
        b[:, 2 * i], b[:, 2 * i + 1] = d[:, i, 0], d[:, i, 1]
    return A, b


def affine_from_points(src, dst):
    """cv2.getAffineTransform (imgwarp.cpp): the 6x6 system solved by cv::solve's LU."""
    A, b = _affine_system(np.asarray(src)[None], np.asarray(dst)[None])
    return lu_solve_batch(A, b)[0].reshape(2, 3)


def warp_matrix(center, scale, output_size, inv=False):
    """mmpose get_warp_matrix with rot=0, shift=0, fix_aspect_ratio=True."""
    src_w = float(scale[0])
    dst_w, dst_h = output_size
    src = np.zeros((3, 2), np.float32)
    dst = np.zeros((3, 2), np.float32)
    src[0] = center
    src[1] = center + np.array([src_w * -0.5, 0.0])
    d = src[0] - src[1]
    src[2] = src[1] + np.array([-d[1], d[0]])
    dst[0] = (dst_w * 0.5, dst_h * 0.5)
    dst[1] = np.array([dst_w * 0.5, dst_h * 0.5]) + np.array([dst_w * -0.5, 0.0])
    d = dst[0] - dst[1]
    dst[2] = dst[1] + np.array([-d[1], d[0]])
    return affine_from_points(dst, src) if inv else affine_from_points(src, dst)


def inverse_map(M):
    """The dst -> src map cv2.warpAffine derives from M (imgwarp.cpp, fp64)."""
    m = [float(v) for v in np.asarray(M, np.float64).ravel()]
    D = m[0] * m[4] - m[1] * m[3]
    D = 1.0 / D if D != 0 else 0.0
    a11, a22 = m[4] * D, m[0] * D
    m[0], m[4] = a11, a22
    m[1] *= -D
    m[3] *= -D
    b1 = -m[0] * m[2] - m[1] * m[5]
    b2 = -m[3] * m[2] - m[4] * m[5]
    m[2], m[5] = b1, b2
    return np.array(m)


def _warp_points(center, scale_w, out_w, out_h):
    """mmpose get_warp_matrix's three point pairs for N boxes (rot 0, shift 0): src (N,3,2)
    and dst (N,3,2) float32, with warp_matrix's f32 rounding points."""
    n = center.shape[0]
    src = np.zeros((n, 3, 2), np.float32)
    dst = np.zeros((n, 3, 2), np.float32)
    src[:, 0] = center
    src[:, 1, 0] = (center[:, 0].astype(np.float64) + scale_w.astype(np.float64) * -0.5).astype(np.float32)
    src[:, 1, 1] = center[:, 1]
    d = src[:, 0] - src[:, 1]
    src[:, 2, 0] = src[:, 1, 0] + -d[:, 1]
    src[:, 2, 1] = src[:, 1, 1] + d[:, 0]
    dst[:, 0] = (out_w * 0.5, out_h * 0.5)
    dst[:, 1] = (out_w * 0.5 + out_w * -0.5, out_h * 0.5)
    dd = dst[:, 0] - dst[:, 1]
    dst[:, 2, 0] = dst[:, 1, 0] + -dd[:, 1]
    dst[:, 2, 1] = dst[:, 1, 1] + dd[:, 0]
    return src, dst


def _affine_batch(src, dst):
    """affine_from_points for N point triples."""
    return lu_solve_batch(*_affine_system(src, dst))


def _inverse_map_batch(M):
    """inverse_map for (N,6) maps (fp64, OpenCV's op order)."""
    m = np.array(M, np.float64, copy=True)
    D = m[:, 0] * m[:, 4] - m[:, 1] * m[:, 3]
    with np.errstate(divide="ignore"):
        D = np.where(D != 0, 1.0 / np.where(D != 0, D, 1.0), 0.0)
    a11, a22 = m[:, 4] * D, m[:, 0] * D
    m[:, 0], m[:, 4] = a11, a22
    m[:, 1] *= -D
    m[:, 3] *= -D
    b1 = -m[:, 0] * m[:, 2] - m[:, 1] * m[:, 5]
    b2 = -m[:, 3] * m[:, 2] - m[:, 4] * m[:, 5]
    m[:, 2], m[:, 5] = b1, b2
    return m


def crop_geometry_batch(bboxes_xyxy, padding=BBOX_PADDING):
    """Vectorised CropGeometry for N boxes: (crop_minv (N,6) f64, revert_minv (N,6) f64,
    center_scale (N,4) f32) — the same numbers CropGeometry(box) gives one box at a time
    (mmpose bbox_xyxy2cs -> TopdownAffine -> get_warp_matrix, mmpose_pose_estimation.py:253)."""
    # mmdet's boxes are float32; the f32 sums / differences are formed exactly in fp64 and rounded once
    bb = np.asarray(bboxes_xyxy, np.float64).reshape(-1, 4).astype(np.float32).astype(np.float64)
    x1, y1, x2, y2 = (bb[:, i] for i in range(4))
    center = (np.stack([x1 + x2, y1 + y2], 1).astype(np.float32) * np.float32(0.5)).astype(np.float32)
    scale = (np.stack([x2 - x1, y2 - y1], 1).astype(np.float32) * np.float32(padding)).astype(np.float32)
    ar = INPUT_SIZE[0] / INPUT_SIZE[1]
    w, h = scale[:, 0].astype(np.float64), scale[:, 1].astype(np.float64)
    wide = w > h * ar
    scale = np.where(wide[:, None], np.stack([w, w / ar], 1), np.stack([h * ar, h], 1)).astype(np.float32)
    s_in, d_in = _warp_points(center, scale[:, 0], *INPUT_SIZE)
    crop_minv = _inverse_map_batch(_affine_batch(s_in, d_in))
    s_hm, d_hm = _warp_points(center, scale[:, 0], *HEATMAP_SIZE)
    revert_minv = _inverse_map_batch(_affine_batch(d_hm, s_hm))
    cs = np.concatenate([center, scale], 1).astype(np.float32)
    return crop_minv, revert_minv, cs


class CropGeometry:
    """Everything the GPU stages need for one bbox: crop map (crop -> image),
    revert map (image -> heatmap), center/scale for the keypoint restore."""

    def __init__(self, bbox_xyxy):
        center, scale = bbox_center_scale(bbox_xyxy)
        scale = fix_aspect_ratio(scale, INPUT_SIZE[0] / INPUT_SIZE[1])
        self.center, self.scale = center, scale
        self.crop_minv = inverse_map(warp_matrix(center, scale, INPUT_SIZE))            # crop -> image
        self.revert_minv = inverse_map(warp_matrix(center, scale, HEATMAP_SIZE, inv=True))  # image -> heatmap
        self.center_scale = np.array([center[0], center[1], scale[0], scale[1]], np.float32)

    @classmethod
    def whole_image(cls, width, height):
        """The reference's no-detection fallback (mmpose_pose_estimation.py:246-250)."""
        return cls([0, 0, width, height])
