"""ORACLE (test infrastructure only) — 2D-stage numerics around the backbone.

Restates, in numpy, what the reference's PoseEstimator.predict
(mmpose_pose_estimation.py:222-272) gets from its external dependencies, plus
the reference's own moment computation:

* mmpose 1.x top-down geometry: bbox_xyxy2cs (padding 1.25), _fix_aspect_ratio,
  get_warp_matrix (-> cv2.getAffineTransform), used by TopdownAffine (crop) and
  revert_heatmap (heatmap -> image) — call sites :253-254;
* cv2.warpAffine(INTER_LINEAR, BORDER_CONSTANT 0) for uint8 (fixed-point
  weights) and float32 (float weights), OpenCV 4.9 imgwarp.cpp
  WarpAffineInvoker + remapBilinear (AB_BITS 10, INTER_BITS 5);
* mmpose flip_heatmaps(flip_mode='heatmap', shift_heatmap=True) + MSRAHeatmap
  decode (get_heatmap_maximum, +-0.25 shift) + TopdownPoseEstimator's
  keypoint restore;
* PoseEstimator.get_heatmap_means_cov (mmpose_pose_estimation.py:163-215) in
  fp64 (the GPU kernel's accumulation precision).

mmpose / OpenCV are absent here: parity of these restatements against the real
libraries is UNPINNED.  The moment computation on top is pinned to
the reference by tests/golden/moments.npz.
"""
from __future__ import annotations

import numpy as np

INTER_BITS = 5
INTER_TAB_SIZE = 1 << INTER_BITS
AB_BITS = 10
AB_SCALE = 1 << AB_BITS
COEF_BITS = 15

COCO_FLIP_INDICES = [0, 2, 1, 4, 3, 6, 5, 8, 7, 10, 9, 12, 11, 14, 13, 16, 15]
MEAN_RGB = np.array([123.675, 116.28, 103.53], np.float32)
STD_RGB = np.array([58.395, 57.12, 57.375], np.float32)


# ---------------------------------------------------------------- geometry --
def bbox_xyxy2cs(bbox, padding=1.25):
    """mmpose bbox_xyxy2cs: (x1,y1,x2,y2) -> center, scale (float32).  The box is
    mmdet's float32 bboxes row (mmpose_pose_estimation.py:242-253)."""
    x1, y1, x2, y2 = [float(np.float32(v)) for v in bbox]
    center = np.array([x1 + x2, y1 + y2], np.float32) * 0.5
    scale = np.array([x2 - x1, y2 - y1], np.float32) * padding
    return center.astype(np.float32), scale.astype(np.float32)


def whole_image_cs(img_w, img_h, padding=1.25):
    """The reference's no-detection fallback: bbox = whole image
    (mmpose inference_topdown with bboxes=None; mmpose_pose_estimation.py:246-253)."""
    return bbox_xyxy2cs([0, 0, img_w, img_h], padding)


def fix_aspect_ratio(scale, aspect_ratio):
    """mmpose TopdownAffine._fix_aspect_ratio (w/h = aspect_ratio)."""
    w, h = float(scale[0]), float(scale[1])
    if w > h * aspect_ratio:
        return np.array([w, w / aspect_ratio], np.float32)
    return np.array([h * aspect_ratio, h], np.float32)


def cv_lu_solve(a, b):
    """cv::solve(DECOMP_LU) on an m x m system: OpenCV 4.9 hal::LU64f -> LUImpl
    (modules/core/src/matrix_decomp.cpp; external, parity unpinned — OpenCV is absent
    here): column pivot = the first row with the largest |a| (strict >), d = -1/pivot,
    row update a[j][k] += (a[j][i]·d)·a[i][k], back substitution s -= a[i][k]·b[k],
    b[i] = s / a[i][i].  A pivot below 100·DBL_EPSILON makes solve() fail and return
    zeros.  Plain Python floats (IEEE fp64, no FMA), so every rounding is OpenCV's."""
    a = [[float(v) for v in row] for row in np.asarray(a, np.float64)]
    b = [float(v) for v in np.asarray(b, np.float64).ravel()]
    m = len(b)
    for i in range(m):
        k = i
        for j in range(i + 1, m):
            if abs(a[j][i]) > abs(a[k][i]):
                k = j
        if abs(a[k][i]) < 100 * np.finfo(np.float64).eps:
            return np.zeros(m)
        if k != i:
            a[i], a[k] = a[k], a[i]
            b[i], b[k] = b[k], b[i]
        d = -1.0 / a[i][i]
        for j in range(i + 1, m):
            alpha = a[j][i] * d
            for c in range(i + 1, m):
                a[j][c] += alpha * a[i][c]
            b[j] += alpha * b[i]
    for i in range(m - 1, -1, -1):
        s = b[i]
        for c in range(i + 1, m):
            s -= a[i][c] * b[c]
        b[i] = s / a[i][i]
    return np.array(b)


def get_affine_transform(src, dst):
    """cv2.getAffineTransform (imgwarp.cpp): the 6x6 system OpenCV builds (rows
    (x, y, 1, 0, 0, 0) and (0, 0, 0, x, y, 1) per point), solved by cv::solve's LU."""
    src = np.asarray(src, np.float32).astype(np.float64)
    dst = np.asarray(dst, np.float32).astype(np.float64)
    a = np.zeros((6, 6))
    b = np.zeros(6)
    for i in range(3):
        a[2 * i, 0:3] = [src[i, 0], src[i, 1], 1.0]
        a[2 * i + 1, 3:6] = [src[i, 0], src[i, 1], 1.0]
        b[2 * i] = dst[i, 0]
        b[2 * i + 1] = dst[i, 1]
    return cv_lu_solve(a, b).reshape(2, 3)


def _rotate_point(pt, angle_rad):
    sn, cs = np.sin(angle_rad), np.cos(angle_rad)
    return np.array([[cs, -sn], [sn, cs]]) @ pt


def _get_3rd_point(a, b):
    direction = a - b
    return b + np.r_[-direction[1], direction[0]]


def get_warp_matrix(center, scale, rot, output_size, shift=(0.0, 0.0), inv=False):
    """mmpose.structures.bbox.get_warp_matrix (fix_aspect_ratio=True)."""
    shift = np.array(shift)
    src_w = scale[0]
    dst_w, dst_h = output_size
    rot_rad = np.deg2rad(rot)
    src_dir = _rotate_point(np.array([src_w * -0.5, 0.0]), rot_rad)
    dst_dir = np.array([dst_w * -0.5, 0.0])
    src = np.zeros((3, 2), np.float32)
    src[0, :] = center + scale * shift
    src[1, :] = center + src_dir + scale * shift
    src[2, :] = _get_3rd_point(src[0, :], src[1, :])
    dst = np.zeros((3, 2), np.float32)
    dst[0, :] = [dst_w * 0.5, dst_h * 0.5]
    dst[1, :] = np.array([dst_w * 0.5, dst_h * 0.5]) + dst_dir
    dst[2, :] = _get_3rd_point(dst[0, :], dst[1, :])
    if inv:
        return get_affine_transform(dst, src)
    return get_affine_transform(src, dst)


def invert_affine(M):
    """warpAffine's internal inversion when WARP_INVERSE_MAP is not set
    (imgwarp.cpp): returns the dst -> src map, fp64, OpenCV's op order."""
    M = [float(v) for v in np.asarray(M, np.float64).ravel()]
    D = M[0] * M[4] - M[1] * M[3]
    D = 1.0 / D if D != 0 else 0.0
    A11 = M[4] * D
    A22 = M[0] * D
    M[0] = A11
    M[1] *= -D
    M[3] *= -D
    M[4] = A22
    b1 = -M[0] * M[2] - M[1] * M[5]
    b2 = -M[3] * M[2] - M[4] * M[5]
    M[2] = b1
    M[5] = b2
    return np.array(M)


def _cv_round(x):
    """saturate_cast<int>(double) = cvRound: round half to even."""
    return np.rint(x).astype(np.int64)


def warp_coords(M_inv6, out_h, out_w):
    """Per output pixel: integer source cell (sx, sy) and 5-bit fractions (tx, ty),
    exactly WarpAffineInvoker's fixed-point mapping.  M_inv6: dst->src map."""
    M = M_inv6
    round_delta = AB_SCALE // INTER_TAB_SIZE // 2
    xs = np.arange(out_w, dtype=np.float64)
    ys = np.arange(out_h, dtype=np.float64)
    adelta = _cv_round(M[0] * xs * AB_SCALE)
    bdelta = _cv_round(M[3] * xs * AB_SCALE)
    X0 = _cv_round((M[1] * ys + M[2]) * AB_SCALE) + round_delta
    Y0 = _cv_round((M[4] * ys + M[5]) * AB_SCALE) + round_delta
    X = (X0[:, None] + adelta[None, :]) >> (AB_BITS - INTER_BITS)
    Y = (Y0[:, None] + bdelta[None, :]) >> (AB_BITS - INTER_BITS)
    sx = X >> INTER_BITS
    sy = Y >> INTER_BITS
    tx = X & (INTER_TAB_SIZE - 1)
    ty = Y & (INTER_TAB_SIZE - 1)
    return sx, sy, tx, ty


def _gather_taps(src, sx, sy):
    """BORDER_CONSTANT(0) bilinear taps. src (C, H, W) -> 4 arrays (C, oh, ow)."""
    C, H, W = src.shape
    taps = []
    for dy, dx in ((0, 0), (0, 1), (1, 0), (1, 1)):
        xx, yy = sx + dx, sy + dy
        ok = (xx >= 0) & (xx < W) & (yy >= 0) & (yy < H)
        v = src[:, np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)]
        taps.append(np.where(ok[None], v, np.zeros((), src.dtype)))
    # fully outside -> border value (same result: all taps already 0)
    return taps


def warp_affine_linear_u8(img_hwc, M, out_h, out_w):
    """cv2.warpAffine(img_u8, M (src->dst), (out_w, out_h), INTER_LINEAR), fixed point.
    Returns (out_h, out_w, C) uint8."""
    Minv = invert_affine(M)
    sx, sy, tx, ty = warp_coords(Minv, out_h, out_w)
    src = np.ascontiguousarray(np.moveaxis(img_hwc, -1, 0)).astype(np.int64)
    v0, v1, v2, v3 = _gather_taps(src, sx, sy)
    # float tab products (1-ty/32)(1-tx/32) etc. are exact multiples of 1/1024;
    # x 2^15 -> integer weights summing to 32768 (no isum correction needed)
    w0 = (32 - ty) * (32 - tx) * 32
    w1 = (32 - ty) * tx * 32
    w2 = ty * (32 - tx) * 32
    w3 = ty * tx * 32
    t = v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3
    out = np.clip((t + (1 << (COEF_BITS - 1))) >> COEF_BITS, 0, 255).astype(np.uint8)
    return np.moveaxis(out, 0, -1)


def warp_affine_linear_f32(src_chw, M, out_h, out_w):
    """cv2.warpAffine(float32 (H,W,C) image given here as (C,H,W), M (src->dst),
    (out_w, out_h), INTER_LINEAR).  Float weights, ((v0 w0 + v1 w1) + v2 w2) + v3 w3
    in float32.  Returns (C, out_h, out_w) float32."""
    Minv = invert_affine(M)
    sx, sy, tx, ty = warp_coords(Minv, out_h, out_w)
    src = np.asarray(src_chw, np.float32)
    v0, v1, v2, v3 = _gather_taps(src, sx, sy)
    fx = (tx.astype(np.float32) * np.float32(1.0 / INTER_TAB_SIZE)).astype(np.float32)
    fy = (ty.astype(np.float32) * np.float32(1.0 / INTER_TAB_SIZE)).astype(np.float32)
    one = np.float32(1.0)
    w0 = ((one - fy) * (one - fx)).astype(np.float32)
    w1 = ((one - fy) * fx).astype(np.float32)
    w2 = (fy * (one - fx)).astype(np.float32)
    w3 = (fy * fx).astype(np.float32)
    t = v0 * w0[None]
    t = t + v1 * w1[None]
    t = t + v2 * w2[None]
    t = t + v3 * w3[None]
    return t.astype(np.float32)


# ---------------------------------------------------------------- preprocess --
def topdown_crop_matrix(img_w, img_h, input_size=(192, 256), padding=1.25):
    """Crop matrix for the whole-image bbox (src->dst), center, scale."""
    center, scale = whole_image_cs(img_w, img_h, padding)
    scale = fix_aspect_ratio(scale, input_size[0] / input_size[1])
    M = get_warp_matrix(center, scale, 0.0, input_size)
    return M, center, scale


def preprocess(frame_hwc_u8, M, input_size=(192, 256), swap_rb=True):
    """TopdownAffine warp (u8) + PoseDataPreprocessor (bgr_to_rgb, (x-mean)/std, f32).
    Returns (3, H, W) float32 (NCHW order for one crop)."""
    w, h = input_size
    crop = warp_affine_linear_u8(frame_hwc_u8, M, h, w)  # (h, w, 3)
    x = np.moveaxis(crop, -1, 0).astype(np.float32)
    if swap_rb:
        x = x[[2, 1, 0]]
    return ((x - MEAN_RGB[:, None, None]) / STD_RGB[:, None, None]).astype(np.float32)


# ---------------------------------------------------------------- decode --
def flip_back_heatmaps(hm_flip, flip_indices=COCO_FLIP_INDICES, shift=True):
    """mmpose flip_heatmaps(flip_mode='heatmap', shift_heatmap=True) on (N,K,H,W)."""
    h = hm_flip[..., ::-1][:, flip_indices].copy()
    if shift:
        h[..., 1:] = h[..., :-1].copy()
    return h


def flip_test_average(hm, hm_flip, flip_indices=COCO_FLIP_INDICES, shift=True):
    return ((hm + flip_back_heatmaps(hm_flip, flip_indices, shift)) * np.float32(0.5)).astype(np.float32)


def get_heatmap_maximum(heatmaps):
    """mmpose get_heatmap_maximum on (K,H,W): first-occurrence argmax."""
    K, H, W = heatmaps.shape
    flat = heatmaps.reshape(K, -1)
    idx = np.argmax(flat, axis=1)
    y, x = np.unravel_index(idx, (H, W))
    locs = np.stack((x, y), axis=-1).astype(np.float32)
    vals = np.amax(flat, axis=1)
    locs[vals <= 0.0] = -1
    return locs, vals, idx.astype(np.int32)


def msra_decode(heatmaps):
    """MSRAHeatmap.decode (unbiased=False) on (K,H,W) -> keypoints (K,2) f32 in
    heatmap*4 (input) pixels, scores (K,), argmax index (K,)."""
    K, H, W = heatmaps.shape
    kpts, scores, idx = get_heatmap_maximum(heatmaps)
    for k in range(K):
        px, py = int(kpts[k, 0]), int(kpts[k, 1])
        if 1 < px < W - 1 and 1 < py < H - 1:
            hm = heatmaps[k]
            diff = np.array([hm[py][px + 1] - hm[py][px - 1], hm[py + 1][px] - hm[py - 1][px]])
            kpts[k] += np.sign(diff) * 0.25
    scale_factor = np.array([192 / W, 256 / H], np.float32)
    return (kpts * scale_factor).astype(np.float32), scores, idx


def keypoints_to_image(kpts_input, center, scale, input_size=(192, 256)):
    """TopdownPoseEstimator.add_pred_to_datasample restore:
    keypoints / input_size * input_scale + input_center - 0.5 * input_scale.
    input_size is TopdownAffine's (w, h) tuple of Python ints, so the f32
    keypoints promote to float64 (int64 array operand); the result is stored
    back into the float32 keypoint array."""
    size = np.asarray(tuple(int(v) for v in input_size))  # int64
    center = np.asarray(center, np.float32)
    scale = np.asarray(scale, np.float32)
    out = np.asarray(kpts_input, np.float32) / size * scale + center - 0.5 * scale
    return out.astype(np.float32)


# ---------------------------------------------------------------- moments --
def heatmap_means_cov_f64(hm, thr=0.01):
    """get_heatmap_means_cov semantics (mmpose_pose_estimation.py:163-215) in fp64:
    hm[hm < thr] = 0; per joint mean x/y, var x/y, cov xy of the normalised map,
    zero-sum -> zeros.  hm (K,H,W) -> (K,6) [mx, my, vxx, vxy, vxy, vyy]."""
    h = np.where(hm < thr, 0.0, hm.astype(np.float64))
    K, H, W = h.shape
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float64)
    out = np.zeros((K, 6))
    for k in range(K):
        s = h[k].sum()
        if s == 0:
            continue
        p = h[k] / s
        mx, my = (xs * p).sum(), (ys * p).sum()
        vx = ((xs - mx) ** 2 * p).sum()
        vy = ((ys - my) ** 2 * p).sum()
        cxy = ((xs - mx) * (ys - my) * p).sum()
        out[k] = [mx, my, vx, cxy, cxy, vy]
    return out
