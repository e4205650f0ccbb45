"""GPU: mvp_bbox_geometry — the detector -> inference_topdown hand-off and TopdownAffine
geometry on the device (mmpose_pose_estimation.py:242-253) — equals its host twin
geometry.crop_geometry_batch bit for bit (crop map, revert map, center/scale), its
separability flags equal mvp_warp_is_separable of each revert map, the score rule
(score > bbox_thr, else the whole image) is applied per row, and BatchPoseEstimator.run
with device boxes equals the same run with the host boxes."""
import ctypes

import numpy as np
import pytest
import torch

from mvpose import _lib, geometry

pytestmark = pytest.mark.gpu


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def _boxes(n, seed):
    rng = np.random.default_rng(seed)
    x1 = rng.uniform(-150, 1250, n)
    y1 = rng.uniform(-100, 700, n)
    b = np.stack([x1, y1, x1 + rng.uniform(0.5, 1400, n), y1 + rng.uniform(0.5, 800, n)], 1).astype(np.float32)
    b[3] = np.nan                                   # no detection
    b[5] = (0, 0, 1280, 720)                        # explicit whole image
    if n > 9:
        b[6] = (640, 360, 640, 380)                 # zero width (the aspect fix widens it)
        b[9] = (100.5, 50.25, 400.0, 700.0)
    return b


def _device_geometry(rows, score_col=-1, thr=0.0, fh=720, fw=1280):
    n = rows.shape[0]
    bx = torch.tensor(rows, device="cuda")
    cm = torch.empty((n, 6), dtype=torch.float64, device="cuda")
    rm = torch.empty((n, 6), dtype=torch.float64, device="cuda")
    cs = torch.empty((n, 4), dtype=torch.float32, device="cuda")
    sep = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    _lib.call("mvp_bbox_geometry", _p(bx), rows.shape[1], n, score_col, ctypes.c_float(thr), fh, fw, _p(cm), _p(rm),
              _p(cs), _p(sep), None)
    torch.cuda.synchronize()
    return cm.cpu().numpy(), rm.cpu().numpy(), cs.cpu().numpy(), sep.cpu().numpy()


def _sep(m, fh=720, fw=1280):
    out = ctypes.c_int()
    m = np.ascontiguousarray(m, np.float64)
    _lib.call("mvp_warp_is_separable", m.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), fh, fw, ctypes.byref(out))
    return out.value


@pytest.mark.parametrize("fh,fw", [(720, 1280), (360, 640), (1080, 1920)])
def test_device_geometry_bit_exact(fh, fw):
    b = _boxes(300, fh)
    cm, rm, cs, sep = _device_geometry(b, fh=fh, fw=fw)
    hb = b.astype(np.float64)
    hb[~np.isfinite(hb).all(1)] = (0, 0, fw, fh)
    hcm, hrm, hcs = geometry.crop_geometry_batch(hb)
    np.testing.assert_array_equal(cs, hcs)
    np.testing.assert_array_equal(cm, hcm)
    np.testing.assert_array_equal(rm, hrm)
    want = np.array([_sep(m, fh, fw) for m in rm])
    np.testing.assert_array_equal(sep, want)
    assert want.mean() > 0.9   # axis-aligned crops: (nearly) all separable


def test_device_geometry_score_rule():
    """Detector best rows {x1, y1, x2, y2, score, prior}: score > bbox_thr keeps the box,
    anything else (including score == thr and the detector's -1 'none') is the whole image."""
    b = _boxes(8, 3)
    b[3] = (10, 20, 300, 400)
    score = np.array([0.9, 0.3, 0.31, -1.0, 0.5, 0.29, 0.7, 1.0], np.float32)
    rows = np.concatenate([b, score[:, None], np.arange(8, dtype=np.float32)[:, None]], 1)
    got = _device_geometry(rows, score_col=4, thr=0.3)
    hb = b.astype(np.float64)
    hb[~(score > np.float32(0.3))] = (0, 0, 1280, 720)
    want = geometry.crop_geometry_batch(hb)
    for g, w in zip(got[:3], want):
        np.testing.assert_array_equal(g, w)


def test_run_with_device_boxes_equals_host_boxes():
    """BatchPoseEstimator.run with the detector's device rows (+ bbox_thr) = run with the
    same boxes handed over from the host (NaN rows where the score fails)."""
    from mvpose import hrnet, synthetic as syn
    from mvpose.estimator import BatchPoseEstimator
    n = 6
    est = BatchPoseEstimator(hrnet.random_state_dict(41), max_frames=n)
    frames = torch.tensor(syn.make_frames(n, seed=44), device="cuda")
    b = _boxes(n, 5)
    b[3] = (50, 60, 700, 710)
    score = np.array([0.9, 0.2, 0.8, 0.6, 0.31, 0.05], np.float32)
    rows = torch.tensor(np.concatenate([b, score[:, None], np.zeros((n, 1), np.float32)], 1), device="cuda")
    a = est.run(frames, bboxes=rows, bbox_thr=0.3)
    ka, ga = a["keypoints"].clone(), a["gaussians"].clone()
    host = b.astype(np.float64)
    host[~(score > np.float32(0.3))] = np.nan
    h = est.run(frames, bboxes=host)
    torch.cuda.synchronize()
    assert torch.equal(ka, h["keypoints"])
    assert torch.equal(ga, h["gaussians"])
