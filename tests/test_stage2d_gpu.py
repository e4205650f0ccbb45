"""GPU parity of the 2D-stage kernels vs the oracle / golden vectors:
preprocess (bit-exact bf16), heatmap decode (argmax bit-exact), moments
(reference get_heatmap_means_cov golden, fp32-summation tolerance)."""
import ctypes
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import heatmap_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import _lib, geometry
    return _lib, geometry


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _s():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def test_preprocess_bit_exact(lib):
    _lib, geometry = lib
    rng = np.random.default_rng(0)
    frames = rng.integers(0, 256, (3, 720, 1280, 3), dtype=np.uint8)
    g = geometry.CropGeometry.whole_image(1280, 720)
    fd = torch.tensor(frames, device="cuda")
    minv = torch.tensor(np.tile(g.crop_minv, (3, 1)), device="cuda")
    out = torch.empty((6, 256, 192, 4), dtype=torch.bfloat16, device="cuda")
    mean = (ctypes.c_float * 3)(*heatmap_ref.MEAN_RGB)
    std = (ctypes.c_float * 3)(*heatmap_ref.STD_RGB)
    _lib.call("mvp_preprocess", _p(fd), 3, 720, 1280, _p(minv), 256, 192, mean, std, 1, 1, _p(out), _s())
    torch.cuda.synchronize()
    M, _, _ = heatmap_ref.topdown_crop_matrix(1280, 720)
    o = out.float().cpu().numpy()
    for i in range(3):
        ref = heatmap_ref.preprocess(frames[i], M)  # (3, 256, 192) f32
        ref_bf = torch.tensor(ref).bfloat16().float().numpy()
        np.testing.assert_array_equal(o[i, :, :, :3], np.moveaxis(ref_bf, 0, -1))
        np.testing.assert_array_equal(o[i + 3, :, :, :3], np.moveaxis(ref_bf, 0, -1)[:, ::-1])
        assert (o[i, :, :, 3] == 0).all()


def _planted_heatmaps(rng, n, K=17, H=64, W=48):
    hm = rng.normal(0, 0.05, (n, K, H, W)).astype(np.float32)
    for i in range(n):
        for k in range(K):
            y, x = rng.integers(0, H), rng.integers(0, W)
            hm[i, k, y, x] += rng.uniform(0.5, 1.0)
    hm[0, 0] = 0.25                      # all-equal map -> first occurrence
    hm[0, 1, 10, 10] = hm[0, 1, 20, 5] = 5.0  # exact tie
    hm[0, 2] = -0.5                      # max <= 0 -> (-1, -1)
    hm[0, 3, 0, 0] = 9.0                 # max on the border -> no refinement
    return hm


def test_decode_vs_oracle(lib):
    _lib, geometry = lib
    rng = np.random.default_rng(1)
    n = 8
    hm = _planted_heatmaps(rng, n)
    hmf = _planted_heatmaps(rng, n)
    g = geometry.CropGeometry.whole_image(1280, 720)
    cs = torch.tensor(np.tile(g.center_scale, (n, 1)), device="cuda")
    hd, hfd = torch.tensor(hm, device="cuda"), torch.tensor(hmf, device="cuda")
    avg = torch.empty_like(hd)
    kp = torch.empty((n, 17, 2), device="cuda")
    sc = torch.empty((n, 17), device="cuda")
    am = torch.empty((n, 17), dtype=torch.int32, device="cuda")
    tkv = torch.empty((n // 2, 17, 3, 2), device="cuda")
    flip = (ctypes.c_int * 17)(*heatmap_ref.COCO_FLIP_INDICES)
    _lib.call("mvp_heatmap_decode", _p(hd), _p(hfd), n, 17, 64, 48, flip, 1, _p(cs), 192, 256, _p(avg), _p(kp),
              _p(sc), _p(am), _p(tkv), 2, _s())
    torch.cuda.synchronize()
    ref_avg = heatmap_ref.flip_test_average(hm, hmf)
    np.testing.assert_array_equal(avg.cpu().numpy(), ref_avg)
    for i in range(n):
        rk, rs, ri = heatmap_ref.msra_decode(ref_avg[i])
        np.testing.assert_array_equal(am[i].cpu().numpy(), ri)
        np.testing.assert_array_equal(sc[i].cpu().numpy(), rs)
        img = heatmap_ref.keypoints_to_image(rk, g.center, g.scale)
        np.testing.assert_array_equal(kp[i].cpu().numpy(), img)
    t = tkv.cpu().numpy()
    k_np, s_np = kp.cpu().numpy(), sc.cpu().numpy()
    for i in range(n):
        np.testing.assert_array_equal(t[i // 2, :, :2, i % 2], k_np[i])
        np.testing.assert_array_equal(t[i // 2, :, 2, i % 2], s_np[i])


def _moments(_lib, hm, minv, img_h, img_w, separable=None):
    from mvpose.estimator import warp_is_separable
    if separable is None:
        separable = warp_is_separable(minv, img_h, img_w)
    N, K, h, w = hm.shape
    hd = torch.tensor(np.ascontiguousarray(hm), device="cuda")
    md = torch.tensor(np.tile(minv, (N, 1)), device="cuda")
    out = torch.empty((N, K, 6), dtype=torch.float64, device="cuda")
    _lib.call("mvp_heatmap_moments", _p(hd), N, K, h, w, _p(md), img_h, img_w, ctypes.c_float(0.01), int(separable),
              None, _p(out), _s())
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _check_moments(out, ref):
    # reference sums 1e4-1e6 f32 terms (numpy / torch pairwise): ~1e-6 relative
    np.testing.assert_allclose(out[:, :2], ref[:, :2], rtol=0, atol=2e-3)
    np.testing.assert_allclose(out[:, 2:], ref[:, 2:], rtol=2e-4, atol=2e-3)


def test_moments_golden_identity_warp(lib):
    _lib, _ = lib
    d = np.load(os.path.join(GOLDEN, "moments.npz"))
    hm = d["hm_full"][None]  # (1,17,72,128) used directly as the image-space map
    out = _moments(_lib, hm, np.array([1.0, 0, 0, 0, 1.0, 0]), 72, 128)
    _check_moments(out[0], d["out_full"])
    assert (out[0, -1] == 0).all()  # all-below-threshold joint -> zeros


def test_moments_golden_revert(lib):
    _lib, geometry = lib
    d = np.load(os.path.join(GOLDEN, "moments.npz"))
    img_h, img_w = [int(v) for v in d["img_hw"]]
    minv = geometry.inverse_map(d["M_inv"])
    out = _moments(_lib, d["hm_low"][None], minv, img_h, img_w)
    _check_moments(out[0], d["out_rev"])


@pytest.mark.parametrize("kind", ["dense", "peaked", "threshold"])
@pytest.mark.parametrize("separable", [True, False])
def test_moments_full_frame_vs_oracle(lib, kind, separable):
    """1280x720 revert of a 64x48 map against oracle warp + fp64 moments, on both
    kernel paths (the separable column-resident path with bbox culling and per-run
    closed forms, and the general per-pixel path); dense maps (every pixel above
    threshold: closed forms), peaked maps (small active region, culling exercised)
    and maps whose taps sit at and around the threshold (thr, thr·(1 ± 1e-6),
    thr·(1 ± 3e-6): the classification margins and the per-row walk)."""
    _lib, geometry = lib
    rng = np.random.default_rng(3)
    hm = _planted_heatmaps(rng, 1)
    if kind == "dense":
        hm = np.abs(hm) + 0.02
    elif kind == "threshold":
        # the separable path evaluates a pixel as gy·a + fy·b, within ~2 f32 ulps of
        # OpenCV's four-product order: a map whose every cell straddles the threshold by a
        # few ulps flips thousands of pixels there, by design (documented tolerance)
        if separable:
            pytest.skip("near-threshold maps: exact-order path here, separable path in "
                        "test_moments_closed_form_matches_walk")
        near = np.float32(0.01) * (1 + np.array([0, 1e-6, -1e-6, 3e-6, -3e-6, 1e-3, -1e-3], np.float32))
        hm = rng.choice(near, size=hm.shape).astype(np.float32)
    else:
        yy, xx = np.mgrid[0:64, 0:48]
        for k in range(17):
            cy, cx = rng.uniform(5, 59), rng.uniform(5, 43)
            hm[0, k] = np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * 2.0 ** 2)) - 0.005
    g = geometry.CropGeometry.whole_image(1280, 720)
    assert geometry is not None
    out = _moments(_lib, hm, g.revert_minv, 720, 1280, separable=separable)
    Mh = heatmap_ref.get_warp_matrix(g.center, g.scale, 0.0, (48, 64), inv=True)
    rev = heatmap_ref.warp_affine_linear_f32(hm[0], Mh, 720, 1280)
    ref = heatmap_ref.heatmap_means_cov_f64(rev)
    # f32 partial sums per run of rows sharing a source row (flushed to fp64), and the
    # separable path's fma-contracted interpolation (gy*a + fy*b: each revert pixel within
    # ~1 ulp of the oracle's four-product order): ~1e-9 relative on the raw second
    # moments, whose magnitude is ~ mean^2 — a covariance (difference of second moments)
    # is judged against that scale.  Still ~1e5x tighter than the reference's own f32
    # moments (~1e-3 px^2 off at this scale, golden test above: rtol 2e-4, atol 2e-3).
    np.testing.assert_allclose(out[0][:, :2], ref[:, :2], rtol=2e-6, atol=1e-6)
    scale = (ref[:, 0] ** 2 + ref[:, 1] ** 2)[:, None]
    assert np.all(np.abs(out[0][:, 2:] - ref[:, 2:]) <= 2e-6 * np.abs(ref[:, 2:]) + 1e-9 * scale + 1e-9)


@pytest.mark.parametrize("kind", ["dense", "peaked", "threshold", "random"])
def test_moments_closed_form_matches_walk(lib, kind):
    """Separable path: the per-run closed forms (columns whose 4 taps are all >= thr·(1+2e-6)
    summed as a·G + b·F, all < thr·(1-2e-6) skipped) against walking every row of every
    column with the same pixel formula (separable=2): identical threshold decisions, so
    only the f32/fp64 summation differs."""
    _lib, geometry = lib
    rng = np.random.default_rng(9)
    hm = _planted_heatmaps(rng, 2)
    if kind == "dense":
        hm = np.abs(hm) + 0.02
    elif kind == "threshold":
        near = np.float32(0.01) * (1 + np.array([0, 1e-6, -1e-6, 2e-6, -2e-6, 3e-6, -3e-6, 1e-3], np.float32))
        hm = rng.choice(near, size=hm.shape).astype(np.float32)
    elif kind == "random":
        hm = (rng.standard_normal(hm.shape) * 0.05).astype(np.float32)
    g = geometry.CropGeometry.whole_image(1280, 720)
    fast = _moments(_lib, hm, g.revert_minv, 720, 1280, separable=1)
    walk = _moments(_lib, hm, g.revert_minv, 720, 1280, separable=2)
    np.testing.assert_allclose(fast[..., :2], walk[..., :2], rtol=1e-6, atol=1e-6)
    scale = (walk[..., 0] ** 2 + walk[..., 1] ** 2)[..., None]
    assert np.all(np.abs(fast[..., 2:] - walk[..., 2:]) <= 1e-6 * np.abs(walk[..., 2:]) + 1e-9 * scale + 1e-9)


@pytest.mark.parametrize("jpb", [1, 4, 5, 17])
@pytest.mark.parametrize("separable", [1, 0])
def test_moments_joints_per_block_bit_identical(lib, jpb, separable, monkeypatch):
    """Workgroups that build the crop's warp tables once and reuse them for jpb joints
    (ragged last group for 4 and 5) give bit-identical moments to one map per workgroup;
    frames carry different warps, so tables must not leak across crops."""
    _lib, geometry = lib
    rng = np.random.default_rng(21)
    hm = _planted_heatmaps(rng, 3)
    g = geometry.CropGeometry.whole_image(1280, 720)
    minv = np.tile(g.revert_minv, (3, 1))
    minv[1, 2] += 3.7
    minv[1, 5] -= 2.1
    minv[2, 0] *= 1.01
    hd = torch.tensor(hm, device="cuda")
    md = torch.tensor(minv, device="cuda")

    def run(j):
        monkeypatch.setenv("MVPOSE_MOM_JPB", str(j))
        out = torch.full((3, 17, 6), float("nan"), dtype=torch.float64, device="cuda")
        _lib.call("mvp_heatmap_moments", _p(hd), 3, 17, 64, 48, _p(md), 720, 1280, ctypes.c_float(0.01),
                  separable, None, _p(out), _s())
        torch.cuda.synchronize()
        return out.cpu().numpy()

    ref = run(1)
    assert not np.isnan(ref).any()
    np.testing.assert_array_equal(run(jpb), ref)
