"""GPU: per-crop person boxes through BatchPoseEstimator.run(bboxes=...) — the
reference's detector -> inference_topdown hand-off (mmpose_pose_estimation.py:242-253:
first person bbox, else the whole image).  Off-centre, non-aspect, partly
out-of-frame and missing (NaN = whole image) boxes in one batch; each stage is
checked against the oracle restated for that box:
* crop + normalise (mvp_preprocess): bit-exact bf16, original and flipped;
* flip-average + MSRA decode + restore with the box's center/scale: bit-exact;
* revert + moments with the box's inverse map: the tolerances of
  test_stage2d_gpu.py::test_moments_full_frame_vs_oracle."""
import numpy as np
import pytest
import torch

from oracle import heatmap_ref

pytestmark = pytest.mark.gpu

BOXES = np.array([[100.5, 50.25, 400.0, 700.0],      # tall, off-centre
                  [500.0, 100.0, 1200.0, 220.0],     # wide (aspect fixed by height growth)
                  [-80.0, 300.0, 260.0, 900.0],      # partly outside the frame
                  [np.nan, np.nan, np.nan, np.nan],  # no detection -> whole image
                  [640.0, 360.0, 650.0, 371.0],      # tiny
                  [0.0, 0.0, 1280.0, 720.0]])        # explicit whole image


def _oracle_geometry(box, W=1280, H=720):
    if not np.isfinite(box).all():
        box = np.array([0.0, 0.0, W, H])
    center, scale = heatmap_ref.bbox_xyxy2cs(box)
    scale = heatmap_ref.fix_aspect_ratio(scale, 192 / 256)
    M = heatmap_ref.get_warp_matrix(center, scale, 0.0, (192, 256))
    Mh = heatmap_ref.get_warp_matrix(center, scale, 0.0, (48, 64), inv=True)
    return center, scale, M, Mh


@pytest.fixture(scope="module")
def run():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import hrnet, synthetic as syn
    from mvpose.estimator import BatchPoseEstimator
    n = len(BOXES)
    est = BatchPoseEstimator(hrnet.random_state_dict(41), max_frames=n)
    frames = syn.make_frames(n, seed=43)
    r = est.run(torch.tensor(frames, device="cuda"), argmax=True, bboxes=BOXES)
    torch.cuda.synchronize()
    out = {k: r[k].cpu().numpy() for k in ("keypoints", "scores", "gaussians", "argmax")}
    out["avg"] = est.avg[:n].cpu().numpy()
    out["crops"] = est.crops[: 2 * n].float().cpu().numpy()
    return est, frames, out


def test_bbox_preprocess_bit_exact(run):
    _, frames, out = run
    n = len(BOXES)
    for i, box in enumerate(BOXES):
        _, _, M, _ = _oracle_geometry(box)
        ref = np.moveaxis(torch.tensor(heatmap_ref.preprocess(frames[i], M)).bfloat16().float().numpy(), 0, -1)
        np.testing.assert_array_equal(out["crops"][i, :, :, :3], ref, err_msg=f"box {i}")
        np.testing.assert_array_equal(out["crops"][n + i, :, :, :3], ref[:, ::-1], err_msg=f"box {i} flipped")


def test_bbox_decode_bit_exact(run):
    _, _, out = run
    for i, box in enumerate(BOXES):
        center, scale, _, _ = _oracle_geometry(box)
        rk, rs, ri = heatmap_ref.msra_decode(out["avg"][i])
        np.testing.assert_array_equal(out["argmax"][i], ri)
        np.testing.assert_array_equal(out["scores"][i], rs)
        np.testing.assert_array_equal(out["keypoints"][i], heatmap_ref.keypoints_to_image(rk, center, scale),
                                      err_msg=f"box {i}")


def test_bbox_moments_vs_oracle(run):
    _, _, out = run
    for i, box in enumerate(BOXES):
        _, _, _, Mh = _oracle_geometry(box)
        rev = heatmap_ref.warp_affine_linear_f32(out["avg"][i], Mh, 720, 1280)
        ref = heatmap_ref.heatmap_means_cov_f64(rev)
        got = out["gaussians"][i]
        np.testing.assert_allclose(got[:, :2], ref[:, :2], rtol=2e-6, atol=1e-6, err_msg=f"box {i}")
        scale = (ref[:, 0] ** 2 + ref[:, 1] ** 2)[:, None]
        assert np.all(np.abs(got[:, 2:] - ref[:, 2:]) <= 2e-6 * np.abs(ref[:, 2:]) + 1e-9 * scale + 1e-9), i


def test_bbox_overlapped_runs_match(run):
    """Double-buffered geometry: alternating box sets with the side-stream moments give
    the serial results."""
    est, frames, out = run
    fd = torch.tensor(frames, device="cuda")
    other = BOXES[::-1].copy()
    ser_b = est.run(fd, bboxes=other)["gaussians"].clone()
    rs = [est.run(fd, bboxes=b, overlap_moments=True) for b in (BOXES, other, BOXES, other)]
    for r in rs:
        est.wait_moments(r)
    torch.cuda.synchronize()
    for j, r in enumerate(rs):
        want = out["gaussians"] if j % 2 == 0 else ser_b.cpu().numpy()
        np.testing.assert_array_equal(r["gaussians"].cpu().numpy(), want)
