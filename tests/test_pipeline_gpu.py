"""GPU: the multi-view pipeline end to end on synthetic frames; every stage
boundary is re-checked against the oracle fed with the GPU's own upstream
output (bf16 backbone numerics differ from fp32, so stages are chained)."""
import numpy as np
import pytest
import torch

from oracle import cv_ref, heatmap_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pipe():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import pipeline, synthetic as syn
    cams = syn.make_rig(2, seed=3)
    p = pipeline.MultiViewPipeline(syn.reference_camera_params(cams), max_frames=8, seed=5)
    return p, cams, syn


def test_pipeline_shapes_and_chain(pipe):
    p, cams, syn = pipe
    T = 4
    frames = torch.tensor(syn.make_frames(T * 2, seed=1).reshape(T, 2, 720, 1280, 3), device="cuda")
    out = p.process(frames)
    torch.cuda.synchronize()
    k2, hm2, k3 = (out[k].cpu().numpy() for k in ("kpts_2d", "heatmaps_2d", "kpts_3d"))
    assert k2.shape == (T, 17, 3, 2) and k2.dtype == np.float32
    assert hm2.shape == (T, 2, 17, 6) and hm2.dtype == np.float64
    assert k3.shape == (T, 17, 3) and k3.dtype == np.float32
    # decode chain: GPU flip-averaged heatmaps -> oracle decode == GPU keypoints
    avg = p.estimator.avg[: T * 2].cpu().numpy()
    g = p.estimator.geometry
    for i in range(T * 2):
        rk, rs, _ = heatmap_ref.msra_decode(avg[i])
        np.testing.assert_array_equal(k2[i // 2, :, :2, i % 2], heatmap_ref.keypoints_to_image(rk, g.center, g.scale))
        np.testing.assert_array_equal(k2[i // 2, :, 2, i % 2], rs)
    # triangulation chain: GPU kpts_2d -> oracle get_pose_3D
    ref3 = cv_ref.get_pose_3D(syn.reference_camera_params(cams), k2, camera_indices=[0, 1])
    np.testing.assert_allclose(k3, ref3, rtol=1e-5, atol=1e-4, equal_nan=True)


def test_predict_contract(pipe):
    """The reference's per-frame callable contract (pose_estimation.py:88, :104-110)."""
    p, _, syn = pipe
    inst, hm = p.estimator.predict(syn.make_frames(1, seed=2)[0])
    assert inst["keypoints"].shape == (1, 17, 2) and inst["keypoints"].dtype == np.float32
    assert inst["keypoint_scores"].shape == (1, 17)
    assert hm.shape == (17, 6) and hm.dtype == np.float64


def test_overlapped_moments_match_serial(pipe):
    """overlap_moments=True (moments on a side stream beside the next batch, double-buffered
    heatmaps) gives bit-identical outputs to the serial path, across buffer reuse."""
    p, _, syn = pipe
    T = 4
    fa = torch.tensor(syn.make_frames(T * 2, seed=11).reshape(T, 2, 720, 1280, 3), device="cuda")
    fb = torch.tensor(syn.make_frames(T * 2, seed=12).reshape(T, 2, 720, 1280, 3), device="cuda")
    serial = [{k: v.clone() for k, v in p.process(f).items()} for f in (fa, fb)]
    outs = [p.process(f, {}, overlap_moments=True) for f in (fa, fb, fa, fb)]
    for o in outs:
        assert o["moments_done"] is not None
        p.wait(o)
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        ref = serial[i % 2]
        for k in ("kpts_2d", "heatmaps_2d", "kpts_3d"):
            assert torch.equal(torch.nan_to_num(o[k]), torch.nan_to_num(ref[k])), (i, k)
    assert "moments_done" not in p.process(fa, outs[0])
