"""GPU: the reference-named Python drop-ins called through the reference's own
signatures, against the oracle / the batched GPU path:
* utils.triangulate_points(kpts_2d, cmtx1, dist1, R1, T1, cmtx2, dist2, R2, T2)
  (ref utils.py:1277) vs oracle/cv_ref.triangulate_points (<= 1e-4, any leading shape);
* mmpose_pose_estimation.PoseEstimator(det_config, det_checkpoint, pose_config,
  pose_checkpoint, ...) (ref mmpose_pose_estimation.py:82) loading a local checkpoint
  (weights_only) — predict(frame) == the batched estimator; the detector hand-off rule
  (:242-250) with a detections callable; predict(return_full_heatmaps=True) == oracle
  revert of the same maps (bit-exact) and get_heatmap_means_cov on it ~ the fused moments;
* pose_estimation.get_pose_2D(frames, model) (ref pose_estimation.py:71) with the GPU
  estimator and with a generic per-frame callable: (17, 3, V) stacks equal the pipeline's
  kpts_2d.
"""
import numpy as np
import pytest
import torch

from oracle import cv_ref, heatmap_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import hrnet, synthetic as syn
    sd = hrnet.random_state_dict(61)
    ck = tmp_path_factory.mktemp("ck") / "hrnet_w32_random.pth"
    torch.save({"state_dict": sd, "meta": {"note": "synthetic"}}, ck)
    return sd, str(ck), syn


def test_triangulate_points_signature(env):
    from mvpose import utils
    _, _, syn = env
    cams = syn.make_rig(2, seed=9)
    poses = syn.make_poses(6, seed=10)
    k = syn.make_kpts_2d(poses, cams, seed=11)            # (6, 17, 3, 2)
    pts = np.moveaxis(k[:, :, :2, :], -1, -2)            # (6, 17, 2 cams, 2)
    args = []
    for c in cams:
        args += [c["K"], c["dist"], c["R"], c["T"]]
    got = utils.triangulate_points(pts, *args)
    ref = cv_ref.triangulate_points(pts, *args)
    assert got.shape == (6, 17, 3) and got.dtype == np.float32
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-4)
    one = utils.triangulate_points(torch.tensor(pts[2, 5]), *args)   # torch input, no leading dims
    assert one.shape == (3,)
    np.testing.assert_allclose(one, ref[2, 5], rtol=1e-5, atol=1e-4)


def test_pose_estimator_signature_and_checkpoint(env):
    from mvpose.estimator import BatchPoseEstimator
    from mvpose.mmpose_pose_estimation import PoseEstimator
    sd, ck, syn = env
    with pytest.raises(FileNotFoundError):   # the detector checkpoint is not a local file
        PoseEstimator("rtmdet_m.py", "rtmdet_m.pth", "td-hm_hrnet-w32.py", ck)
    pe = PoseEstimator("rtmdet_m.py", "rtmdet_m.pth", "td-hm_hrnet-w32.py", ck, using_detector=False)   # device='cpu'
    frame = syn.make_frames(1, seed=12)[0]
    inst, hm = pe(frame)
    ref = BatchPoseEstimator(sd, max_frames=1, swap_rb=False)
    rinst, rhm = ref.predict(frame)
    assert inst["keypoints"].shape == (1, 17, 2) and inst["keypoint_scores"].shape == (1, 17)
    np.testing.assert_array_equal(inst["keypoints"], rinst["keypoints"])
    np.testing.assert_array_equal(hm, rhm)
    assert hm.shape == (17, 6) and hm.dtype == np.float64


def test_detector_handoff_rule(env):
    from mvpose.mmpose_pose_estimation import PoseEstimator, select_person_bbox
    sd, ck, syn = env
    dets = np.array([[10, 10, 50, 80, 0.9, 1],      # not a person
                     [100, 40, 300, 650, 0.2, 0],   # person below bbox_thr
                     [400, 60, 700, 700, 0.8, 0],   # first person above 0.3 -> chosen
                     [20, 20, 900, 700, 0.95, 0]])
    np.testing.assert_array_equal(select_person_bbox(dets), np.float32([400, 60, 700, 700]))
    assert select_person_bbox(dets[:2]) is None
    pe = PoseEstimator(None, None, None, ck, detector=lambda f: dets, max_frames=1)
    frame = syn.make_frames(1, seed=13)[0]
    inst, _ = pe.predict(frame)
    direct = pe.estimator(frame.shape[:2]).run(torch.tensor(frame[None], device="cuda"),
                                               bboxes=[[400, 60, 700, 700]])
    np.testing.assert_array_equal(inst["keypoints"][0], direct["keypoints"][0].cpu().numpy())
    none = PoseEstimator(None, None, None, ck, detector=lambda f: dets[:2], max_frames=1)
    inst2, _ = none.predict(frame)
    whole = PoseEstimator(None, None, None, ck, using_detector=False, max_frames=1)
    inst3, _ = whole.predict(frame)
    np.testing.assert_array_equal(inst2["keypoints"], inst3["keypoints"])   # no person -> whole image


def test_full_heatmaps_and_means_cov(env):
    from mvpose.mmpose_pose_estimation import PoseEstimator
    _, ck, syn = env
    pe = PoseEstimator(None, None, None, ck, using_detector=False, max_frames=1)
    frame = syn.make_frames(1, seed=14)[0]
    _, gauss = pe.predict(frame)
    _, full = pe.predict(frame, return_full_heatmaps=True)
    est = pe.estimator(frame.shape[:2])
    avg = est.avg[0].cpu().numpy()
    g = est.geometry
    Mh = heatmap_ref.get_warp_matrix(g.center, g.scale, 0.0, (48, 64), inv=True)
    ref = heatmap_ref.warp_affine_linear_f32(avg, Mh, 720, 1280)
    assert full.shape == (17, 720, 1280) and full.dtype == np.float32
    np.testing.assert_array_equal(full, ref)
    mc = PoseEstimator.get_heatmap_means_cov(full.copy())
    # torch-f32 restatement of the reference's own f32 sums vs the fused fp64 kernel
    np.testing.assert_allclose(mc[:, :2], gauss[:, :2], rtol=0, atol=5e-2)
    np.testing.assert_allclose(mc[:, 2:], gauss[:, 2:], rtol=2e-3, atol=5e-1)


def test_get_pose_2D_batched_and_callable(env):
    from mvpose import pipeline
    from mvpose.mmpose_pose_estimation import PoseEstimator
    from mvpose.pose_estimation import get_pose_2D
    sd, ck, syn = env
    frames = syn.make_frames(2, seed=15)
    pe = PoseEstimator(None, None, None, ck, using_detector=False, max_frames=2)
    stacked, heat = get_pose_2D(list(frames), pe)
    assert stacked.shape == (17, 3, 2) and stacked.dtype == np.float32 and len(heat) == 2
    p = pipeline.MultiViewPipeline(syn.reference_camera_params(syn.make_rig(2, seed=1)),
                                   max_frames=2, state_dict=sd, swap_rb=False)
    out = p.process(torch.tensor(frames[None], device="cuda"))
    np.testing.assert_array_equal(stacked, out["kpts_2d"][0].cpu().numpy())
    np.testing.assert_array_equal(np.stack(heat), out["heatmaps_2d"][0].cpu().numpy())

    class PerFrame:  # a generic per-frame callable with the reference contract
        def __call__(self, f):
            return pe.predict(f)
    s2, h2 = get_pose_2D(list(frames), PerFrame(), confidence=0.9, pose_keypoints=range(5))
    np.testing.assert_array_equal(s2, stacked)
    np.testing.assert_array_equal(np.stack(h2), np.stack(heat))
