"""CPU: host-side logic of the product package (no GPU calls)."""
import os
import pickle

import numpy as np
import pytest
import torch

from oracle import heatmap_ref, hrnet_ref
from mvpose import geometry, hrnet


def test_crop_geometry_matches_oracle():
    g = geometry.CropGeometry.whole_image(1280, 720)
    M, c, s = heatmap_ref.topdown_crop_matrix(1280, 720)
    np.testing.assert_array_equal(g.center, c)
    np.testing.assert_array_equal(g.scale, s)
    np.testing.assert_array_equal(g.crop_minv, heatmap_ref.invert_affine(M))
    Mh = heatmap_ref.get_warp_matrix(c, s, 0.0, (48, 64), inv=True)
    np.testing.assert_array_equal(g.revert_minv, heatmap_ref.invert_affine(Mh))
    # whole 1280x720 frame -> 1600x2133.3 bbox -> 0.12 crop scale
    assert abs(g.crop_minv[0] - 1 / 0.12) < 1e-9


def test_graph_matches_oracle_topology():
    sd = hrnet.random_state_dict(0)
    model = hrnet_ref.build(sd)  # loads with strict=True -> names/shapes agree with mmpose naming
    rows = hrnet_ref.conv_macs(model)
    spec, x_in, out = hrnet.build_hrnet_w32(sd)
    convs = [op for op in spec.ops if op["kind"] in (hrnet.OP_CONV, hrnet.OP_STEM)]
    assert len(convs) == len(rows) == 293
    macs_spec = sum(spec.tensors[op["out"]][0] * spec.tensors[op["out"]][1] * op["cout"] *
                    (3 if op["kind"] == hrnet.OP_STEM else op["cin"]) * op["ks"] ** 2 for op in convs)
    assert macs_spec == sum(r[-1] for r in rows)
    assert spec.tensors[out] == (64, 48, 17, hrnet.DT_F32)
    fuses = [op for op in spec.ops if op["kind"] == hrnet.OP_FUSE]
    assert len(fuses) == 2 + 4 * 3 + 2 * 4 + 1


def test_bn_folding():
    sd = hrnet.random_state_dict(1)
    w, b = hrnet.fold_bn(sd, "backbone.conv2", "backbone.bn2")
    conv = torch.nn.Conv2d(64, 64, 3, 2, 1, bias=False).double()
    bn = torch.nn.BatchNorm2d(64).double().eval()
    conv.weight.data = sd["backbone.conv2.weight"].double()
    for k in ("weight", "bias", "running_mean", "running_var"):
        getattr(bn, k).data = sd["backbone.bn2." + k].double()
    x = torch.randn(1, 64, 9, 7, dtype=torch.float64)
    ref = bn(conv(x))
    fused = torch.nn.functional.conv2d(x, torch.from_numpy(w).permute(0, 3, 1, 2), torch.from_numpy(b), 2, 1)
    torch.testing.assert_close(fused, ref, rtol=1e-10, atol=1e-10)


def test_bf16_rounding():
    a = np.array([1.0, 1.00390625, 1.005859375, -2.5, 3.0e-20], np.float32)
    bits = hrnet.to_bf16_bits(a)
    back = torch.from_numpy(bits.view(np.int16)).view(torch.bfloat16).float().numpy()
    np.testing.assert_array_equal(back, torch.tensor(a).bfloat16().float().numpy())


def test_calibration_files_roundtrip(tmp_path):
    K = np.array([[1000.5, 0, 640.25], [0, 999.0, 360.0], [0, 0, 1.0]])
    dist = np.array([[0.1, -0.02, 0.001, -0.0005, 0.003]])
    R = np.eye(3)
    T = np.array([[1.5], [2.0], [-3.25]])
    geometry.write_camera_parameters("camA", K, dist, str(tmp_path / "intr"))
    geometry.write_rotation_translation("camA", R, T, str(tmp_path / "extr"))
    P, (K2, R2, T2, d2) = geometry.get_params_from_name("camA", str(tmp_path / "intr"), str(tmp_path / "extr"))
    np.testing.assert_array_equal(K2, K)
    np.testing.assert_array_equal(d2, dist)
    np.testing.assert_array_equal(T2, T)
    np.testing.assert_allclose(P, K @ np.hstack([R, T]))
    geometry.save_camera_names(str(tmp_path / "extr"), {0: "camA", 1: "camB"}, "camA")
    names, origin = geometry.load_camera_names(str(tmp_path / "extr"))
    assert names == {0: "camA", 1: "camB"} and origin == "camA"


def test_camera_names_loader_rejects_code(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))
    d = tmp_path / "x"
    d.mkdir()
    with open(d / "camera_names.pkl", "wb") as f:
        pickle.dump(({0: Evil()}, "a"), f)
    with pytest.raises(pickle.UnpicklingError):
        geometry.load_camera_names(str(d))


def _random_boxes(n, seed):
    rng = np.random.default_rng(seed)
    x1 = rng.uniform(-150, 1250, n)
    y1 = rng.uniform(-100, 700, n)
    return np.stack([x1, y1, x1 + rng.uniform(0.5, 1400, n), y1 + rng.uniform(0.5, 800, n)], 1).astype(np.float32)


def test_crop_geometry_batch_matches_oracle_per_box():
    """geometry.crop_geometry_batch (the host twin of mvp_bbox_geometry) = the oracle's
    mmpose bbox_xyxy2cs -> _fix_aspect_ratio -> get_warp_matrix (OpenCV LU) ->
    warpAffine inversion, bit for bit, box by box (f32 boxes as mmdet returns them)."""
    bb = _random_boxes(200, 1)
    cm, rm, cs = geometry.crop_geometry_batch(bb)
    for i in range(len(bb)):
        c, s = heatmap_ref.bbox_xyxy2cs(bb[i])
        s = heatmap_ref.fix_aspect_ratio(s, 192 / 256)
        np.testing.assert_array_equal(cs[i], np.r_[c, s].astype(np.float32))
        np.testing.assert_array_equal(cm[i], heatmap_ref.invert_affine(heatmap_ref.get_warp_matrix(c, s, 0.0, (192, 256))))
        np.testing.assert_array_equal(
            rm[i], heatmap_ref.invert_affine(heatmap_ref.get_warp_matrix(c, s, 0.0, (48, 64), inv=True)))


def test_lu_solve_batch_is_opencv_lu():
    """The vectorised LU = the oracle's scalar OpenCV LUImpl restatement on general systems
    (pivoting exercised), and a singular system gives zeros like cv::solve's failure."""
    rng = np.random.default_rng(2)
    A = rng.normal(size=(50, 6, 6)) * rng.uniform(0.1, 100, (50, 1, 6))
    b = rng.normal(size=(50, 6))
    A[7] = 0.0
    A[7, :, 0] = 1.0
    got = geometry.lu_solve_batch(A, b)
    for i in range(50):
        np.testing.assert_array_equal(got[i], heatmap_ref.cv_lu_solve(A[i], b[i]))
    assert not got[7].any()
    np.testing.assert_allclose(got[:7], np.linalg.solve(A[:7], b[:7, :, None])[..., 0], rtol=1e-9, atol=1e-12)


def test_detector_checkpoint_must_be_local(monkeypatch):
    """The reference always builds its detector (mmpose_pose_estimation.py:98-99): a
    det_checkpoint that is not a local file raises instead of silently cropping the whole
    image; MVPOSE_NO_DETECTOR=1 / using_detector=False are the explicit opt-outs."""
    from mvpose.mmpose_pose_estimation import PoseEstimator, build_detector
    monkeypatch.delenv("MVPOSE_RANDOM_DETECTOR", raising=False)
    url = "https://download.openmmlab.com/mmpose/v1/projects/rtmpose/rtmdet_m_8xb32-100e_coco-obj365-person.pth"
    with pytest.raises(FileNotFoundError):
        build_detector(url)
    with pytest.raises(FileNotFoundError):
        PoseEstimator("rtmdet_m.py", url, "hrnet.py", "hrnet.pth")
    monkeypatch.setenv("MVPOSE_RANDOM_WEIGHTS", "1")
    monkeypatch.setenv("MVPOSE_NO_DETECTOR", "1")
    pe = PoseEstimator("rtmdet_m.py", url, "hrnet.py", "hrnet.pth")
    assert pe.detector is None and not pe.using_detector


def test_build_estimator_from_model_yaml(tmp_path, monkeypatch):
    """estimate_pose_from_video's model-name path (pose_estimation.py:290-297): the detector
    and the pose model come from model_yaml; estimator objects and their bound predict pass
    through unchanged (no yaml lookup)."""
    import yaml as _yaml
    from mvpose import pose_estimation as pe_mod
    from mvpose.mmpose_pose_estimation import PoseEstimator
    y = tmp_path / "model_paths.yaml"
    _yaml.safe_dump({"detectors": {"coco_base": ["rtmdet_m.py", str(tmp_path / "missing_det.pth")]},
                     "pose_estimators": {"coco_base": ["hrnet.py", str(tmp_path / "missing_pose.pth")]}},
                    open(y, "w"))
    monkeypatch.delenv("MVPOSE_RANDOM_DETECTOR", raising=False)
    monkeypatch.delenv("MVPOSE_NO_DETECTOR", raising=False)
    monkeypatch.setenv("MVPOSE_RANDOM_WEIGHTS", "1")
    with pytest.raises(FileNotFoundError, match="detector checkpoint"):
        pe_mod.build_estimator("coco_base", "coco_base", str(y))
    monkeypatch.setenv("MVPOSE_NO_DETECTOR", "1")
    est = pe_mod.build_estimator("coco_base", "coco_base", str(y), max_frames=8)
    assert isinstance(est, PoseEstimator) and est.detector is None
    assert pe_mod.build_estimator(est) is est
    assert pe_mod.build_estimator(est.predict) is est
    assert pe_mod.resolve_estimator(lambda f: None) is None
