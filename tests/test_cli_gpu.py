"""GPU: the drop-in command lines end to end on a synthetic project directory.

record_and_estimate_pose (random weights, 2 cameras, decoded frames as .npy)
must write the reference's four outputs with the reference's shapes/dtypes,
and its kpts_3d must be the oracle's get_pose_3D of its kpts_2d (1e-4);
pose_refinement must then write kpts_3d_linear_interpolation.npy and
kpts_3d_SGD.npy equal to the library calls it wraps."""
import json
import os

import numpy as np
import pytest
import torch
import yaml

from conftest import GOLDEN
from oracle import cv_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def project(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import geometry, synthetic as syn
    root = tmp_path_factory.mktemp("proj")
    cams = syn.make_rig(2, seed=4)
    cfg = root / "configurations" / "1"
    ext = cfg / "extrinsic_camera_parameters"
    intr = root / "intrinsic_camera_parameters"
    names = ["camA", "camB"]
    for name, c in zip(names, cams):
        geometry.write_camera_parameters(name, c["K"], c["dist"], str(intr))
        geometry.write_rotation_translation(name, c["R"], c["T"], str(ext))
    geometry.save_camera_names(str(ext), {0: "camA", 1: "camB"}, "camA")
    rec = cfg / "recordings" / "0"
    rec.mkdir(parents=True)
    rng = np.random.default_rng(0)
    paths = []
    for v in range(2):
        p = rec / f"camera{v}.npy"
        np.save(p, rng.integers(0, 256, (4, 360, 640, 3), dtype=np.uint8))
        paths.append(str(p))
    return root, names, paths, cams


def test_record_and_estimate_pose_cli(project, monkeypatch):
    from mvpose import cli
    root, names, paths, cams = project
    monkeypatch.setenv("MVPOSE_RANDOM_WEIGHTS", "1")
    monkeypatch.chdir(root)
    log = cli.record_and_estimate_pose_main(["--camera_names", *names, "--configuration_number", "1",
                                             "--recording_paths", *paths])
    k2 = np.load(log["kpts_2d"])
    hm = np.load(log["heatmaps_2d"])
    k3 = np.load(log["kpts_3d"])
    assert k2.shape == (3, 17, 3, 2) and k2.dtype == np.float32      # last frame dropped ([0, -1])
    assert hm.shape == (3, 2, 17, 6) and hm.dtype == np.float64
    assert k3.shape == (3, 17, 3) and k3.dtype == np.float32
    with open(os.path.join(os.path.dirname(paths[0]), "recording_log.yaml")) as f:
        assert yaml.safe_load(f)["kpts_3d"] == log["kpts_3d"]
    from mvpose import synthetic as syn
    ref = cv_ref.get_pose_3D(syn.reference_camera_params(cams), k2, camera_indices=[0, 1])
    ok = np.isfinite(ref)
    np.testing.assert_allclose(k3[ok], ref[ok], rtol=0, atol=1e-4)


def test_pose_refinement_cli(project, monkeypatch):
    from mvpose import cli, refine
    from test_sgd_gpu import _problem
    root, names, paths, cams = project
    run = os.path.dirname(paths[0])
    # replace the random-weight outputs by a well-posed synthetic sequence on the same rig
    cam_list, gauss, init = _problem(2, 24, seed=11)
    cam_list = [[c["K"], c["R"], c["T"], c["dist"]] for c in cams]
    np.save(os.path.join(run, "kpts_3d.npy"), init)
    np.save(os.path.join(run, "heatmaps_2d.npy"), gauss)
    with open(os.path.join(GOLDEN, "body_part_lengths.json")) as f:
        lengths = json.load(f)
    with open(root / "body_part_lengths.yaml", "w") as f:
        yaml.safe_dump(lengths, f, sort_keys=False)
    sgd = {"lr": 0.01, "max_iter": 6, "lambda_smooth": 1e-6, "lambda_body_length": 1.0, "print_frequency": 1000}
    with open(root / "params.yaml", "w") as f:
        yaml.safe_dump({"SGD": sgd, "linear_interpolation": {"k": 5}}, f)
    monkeypatch.chdir(root)
    out = cli.pose_refinement_main(["--run_path", run, "--refinement_types", "SGD", "linear_interpolation",
                                    "--refinement_params_yaml", str(root / "params.yaml"),
                                    "--intrinsic_params_dir", str(root / "intrinsic_camera_parameters")])
    lin = np.load(out["linear_interpolation"])
    np.testing.assert_array_equal(lin, refine.linear_interpolation(init))
    got = np.load(out["SGD"])
    opt = refine.Optimized_3d_Pose_Estimation(gauss, init, decomposed_cam_params_initial=dict(enumerate(cam_list)),
                                              body_lengths=lengths["my_lengths"])
    opt.sgd_optimize(**{**sgd, "print_frequency": 10 ** 9})
    assert got.shape == (23, 17, 3)
    np.testing.assert_allclose(got, opt.best_trajectory.numpy(), rtol=0, atol=1e-5)


def test_avi_recordings_match_npy(project, monkeypatch, tmp_path):
    """The same frames as uncompressed AVIs (bit-exact decode, mvpose.video) give the same
    2D keypoints and Gaussians as the .npy recordings."""
    from mvpose import pose_estimation, video
    _, _, paths, _ = project
    monkeypatch.setenv("MVPOSE_RANDOM_WEIGHTS", "1")
    est = pose_estimation.build_estimator("random", frame_hw=(360, 640), max_frames=16)
    avis = []
    for v, p in enumerate(paths):
        a = str(tmp_path / f"camera{v}.avi")
        video.write_avi(a, np.load(p), codec="rgb")
        avis.append(a)
    k_npy, h_npy = pose_estimation.run_pose_est(est, recording_paths=paths)
    k_avi, h_avi = pose_estimation.run_pose_est(est, recording_paths=avis)
    assert k_npy.shape == (3, 17, 3, 2)
    np.testing.assert_array_equal(k_avi, k_npy)
    np.testing.assert_array_equal(h_avi, h_npy)
