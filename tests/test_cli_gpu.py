"""GPU: the drop-in command lines end to end on a synthetic project directory.

record_and_estimate_pose (random pose + detector weights, 2 cameras, decoded frames as .npy)
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
    monkeypatch.setenv("MVPOSE_RANDOM_DETECTOR", "1")
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
    monkeypatch.setenv("MVPOSE_NO_DETECTOR", "1")
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


def test_cli_runs_the_detector_like_the_reference(project, monkeypatch, tmp_path):
    """record_and_estimate_pose builds PoseEstimator(detector, pose model) from the model name
    (ref pose_estimation.py:290-297) and crops every camera-frame to its first person box
    (ref mmpose_pose_estimation.py:234-253).  With the seeded synthetic detector, the CLI's
    kpts_2d.npy / heatmaps_2d.npy equal the reference's own loop — get_pose_2D calling
    PoseEstimator.predict frame by frame (ref pose_estimation.py:184-190, :88) — bit for bit;
    frames with a box differ from the whole-frame run (MVPOSE_NO_DETECTOR=1), the others
    equal it."""
    from mvpose import cli
    from mvpose.mmpose_pose_estimation import PoseEstimator
    from mvpose.pose_estimation import get_pose_2D
    root, names, _, _ = project
    rec = root / "configurations" / "1" / "recordings" / "det"
    rec.mkdir(parents=True, exist_ok=True)
    rng = np.random.default_rng(7)
    stacks, paths = [], []
    for v in range(2):
        s = rng.integers(0, 256, (4, 720, 1280, 3), dtype=np.uint8)
        p = rec / f"camera{v}.npy"
        np.save(p, s)
        stacks.append(s)
        paths.append(str(p))
    monkeypatch.setenv("MVPOSE_RANDOM_WEIGHTS", "1")
    monkeypatch.setenv("MVPOSE_RANDOM_DETECTOR", "1")
    monkeypatch.delenv("MVPOSE_NO_DETECTOR", raising=False)
    monkeypatch.chdir(root)
    argv = ["--camera_names", *names, "--configuration_number", "1", "--recording_paths", *paths]
    log = cli.record_and_estimate_pose_main(argv)
    k2, hm = np.load(log["kpts_2d"]), np.load(log["heatmaps_2d"])
    assert k2.shape == (3, 17, 3, 2)
    pe = PoseEstimator(None, None, None, None, max_frames=2)        # the same seeded detector + pose weights
    assert pe.detector is not None
    for t in range(3):
        s2, h2 = get_pose_2D([stacks[0][t], stacks[1][t]], lambda f: pe.predict(f))
        np.testing.assert_array_equal(k2[t], s2, err_msg=f"frame {t}")
        np.testing.assert_array_equal(hm[t], np.stack(h2), err_msg=f"frame {t}")
    best = pe.bboxes_for(torch.from_numpy(np.stack([stacks[v][t] for t in range(3) for v in range(2)])).cuda())
    has_box = (best[:, 4] > 0.3).cpu().numpy().reshape(3, 2)
    monkeypatch.setenv("MVPOSE_NO_DETECTOR", "1")
    whole = np.load(cli.record_and_estimate_pose_main(argv)["kpts_2d"])
    print(f"camera-frames with a person box: {int(has_box.sum())}/6")
    assert has_box.any()
    for t in range(3):
        for v in range(2):
            same = np.array_equal(whole[t, :, :, v], k2[t, :, :, v])
            assert same != bool(has_box[t, v]), (t, v, bool(has_box[t, v]))


def _mp4v_recording(path, n_frames, w, h, seed):
    """A per-camera mp4v MP4 (the reference's *_synced.mp4, synchronize_videos.py:64,240) written
    from seeded coefficients and motion vectors by tests/mp4v_writer.py: I-VOP + P-VOPs."""
    import mp4v_writer as W
    rng = np.random.default_rng(seed)
    mw, mh = w // 16, h // 16

    def intra():
        b = np.zeros((6, 64), np.int64)
        for n in range(6):
            b[n, 0] = rng.integers(40, 160) if n < 4 else rng.integers(80, 140)
            m = rng.random(63) < 0.1
            b[n, 1:][m] = rng.integers(-6, 7, m.sum())
        return {"q": 4, "blocks": b, "ac_pred": False}

    def inter():
        b = np.zeros((6, 64), np.int64)
        m = rng.random((6, 64)) < 0.03
        b[m] = rng.integers(-3, 4, m.sum())
        return {"type": "inter", "mv": (int(rng.integers(-9, 10)), int(rng.integers(-9, 10))), "blocks": b}

    vw = W.VopWriter(w, h)
    samples = [vw.i_vop([[intra() for _ in range(mw)] for _ in range(mh)], 4)]
    samples += [vw.p_vop([[inter() for _ in range(mw)] for _ in range(mh)], 4, rounding=k % 2)
                for k in range(n_frames - 1)]
    with open(path, "wb") as f:
        f.write(W.mp4_file(W.vol_header(w, h), samples, w, h))


def test_mp4v_recordings_match_npy(project, monkeypatch, tmp_path):
    """f2 on the GPU path: record_and_estimate_pose on per-camera mp4v MP4 recordings (what the
    reference's synchronize_videos.py writes and utils.frame_generator reads back with
    cv.VideoCapture, utils.py:849-909) writes kpts_2d / heatmaps_2d / kpts_3d equal, bit for bit,
    to the run fed the same decoded frames as .npy stacks."""
    from mvpose import cli, video
    root, names, _, _ = project
    monkeypatch.setenv("MVPOSE_RANDOM_WEIGHTS", "1")
    monkeypatch.setenv("MVPOSE_NO_DETECTOR", "1")
    monkeypatch.chdir(root)
    runs = {}
    for kind in ("mp4", "npy"):
        rec = root / "configurations" / "1" / "recordings" / f"mp4v_{kind}"
        rec.mkdir(parents=True, exist_ok=True)
        paths = []
        for v in range(2):
            mp4 = tmp_path / f"camera{v}_synced.mp4"
            if kind == "mp4":
                _mp4v_recording(mp4, 5, 640, 352, seed=40 + v)
                p = rec / f"camera{v}_synced.mp4"
                p.write_bytes(mp4.read_bytes())
            else:
                p = rec / f"camera{v}.npy"
                np.save(p, video.read_recording(mp4, 0, None))
            paths.append(str(p))
        log = cli.record_and_estimate_pose_main(["--camera_names", *names, "--configuration_number", "1",
                                                 "--recording_paths", *paths])
        runs[kind] = {k: np.load(log[k]) for k in ("kpts_2d", "heatmaps_2d", "kpts_3d")}
    assert runs["mp4"]["kpts_2d"].shape == (4, 17, 3, 2)              # 5 frames, the last dropped ([0, -1])
    for k in ("kpts_2d", "heatmaps_2d", "kpts_3d"):
        np.testing.assert_array_equal(runs["mp4"][k], runs["npy"][k], err_msg=k)
