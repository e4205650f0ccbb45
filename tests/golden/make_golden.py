"""Generate the golden vectors under tests/golden/ by importing the REFERENCE
itself (sashapersonxyz/Multi-camera_3D_Pose_Estimation at /root/reference).

Runs ONLY in the build container (the reference never travels to the GPU box):
    python tests/golden/make_golden.py [generator ...]   (default: all)
The reference needs cv2 and mmpose, which are absent here; they are replaced by
stub modules.  The stub cv2 is populated with the oracle's OpenCV-4.9
restatement (oracle/cv_ref.py), so fixtures that go through cv2
(pose3d_select) pin the reference's selection / ordering / reshape / dtype
orchestration, not cv2's numerics.  Every other fixture calls reference
functions that are pure numpy / torch and is pinned to the reference's own
arithmetic.  Each fixture records its generator seeds.

Only data (inputs and expected outputs) is written; no reference source.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))

from mvpose import synthetic as syn  # noqa: E402
from oracle import cv_ref  # noqa: E402
from oracle import heatmap_ref  # noqa: E402
sys.path.insert(0, os.path.dirname(HERE))
from sgd_problem import BENCH_C5_KW, bench_c5_inputs, inputs_digest, sgd_inputs  # noqa: E402

REF = "/root/reference"


def _install_stubs():
    cv2 = types.ModuleType("cv2")
    cv2.undistortPoints = cv_ref.undistort_points
    cv2.triangulatePoints = cv_ref.triangulate_points_cv
    cv2.convertPointsFromHomogeneous = cv_ref.convert_points_from_homogeneous
    sys.modules["cv2"] = cv2
    for name in ("mmpose", "mmpose.apis", "mmpose.structures", "mmpose.utils"):
        sys.modules[name] = types.ModuleType(name)
    sys.modules["mmpose.apis"].inference_topdown = None
    sys.modules["mmpose.apis"].init_model = None
    sys.modules["mmpose.structures"].merge_data_samples = None
    sys.modules["mmpose.utils"].adapt_mmdet_pipeline = None
    sys.path.insert(0, REF)


def _save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path)} B)")


def gen_dlt(ref_utils):
    """utils.DLT known answers (utils.py:19-34), zero distortion."""
    rig_seed, pose_seed, kp_seed = 11, 12, 13
    cams = syn.make_rig(2, seed=rig_seed, distortion=False)
    poses = syn.make_poses(6, seed=pose_seed)
    k = syn.make_kpts_2d(poses, cams, seed=kp_seed)
    P0 = cv_ref.projection_matrix(cams[0]["K"], cams[0]["R"], cams[0]["T"])
    P1 = cv_ref.projection_matrix(cams[1]["K"], cams[1]["R"], cams[1]["T"])
    pts = k[:, :, :2, :].reshape(-1, 2, 2).astype(np.float64)  # (n, xy, view)
    out = np.array([ref_utils.DLT(P0, P1, p[:, 0], p[:, 1]) for p in pts])
    _save("dlt_kat.npz", P0=P0, P1=P1, kpts=k, out=out,
          K=np.stack([c["K"] for c in cams]), R=np.stack([c["R"] for c in cams]),
          T=np.stack([c["T"] for c in cams]), dist=np.stack([c["dist"] for c in cams]),
          seeds=np.array([rig_seed, pose_seed, kp_seed]))


def gen_pose3d(pose_estimation):
    """pose_estimation.get_pose_3D selection / ordering (pose_estimation.py:11-65)."""
    rig_seed, pose_seed, kp_seed = 21, 22, 23
    cams = syn.make_rig(3, seed=rig_seed)
    poses = syn.make_poses(8, seed=pose_seed)
    k = syn.make_kpts_2d(poses, cams, seed=kp_seed)
    # planted exact confidence ties and NaN confidences
    k[0, :5, 2, 1] = k[0, :5, 2, 0]
    k[1, 3, 2, :] = 0.5
    k[2, 4, 2, 0] = np.nan
    k[2, 5, 2, 1] = np.nan
    k[2, 6, 2, :] = np.nan
    k[3, 7, 2, 2] = np.nan
    cp = syn.reference_camera_params(cams)
    outs = {}
    for tag, ci, ign in (("01", [0, 1], False), ("012", [0, 1, 2], False), ("12", [1, 2], False),
                         ("01_nodist", [0, 1], True)):
        outs["out_" + tag] = pose_estimation.get_pose_3D(dict(cp), k, camera_indices=ci,
                                                        ignore_nonlinear_distortions=ign)
    _save("pose3d_select.npz", kpts=k, K=np.stack([c["K"] for c in cams]),
          R=np.stack([c["R"] for c in cams]), T=np.stack([c["T"] for c in cams]),
          dist=np.stack([c["dist"] for c in cams]), seeds=np.array([rig_seed, pose_seed, kp_seed]),
          **outs)


def _synthetic_heatmaps(rng, K, H, W, scale=1.0):
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    hm = np.empty((K, H, W), np.float32)
    for j in range(K):
        cx, cy = rng.uniform(0.1 * W, 0.9 * W), rng.uniform(0.1 * H, 0.9 * H)
        sx, sy = rng.uniform(1.5, 4.0) * scale, rng.uniform(1.5, 4.0) * scale
        rho = rng.uniform(-0.5, 0.5)
        dx, dy = (xx - cx) / sx, (yy - cy) / sy
        g = np.exp(-0.5 * (dx * dx - 2 * rho * dx * dy + dy * dy) / (1 - rho * rho))
        hm[j] = (rng.uniform(0.3, 1.0) * g + rng.normal(0, 0.01, (H, W))).astype(np.float32)
    hm[K - 1] = rng.uniform(-0.05, 0.0099, (H, W)).astype(np.float32)  # all below threshold -> zeros
    return hm


def gen_moments(PoseEstimator):
    """PoseEstimator.get_heatmap_means_cov (mmpose_pose_estimation.py:163-215) on
    (a) a full-resolution heatmap directly, (b) a 64x48 heatmap reverted to a
    small image with the oracle's cv2.warpAffine restatement (revert_heatmap)."""
    seed = 31
    rng = np.random.default_rng(seed)
    hm_full = _synthetic_heatmaps(rng, 17, 72, 128, scale=3.0)
    out_full = PoseEstimator.get_heatmap_means_cov(None, hm_full.copy())
    hm_low = _synthetic_heatmaps(rng, 17, 64, 48)
    img_h, img_w = 90, 160
    center, scale = heatmap_ref.whole_image_cs(img_w, img_h)
    scale = heatmap_ref.fix_aspect_ratio(scale, 192 / 256)
    M_inv = heatmap_ref.get_warp_matrix(center, scale, 0.0, (48, 64), inv=True)
    reverted = heatmap_ref.warp_affine_linear_f32(hm_low, M_inv, img_h, img_w)
    out_rev = PoseEstimator.get_heatmap_means_cov(None, reverted.copy())
    _save("moments.npz", hm_full=hm_full, out_full=out_full, hm_low=hm_low, M_inv=M_inv,
          img_hw=np.array([img_h, img_w]), out_rev=out_rev, seeds=np.array([seed]))


def gen_project(pr):
    """project_points_torch (pose_refinement.py:94-179)."""
    seed = 41
    cams = syn.make_rig(3, seed=seed)
    poses = syn.make_poses(5, seed=seed + 1)
    pts = torch.tensor(poses, dtype=torch.float32)
    outs = {}
    for v, c in enumerate(cams):
        for ign in (False, True):
            outs[f"out_c{v}_{int(ign)}"] = pr.project_points_torch(pts, c["K"], c["R"], c["T"], c["dist"],
                                                                   ignore_distortions=ign).numpy()
    rvec = np.array([0.1, -0.2, 0.05])
    outs["out_axisangle"] = pr.project_points_torch(pts, cams[1]["K"], torch.tensor(rvec, dtype=torch.float32),
                                                    cams[1]["T"], cams[1]["dist"]).numpy()
    _save("project.npz", points=poses.astype(np.float32), K=np.stack([c["K"] for c in cams]),
          R=np.stack([c["R"] for c in cams]), T=np.stack([c["T"] for c in cams]),
          dist=np.stack([c["dist"] for c in cams]), rvec=rvec, seeds=np.array([seed]), **outs)


def gen_bodylen(ref_utils):
    seed = 51
    poses = torch.tensor(syn.make_poses(7, seed=seed), dtype=torch.float32)
    L = ref_utils.get_body_part_lengths(poses)
    names = list(L.keys())
    _save("bodylen.npz", poses=poses.numpy(), names=np.array(names),
          lengths=np.stack([L[n].numpy() for n in names]), seeds=np.array([seed]))


MY_LENGTHS = {  # reference examples/body_part_lengths.yaml:my_lengths (key order kept)
    "left_shoulder_left_elbow": 38, "left_elbow_left_wrist": 27,
    "right_shoulder_right_elbow": 38, "right_elbow_right_wrist": 27,
    "left_hip_left_knee": 51, "left_knee_left_ankle": 40,
    "right_hip_right_knee": 51, "right_knee_right_ankle": 40,
    "left_hip_right_hip": 31, "left_shoulder_left_hip": 54,
    "right_shoulder_right_hip": 54, "left_shoulder_right_shoulder": 47,
}


def gen_sgd(pr):
    """Optimized_3d_Pose_Estimation.sgd_optimize (pose_refinement.py:894-1096),
    trajectory-only path, as the CLI drives it (pose_refinement.py:1210-1214)."""
    cases = [
        # name, V, T, seed, kwargs
        ("sgd_V2_T40", 2, 40, 61, dict(lr=0.01, lambda_smooth=1e-6, lambda_body_length=1.0, patience=100,
                                       max_iter=10, batch_size=None)),
        ("sgd_V2_T40_b8", 2, 40, 62, dict(lr=0.01, lambda_smooth=1e-3, lambda_body_length=0.5, patience=100,
                                          max_iter=5, batch_size=8)),
        ("sgd_V8_T20", 8, 20, 63, dict(lr=0.01, lambda_smooth=1e-6, lambda_body_length=1.0, patience=100,
                                       max_iter=60, batch_size=None)),
        ("sgd_V2_T24_stop", 2, 24, 64, dict(lr=0.05, lambda_smooth=1e-6, lambda_body_length=1.0, patience=3,
                                            max_iter=400, batch_size=None, tolerance=0.2)),
    ]
    for name, V, T, seed, kw in cases:
        cams, gauss, init = sgd_inputs(V, T, seed)
        params = {i: [c["K"].copy(), c["R"].copy(), c["T"].copy(), c["dist"].copy()] for i, c in enumerate(cams)}
        torch.manual_seed(0)
        opt = pr.Optimized_3d_Pose_Estimation(torch.tensor(gauss), init, decomposed_cam_params_initial=params,
                                              body_lengths=dict(MY_LENGTHS))
        full_kw = dict(print_frequency=10 ** 9)
        full_kw.update(kw)
        opt.sgd_optimize(**full_kw)
        hist = {k: np.array([float(x) for x in v], np.float64) for k, v in opt.all_costs_total.items()}
        _save(f"{name}.npz", gauss=gauss, init=init, K=np.stack([c["K"] for c in cams]),
              R=np.stack([c["R"] for c in cams]), T=np.stack([c["T"] for c in cams]),
              dist=np.stack([c["dist"] for c in cams]), best=opt.best_trajectory.numpy(),
              final=opt.trajectory.detach().numpy(),
              kw_names=np.array(list(kw.keys())), kw_vals=np.array([np.nan if v is None else float(v)
                                                                  for v in kw.values()]),
              seeds=np.array([seed]), **{"hist_" + k: v for k, v in hist.items()})


C5_CASES = [
    # BASELINE config 5 (V=8, T=400): T*J = 399*17 > 1024 runs sgd_kernel<1024, false> (csrc/sgd.hip).
    # name, seed, kwargs
    ("sgd_V8_T400", 65, dict(lr=0.01, lambda_smooth=1e-6, lambda_body_length=1.0, patience=100, max_iter=8,
                             batch_size=None)),
    ("sgd_V8_T400_b100", 66, dict(lr=0.01, lambda_smooth=1e-3, lambda_body_length=0.5, patience=100,
                                  max_iter=8, batch_size=100)),
    ("sgd_V8_T400_stop", 67, dict(lr=0.05, lambda_smooth=1e-6, lambda_body_length=1.0, patience=3,
                                  max_iter=400, batch_size=None, tolerance=1.0)),
]


def gen_sgd_c5(pr):
    """sgd_optimize at BASELINE config 5's size (pose_refinement.py:894-1096): one window,
    overlapping windows of 100 frames, and an early stop.  The 2.6 MB inputs are rebuilt by
    the tests from the seed (tests/sgd_problem.py) and checked against the stored digest."""
    for name, seed, kw in C5_CASES:
        cams, gauss, init = sgd_inputs(8, 400, seed)
        params = {i: [c["K"].copy(), c["R"].copy(), c["T"].copy(), c["dist"].copy()] for i, c in enumerate(cams)}
        torch.manual_seed(0)
        opt = pr.Optimized_3d_Pose_Estimation(torch.tensor(gauss), init, decomposed_cam_params_initial=params,
                                              body_lengths=dict(MY_LENGTHS))
        full_kw = dict(print_frequency=10 ** 9)
        full_kw.update(kw)
        opt.sgd_optimize(**full_kw)
        hist = {k: np.array([float(x) for x in v], np.float64) for k, v in opt.all_costs_total.items()}
        print(name, "history length", len(hist["total_cost"]))
        _save(f"{name}.npz", V=np.array([8]), T=np.array([400]), digest=np.array(inputs_digest(cams, gauss, init)),
              best=opt.best_trajectory.numpy(), final=opt.trajectory.detach().numpy(),
              kw_names=np.array(list(kw.keys())), kw_vals=np.array([np.nan if v is None else float(v)
                                                                  for v in kw.values()]),
              seeds=np.array([seed]), **{"hist_" + k: v for k, v in hist.items()})


def gen_bench_sgd(pr):
    """The bench's config-5 SGD line (bench.py::sgd_line, 40 Adam iterations on all 400 rows:
    time_interval [0, None]) run by the reference; the bench asserts its final trajectory
    against this."""
    cams, gauss, init = bench_c5_inputs()
    params = {i: [c["K"].copy(), c["R"].copy(), c["T"].copy(), c["dist"].copy()] for i, c in enumerate(cams)}
    torch.manual_seed(0)
    opt = pr.Optimized_3d_Pose_Estimation(torch.tensor(gauss), init, decomposed_cam_params_initial=params,
                                          body_lengths=dict(MY_LENGTHS))
    opt.sgd_optimize(print_frequency=10 ** 9, time_interval=[0, None], batch_size=None, **BENCH_C5_KW)
    _save("bench_sgd_c5.npz", digest=np.array(inputs_digest(cams, gauss, init)),
          final=opt.trajectory.detach().numpy(), n_hist=np.array([len(opt.all_costs_total["total_cost"])]))


def _rotation(rvec):
    th = np.linalg.norm(rvec)
    k = np.asarray(rvec) / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx


EXTRINSIC_CASES = [
    # name, seed, learnable ID, GT IDs, (rvec perturbation, T offset), kwargs
    ("sgd_ext_c2", 81, 2, [0, 1], ([0.02, -0.03, 0.01], [6.0, -4.0, 3.0]),
     dict(lr=0.01, lambda_smooth=1e-6, lambda_body_length=1.0, patience=100, max_iter=12, batch_size=4,
          N_sample_points=20)),
    # camera 0 is R = I, T = 0: every zero entry becomes random.random()/1e6 (:939-940)
    ("sgd_ext_c0", 82, 0, [1, 2], None,
     dict(lr=0.02, lambda_smooth=1e-3, lambda_body_length=0.0, patience=3, max_iter=40, batch_size=None,
          N_sample_points=12, tolerance=1e-3)),
]


def gen_sgd_extrinsic(pr):
    """sgd_optimize(extrinsic_optimization_IDs=[id], optimize_trajectory=False,
    GT_camera_IDs=[a, b]) (pose_refinement.py:684-706, :800-831, :894-1096).  The float64
    samples go through the stub cv2 in float64, as real cv2 keeps CV_64F (the oracle's
    float64 undistortPoints / triangulatePoints / convertPointsFromHomogeneous)."""
    import random
    for name, seed, ext_id, gt, pert, kw in EXTRINSIC_CASES:
        kw = dict(kw)
        T = 9        # time_interval [0, -1] keeps 8 rows: batch_size 4 -> windows [0,4) [2,6) [4,8)
        cams, gauss, init = sgd_inputs(3, T, seed)
        params = {i: [c["K"].copy(), c["R"].copy(), c["T"].copy(), c["dist"].copy()] for i, c in enumerate(cams)}
        if pert is not None:
            params[ext_id][1] = _rotation(pert[0]) @ params[ext_id][1]
            params[ext_id][2] = params[ext_id][2] + np.array(pert[1]).reshape(3, 1)
        R0 = np.stack([p[1] for p in params.values()])
        T0 = np.stack([p[2] for p in params.values()])
        np.random.seed(seed)
        random.seed(seed + 1)
        torch.manual_seed(0)
        n_samples = kw.pop("N_sample_points")   # sgd_optimize's own N_sample_points is unused (:684)
        opt = pr.Optimized_3d_Pose_Estimation(torch.tensor(gauss), init, decomposed_cam_params_initial=params,
                                              body_lengths=dict(MY_LENGTHS), N_sample_points=n_samples)
        full_kw = dict(print_frequency=10 ** 9, extrinsic_optimization_IDs=[ext_id], optimize_trajectory=False,
                       GT_camera_IDs=gt)
        full_kw.update(kw)
        opt.sgd_optimize(**full_kw)
        hist = {k: np.array([float(x) for x in v], np.float64) for k, v in opt.all_costs_total.items()}
        best = opt.best_decomposed_cam_params[ext_id]
        fin = opt.decomposed_cam_params[ext_id]
        _save(f"{name}.npz", gauss=gauss, init=init, K=np.stack([c["K"] for c in cams]), R=R0, T=T0,
              dist=np.stack([c["dist"] for c in cams]), ext_id=np.array([ext_id]), gt_ids=np.array(gt),
              n_samples=np.array([n_samples]),
              samples=opt.samples, samples_3d=opt.samples_3d.numpy(),
              best_R=best[1].detach().numpy(), best_T=best[2].detach().numpy(),
              final_R=fin[1].detach().numpy(), final_T=fin[2].detach().numpy(),
              kw_names=np.array(list(kw.keys())),
              kw_vals=np.array([np.nan if v is None else float(v) for v in kw.values()]),
              seeds=np.array([seed, seed + 1, 0]), **{"hist_" + k: v for k, v in hist.items()})


JOINT_CASES = [
    # name, seed, learnable IDs, (rvec perturbation, T offset) per learnable ID, kwargs
    ("sgd_joint_c2", 91, [2], [([0.015, -0.02, 0.01], [4.0, -3.0, 2.0])],
     dict(lr=0.01, lambda_smooth=1e-6, lambda_body_length=1.0, patience=100, max_iter=10, batch_size=None)),
    # camera 0 is R = I, T = 0: zero entries become random.random()/1e6 (:939-940); two learnable
    # cameras, overlapping windows, early stop
    ("sgd_joint_c01", 92, [0, 1], [None, ([-0.01, 0.02, 0.0], [-3.0, 2.0, 5.0])],
     dict(lr=0.02, lambda_smooth=1e-3, lambda_body_length=0.5, patience=3, max_iter=30, batch_size=8,
          tolerance=1e-2)),
]


def gen_sgd_joint(pr):
    """sgd_optimize(extrinsic_optimization_IDs=ids, optimize_trajectory=True)
    (pose_refinement.py:894-1096 with :931-954): trajectory + the listed cameras' R (3x3) and T
    in one Adam / clip_grad_norm_."""
    import random
    for name, seed, ids, perts, kw in JOINT_CASES:
        T = 16
        cams, gauss, init = sgd_inputs(3, T, seed)
        params = {i: [c["K"].copy(), c["R"].copy(), c["T"].copy(), c["dist"].copy()] for i, c in enumerate(cams)}
        for ID, pert in zip(ids, perts):
            if pert is not None:
                params[ID][1] = _rotation(pert[0]) @ params[ID][1]
                params[ID][2] = params[ID][2] + np.array(pert[1]).reshape(3, 1)
            else:
                params[ID][1] = np.eye(3)
                params[ID][2] = np.zeros((3, 1))
        R0 = np.stack([p[1] for p in params.values()])
        T0 = np.stack([p[2] for p in params.values()])
        random.seed(seed + 1)
        torch.manual_seed(0)
        opt = pr.Optimized_3d_Pose_Estimation(torch.tensor(gauss), init, decomposed_cam_params_initial=params,
                                              body_lengths=dict(MY_LENGTHS))
        full_kw = dict(print_frequency=10 ** 9, extrinsic_optimization_IDs=list(ids), optimize_trajectory=True)
        full_kw.update(kw)
        opt.sgd_optimize(**full_kw)
        hist = {k: np.array([float(x) for x in v], np.float64) for k, v in opt.all_costs_total.items()}
        best = opt.best_decomposed_cam_params
        fin = opt.decomposed_cam_params
        _save(f"{name}.npz", gauss=gauss, init=init, K=np.stack([c["K"] for c in cams]), R=R0, T=T0,
              dist=np.stack([c["dist"] for c in cams]), ext_ids=np.array(ids),
              best=opt.best_trajectory.numpy(), final=opt.trajectory.detach().numpy(),
              best_R=np.stack([best[i][1].detach().numpy() for i in ids]),
              best_T=np.stack([best[i][2].detach().numpy() for i in ids]),
              final_R=np.stack([fin[i][1].detach().numpy() for i in ids]),
              final_T=np.stack([fin[i][2].detach().numpy() for i in ids]),
              kw_names=np.array(list(kw.keys())),
              kw_vals=np.array([np.nan if v is None else float(v) for v in kw.values()]),
              seeds=np.array([seed, seed + 1, 0]), **{"hist_" + k: v for k, v in hist.items()})


def gen_interp(pr):
    """pose_refinement.linear_interpolation (pose_refinement.py:15-84) on a noisy
    kpts_3d-like sequence with spikes, a NaN frame and constant stretches."""
    seed = 71
    rng = np.random.default_rng(seed)
    pts = syn.make_poses(40, seed=seed).astype(np.float32)
    pts += rng.normal(0, 0.5, pts.shape).astype(np.float32)
    spikes = rng.integers(0, 40, 25)
    pts[spikes, rng.integers(0, 17, 25), rng.integers(0, 3, 25)] += rng.choice([-40, 40], 25).astype(np.float32)
    pts[17, 3, :] = np.nan
    pts[5:12, 8, 1] = 7.25
    cases = {"default": {}, "rolling": dict(use_rolling_average=True), "nomedian": dict(filter_distance_from_median=False),
             "k7": dict(k=7, k_std=1.5, median_std=3)}
    outs = {f"out_{n}": pr.linear_interpolation(pts.copy(), **kw) for n, kw in cases.items()}
    _save("interp.npz", points=pts, seeds=np.array([seed]), **outs)


GENERATORS = ("dlt", "pose3d", "moments", "project", "bodylen", "sgd", "sgd_c5", "bench_sgd", "sgd_extrinsic", "sgd_joint",
              "interp")


def main():
    only = set(sys.argv[1:]) or set(GENERATORS)
    _install_stubs()
    import utils as ref_utils  # noqa: E402  (reference utils.py)
    import pose_estimation  # noqa: E402
    import pose_refinement as pr  # noqa: E402
    from mmpose_pose_estimation import PoseEstimator  # noqa: E402
    gens = {"dlt": lambda: gen_dlt(ref_utils), "pose3d": lambda: gen_pose3d(pose_estimation),
            "moments": lambda: gen_moments(PoseEstimator), "project": lambda: gen_project(pr),
            "bodylen": lambda: gen_bodylen(ref_utils), "sgd": lambda: gen_sgd(pr), "sgd_c5": lambda: gen_sgd_c5(pr),
            "bench_sgd": lambda: gen_bench_sgd(pr),
            "sgd_extrinsic": lambda: gen_sgd_extrinsic(pr), "sgd_joint": lambda: gen_sgd_joint(pr),
            "interp": lambda: gen_interp(pr)}
    for name in GENERATORS:
        if name in only:
            gens[name]()


if __name__ == "__main__":
    main()
