"""GPU mirror of the reference's pose_estimation.py module surface.

* ``get_pose_3D(camera_params, all_kpts_2d, world_trans_rot=None, camera_indices=None,
  ignore_nonlinear_distortions=False)`` (pose_estimation.py:11-65): one batched
  ``mvp_triangulate`` launch instead of T·J ``utils.triangulate_points`` calls;
  same selection quirks, float32 output, optional inv(R_W0) rotation.
* ``load_frames(recording_paths, start_end_frames)`` (utils.py:849-909): decoded
  frame stacks, one per camera, sliced ``[start:end]`` (the default ``[0, -1]``
  drops the last frame, quirk F4).  Video decoding itself is outside this
  package's scope; a recording is a ``.npy`` (T, H, W, 3) uint8
  array of frames as a video decoder (BGR) returns them.
* ``run_pose_est`` (:157-244) and ``estimate_pose_from_video`` (:259-327): every
  frame of every camera through the batched GPU pipeline (crop, HRNet-W32 with
  flip test, decode, heatmap moments), then get_pose_3D over ``camera_indices=[0, 1]``
  as the reference hard-codes (:319).
"""
from __future__ import annotations

import os

import numpy as np
import torch
import yaml

from . import geometry, ops
from .estimator import BatchPoseEstimator
from .hrnet import N_JOINTS


def get_pose_3D(camera_params, all_kpts_2d, world_trans_rot=None, camera_indices=None,
                ignore_nonlinear_distortions=False, device=None):
    """camera_params {key: [K, R, T, dist]} (get_params_from_name order), all_kpts_2d
    (T, J, 3, V) -> (T, J, 3) float32 numpy (float64 if world_trans_rot is given)."""
    dev = torch.device(device if device is not None else "cuda")
    keys = list(camera_params.keys())
    params = {}
    for k in keys:
        K, R, T, dist = camera_params[k]
        params[k] = [K, R, T, np.asarray(dist) * 0 if ignore_nonlinear_distortions else dist]
    if camera_indices is None:
        camera_indices = keys
    positions = [keys.index(c) for c in camera_indices]
    kp = torch.as_tensor(np.ascontiguousarray(np.asarray(all_kpts_2d, dtype=np.float32)), device=dev)
    cams = torch.tensor(ops.pack_cameras(params), device=dev)
    out = ops.triangulate(kp, cams, positions, mode=ops.TRI_REFERENCE).cpu().numpy()
    if world_trans_rot is not None:
        R_W0, _ = world_trans_rot
        out = np.einsum("ij,tpj->tpi", np.linalg.inv(R_W0), out)
    return out


def load_frames(recording_paths, start_end_frames=(0, -1)):
    """{camera: (T', H, W, 3) uint8} memory-mapped, sliced [start:end]."""
    if isinstance(recording_paths, (list, tuple)):
        recording_paths = dict(enumerate(recording_paths))
    if not isinstance(recording_paths, dict):
        return None
    a, b = (0, -1) if start_end_frames is None else start_end_frames
    out = {}
    for k, path in recording_paths.items():
        if not str(path).endswith(".npy"):
            raise NotImplementedError(
                f"{path}: video decoding is not part of the GPU hot path; pass decoded frames as a "
                ".npy (T, H, W, 3) uint8 array (cv2 BGR order)")
        arr = np.load(path, mmap_mode="r")
        if arr.dtype != np.uint8 or arr.ndim != 4 or arr.shape[-1] != 3:
            raise ValueError(f"{path}: expected (T, H, W, 3) uint8 frames, got {arr.shape} {arr.dtype}")
        out[k] = arr[a:b]
    return out


def build_estimator(model, detector_model="coco_base", model_yaml="", frame_hw=(720, 1280), max_frames=256,
                    device=None):
    """A BatchPoseEstimator for the reference's model argument: an estimator instance, or a
    model name looked up in model_yaml (pose_estimators: {name: [config, checkpoint]}) whose
    checkpoint is a LOCAL mmpose HRNet-W32 .pth (loaded with weights_only=True).
    MVPOSE_RANDOM_WEIGHTS=1 selects seeded random weights (synthetic runs/tests)."""
    if isinstance(model, BatchPoseEstimator):
        return model
    dev = torch.device(device if device is not None else "cuda")
    sd = None
    if os.environ.get("MVPOSE_RANDOM_WEIGHTS") != "1":
        if not model_yaml or not os.path.exists(model_yaml):
            raise FileNotFoundError(f"model_yaml {model_yaml!r} not found (set MVPOSE_RANDOM_WEIGHTS=1 for "
                                    "random weights)")
        with open(model_yaml) as f:
            paths = yaml.safe_load(f)
        _, ckpt = paths["pose_estimators"][model]
        if not os.path.exists(ckpt):
            raise FileNotFoundError(f"pose checkpoint {ckpt!r} is not a local file (no network here)")
        blob = torch.load(ckpt, map_location="cpu", weights_only=True)
        sd = blob.get("state_dict", blob)
    return BatchPoseEstimator(sd, max_frames=max_frames, frame_hw=tuple(frame_hw), swap_rb=False, device=dev)


def run_pose_est(model, confidence=0.5, camera_indices=None, recording_paths=None, start_end_frames=(0, -1),
                 frame_shape=(1080, 1920), batch_frames=128):
    """-> kpts_2d (T, 17, 3, V) float32, heatmaps (T, V, 17, 6) float64 (numpy)."""
    frames = load_frames(recording_paths, start_end_frames)
    cams = list(frames.keys()) if camera_indices is None else list(camera_indices)
    stacks = [frames[c] for c in cams]
    T = min(len(s) for s in stacks)
    V = len(stacks)
    H, W = stacks[0].shape[1:3]
    est = model if isinstance(model, BatchPoseEstimator) else build_estimator(model, frame_hw=(H, W))
    dev = est.device
    step = max(1, min(batch_frames, est.max_frames // V))
    kpts_2d = np.zeros((T, N_JOINTS, 3, V), np.float32)
    heat = np.zeros((T, V, N_JOINTS, 6), np.float64)
    for t0 in range(0, T, step):
        t1 = min(T, t0 + step)
        host = np.stack([np.stack([s[t] for s in stacks]) for t in range(t0, t1)])   # (t, v, H, W, 3)
        fr = torch.from_numpy(host).to(dev).reshape((t1 - t0) * V, H, W, 3).contiguous()
        kt = torch.empty((t1 - t0, N_JOINTS, 3, V), dtype=torch.float32, device=dev)
        r = est.run(fr, n_views=V, kpts_tkv=kt)
        kpts_2d[t0:t1] = kt.cpu().numpy()
        heat[t0:t1] = r["gaussians"].reshape(t1 - t0, V, N_JOINTS, 6).cpu().numpy()
    return kpts_2d, heat


def estimate_pose_from_video(camera_names, recording_paths, model, detector_model="coco_base", model_yaml="",
                             start_end_frames=(0, -1), confidence=0, extrinsic_params_dir="",
                             recompute_kpts_2d=True):
    """pose_estimation.py:259-327.  recompute_kpts_2d replaces the reference's interactive
    y/n prompt when kpts_2d.npy already exists (:287-289)."""
    index_name, _origin = geometry.load_camera_names(extrinsic_params_dir)
    name_index = {v: k for k, v in index_name.items()}
    camera_indices = [name_index[n] for n in camera_names]
    camera_params = {}
    for i, name in enumerate(camera_names):
        _, camera_params[i] = geometry.get_params_from_name(name, extrinsic_params_dir=extrinsic_params_dir)
    folder = os.path.dirname(recording_paths[0])
    existing = os.path.join(folder, "kpts_2d.npy")
    heatmaps = None
    if os.path.exists(existing) and not recompute_kpts_2d:
        kpts_2d = np.load(existing)
    else:
        if isinstance(model, str):
            first = np.load(recording_paths[0], mmap_mode="r")
            model = build_estimator(model, detector_model, model_yaml, frame_hw=first.shape[1:3])
        paths = {i: recording_paths[i] for i in camera_indices}   # as :281 indexes them
        kpts_2d, heatmaps = run_pose_est(model, confidence=confidence, camera_indices=camera_indices,
                                         recording_paths=paths, start_end_frames=start_end_frames)
    kpts_3d = get_pose_3D(camera_params, kpts_2d, camera_indices=[0, 1])
    return kpts_2d, heatmaps, kpts_3d
