"""The reference's two command lines, same flags / YAML / output files, GPU hot path.

* ``record_and_estimate_pose`` (record_and_estimate_pose.py:12-84): for a given
  configuration and recordings, 2D pose per frame + triangulation ->
  ``kpts_2d.npy`` (T,17,3,V) f32, ``heatmaps_2d.npy`` (T,V,17,6) f64,
  ``kpts_3d.npy`` (T,17,3) f32 and ``recording_log.yaml`` in the recordings
  folder.  Camera configuration (GUI), webcam recording and audio-clap
  synchronisation are outside the hot path: the flags are accepted, and asking
  for those steps raises NotImplementedError.
* ``pose_refinement`` (pose_refinement.py:1099-1255): missing arguments filled
  from recording_log.yaml; ``linear_interpolation`` always runs (GPU kernel) and
  is saved when requested; ``SGD`` runs the one-launch GPU refinement with the
  ``SGD`` section of --refinement_params_yaml and saves ``kpts_3d_SGD.npy``.
"""
from __future__ import annotations

import argparse
import inspect
import os
from pathlib import Path

import numpy as np
import torch
import yaml

from . import geometry


def load_config(config_path=None):
    """utils.load_config (utils.py:1376-1381)."""
    if config_path is None:
        return {}
    with open(config_path) as f:
        return yaml.safe_load(f) or {}


def prepare_kwargs(func, user_kwargs):
    """utils.prepare_kwargs (utils.py:1388-1399): function defaults updated by the YAML
    section; ".inf" -> np.inf, betas list -> tuple."""
    kw = {k: v.default for k, v in inspect.signature(func).parameters.items()
          if v.default is not inspect.Parameter.empty}
    kw.update(user_kwargs or {})
    for k, v in kw.items():
        if v == ".inf":
            kw[k] = np.inf
        if k == "betas" and isinstance(v, list):
            kw[k] = tuple(v)
    return kw


# --------------------------------------------------------------------- record + estimate
def record_and_estimate_pose(camera_names, estimator_model="coco_base", detector_model="coco_base",
                             configuration_number=None, recording_paths=None, synchronize_video=True,
                             model_yaml="./model_paths.yaml", calibration_settings_yaml="./calibration_settings.yaml",
                             checkerboard_display_parameter_yaml="./checkerboard_display_parameters.yaml",
                             origin_camera_idx=0, script_path=None, project_dir="", recording_length_seconds=10,
                             keep_unsynced_files=False):
    from .pose_estimation import estimate_pose_from_video
    if project_dir:
        os.chdir(project_dir)
    if configuration_number is None:
        raise NotImplementedError("camera configuration (setup_camera_configuration) is outside the GPU hot "
                                  "path: pass --configuration_number of an existing configuration")
    configuration_dir = f"./configurations/{configuration_number}/"
    if not recording_paths:
        raise NotImplementedError("webcam recording is outside the GPU hot path: pass --recording_paths")
    if synchronize_video:
        raise NotImplementedError("audio-based video synchronisation is outside the GPU hot path: pass "
                                  "already synchronised recordings (omit --synchronize_video)")
    recordings_folder = os.path.dirname(recording_paths[0])
    kpts_2d, heatmaps, kpts_3d = estimate_pose_from_video(
        camera_names, recording_paths, estimator_model, detector_model=detector_model, model_yaml=model_yaml,
        start_end_frames=[0, -1], confidence=0,
        extrinsic_params_dir=os.path.join(configuration_dir, "extrinsic_camera_parameters"))
    log = {"recording_paths": [str(p) for p in recording_paths],
           "kpts_2d": str(os.path.join(recordings_folder, "kpts_2d.npy")),
           "heatmaps_2d": str(os.path.join(recordings_folder, "heatmaps_2d.npy")),
           "kpts_3d": str(os.path.join(recordings_folder, "kpts_3d.npy")),
           "estimator_model": estimator_model, "detector_model": detector_model}
    with open(os.path.join(recordings_folder, "recording_log.yaml"), "w") as f:
        yaml.dump(log, f)
    if kpts_2d is not None:
        np.save(log["kpts_2d"], kpts_2d)
    if heatmaps is not None:
        np.save(log["heatmaps_2d"], heatmaps)
    if kpts_3d is not None:
        np.save(log["kpts_3d"], kpts_3d)
    return log


def record_and_estimate_pose_parser():
    """Flags of record_and_estimate_pose.py:63-78."""
    p = argparse.ArgumentParser()
    p.add_argument("--camera_names", nargs="+", required=True, help="List of camera names")
    p.add_argument("--estimator_model")
    p.add_argument("--detector_model")
    p.add_argument("--configuration_number", type=int)
    p.add_argument("--recording_paths", nargs="*")
    p.add_argument("--synchronize_video", action="store_true")
    p.add_argument("--model_yaml")
    p.add_argument("--calibration_settings_yaml")
    p.add_argument("--checkerboard_display_parameter_yaml")
    p.add_argument("--origin_camera_idx", type=int)
    p.add_argument("--script_path")
    p.add_argument("--project_dir")
    p.add_argument("--recording_length_seconds", type=int)
    p.add_argument("--keep_unsynced_files", action="store_true")
    return p


def record_and_estimate_pose_main(argv=None):
    args = record_and_estimate_pose_parser().parse_args(argv)
    return record_and_estimate_pose(**{k: v for k, v in vars(args).items() if v is not None})


# --------------------------------------------------------------------- refinement
def pose_refinement_parser():
    """Flags of pose_refinement.py:1100-1116."""
    p = argparse.ArgumentParser()
    p.add_argument("--run_path", type=str)
    p.add_argument("--refinement_types", nargs="+", default=["linear_interpolation"])
    p.add_argument("--recording_log", type=str)
    p.add_argument("--heatmaps_2d", type=str)
    p.add_argument("--kpts_2d", type=str)
    p.add_argument("--kpts_3d", type=str)
    p.add_argument("--model", type=str)
    p.add_argument("--save_path", type=str)
    p.add_argument("--extrinsic_params_dir", type=str)
    p.add_argument("--intrinsic_params_dir", type=str)
    p.add_argument("--refinement_params_yaml", type=str)
    p.add_argument("--body_part_lengths_yaml", type=str)
    p.add_argument("--body_part_lengths_individual_name_yaml", default="my_lengths", type=str)
    p.add_argument("--ignore_body_lengths", action="store_true")
    p.add_argument("--interpolate_before_SGD", action="store_true")
    return p


def _load_if_exists(path):
    return np.load(path) if path is not None and os.path.exists(str(path)) else None


def pose_refinement_main(argv=None):
    from .refine import Optimized_3d_Pose_Estimation, linear_interpolation
    args = pose_refinement_parser().parse_args(argv)
    if args.run_path is None:
        args.run_path = os.getcwd()
    if args.save_path is None:
        args.save_path = args.run_path
    if args.extrinsic_params_dir is None:
        args.extrinsic_params_dir = Path(args.run_path).parent.parent / "extrinsic_camera_parameters"
    if args.intrinsic_params_dir is None:
        args.intrinsic_params_dir = os.path.join(os.getcwd(), "intrinsic_camera_parameters")
    log_path = args.recording_log or os.path.join(args.run_path, "recording_log.yaml")
    log = {}
    if os.path.exists(log_path):
        with open(log_path) as f:
            log = yaml.safe_load(f) or {}
    for k, v in vars(args).items():      # fill missing args from the log (:1137-1144)
        if v is None and k in log:
            setattr(args, k, log[k])
    kpts_3d = _load_if_exists(args.kpts_3d)
    heatmaps = _load_if_exists(args.heatmaps_2d)
    params = load_config(args.refinement_params_yaml)
    types = set(args.refinement_types)
    interp = linear_interpolation(kpts_3d, **prepare_kwargs(linear_interpolation, params.get("linear_interpolation")))
    outputs = {}
    if "linear_interpolation" in types:
        path = os.path.join(args.save_path, "kpts_3d_linear_interpolation.npy")
        print(f"saving linear interpolation at {path}")
        np.save(path, interp)
        outputs["linear_interpolation"] = path
        types.discard("linear_interpolation")
    if "SGD" in types:
        cameras, _origin = geometry.load_camera_names(str(args.extrinsic_params_dir))
        cam_params = {}
        for i in cameras:
            _, cam_params[i] = geometry.get_params_from_name(cameras[i], intrinsic_params_dir=str(
                args.intrinsic_params_dir), extrinsic_params_dir=str(args.extrinsic_params_dir))
        my_lengths = None
        if not args.ignore_body_lengths:
            if args.body_part_lengths_yaml is None and os.path.exists("./body_part_lengths.yaml"):
                args.body_part_lengths_yaml = "./body_part_lengths.yaml"
            if args.body_part_lengths_yaml is not None:
                with open(args.body_part_lengths_yaml) as f:
                    my_lengths = yaml.safe_load(f)[args.body_part_lengths_individual_name_yaml]
        init = interp if args.interpolate_before_SGD else kpts_3d
        opt = Optimized_3d_Pose_Estimation(torch.tensor(heatmaps), init, decomposed_cam_params_initial=cam_params,
                                           body_lengths=my_lengths)
        kw = prepare_kwargs(opt.sgd_optimize, params.get("SGD"))
        kw.pop("own_camera_gaussians", None)
        opt.sgd_optimize(**kw)
        path = os.path.join(args.save_path, "kpts_3d_SGD.npy")
        print(f"saving SGD at {path}")
        best = opt.best_trajectory
        np.save(path, best.numpy() if best is not None else np.array(None))
        outputs["SGD"] = path
        types.discard("SGD")
    if types:
        raise ValueError(f"unknown refinement type(s) {sorted(types)}; expected linear_interpolation and/or SGD")
    return outputs
