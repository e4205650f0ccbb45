"""CPU: the drop-in command lines keep the reference's flags and YAML helpers.

Flag lists are the reference's (record_and_estimate_pose.py:63-78,
pose_refinement.py:1100-1116); prepare_kwargs follows utils.py:1388-1399."""
import numpy as np
import pytest

from mvpose import cli

REC_FLAGS = ["camera_names", "estimator_model", "detector_model", "configuration_number", "recording_paths",
             "synchronize_video", "model_yaml", "calibration_settings_yaml", "checkerboard_display_parameter_yaml",
             "origin_camera_idx", "script_path", "project_dir", "recording_length_seconds", "keep_unsynced_files"]
REF_FLAGS = ["run_path", "refinement_types", "recording_log", "heatmaps_2d", "kpts_2d", "kpts_3d", "model",
             "save_path", "extrinsic_params_dir", "intrinsic_params_dir", "refinement_params_yaml",
             "body_part_lengths_yaml", "body_part_lengths_individual_name_yaml", "ignore_body_lengths",
             "interpolate_before_SGD"]


def _dests(parser):
    return [a.dest for a in parser._actions if a.dest != "help"]


def test_record_and_estimate_flags():
    assert _dests(cli.record_and_estimate_pose_parser()) == REC_FLAGS
    a = cli.record_and_estimate_pose_parser().parse_args(["--camera_names", "c0", "c1", "--configuration_number", "3",
                                                          "--recording_paths", "a.npy", "b.npy"])
    assert a.synchronize_video is False and a.configuration_number == 3 and a.recording_paths == ["a.npy", "b.npy"]


def test_refinement_flags_and_defaults():
    p = cli.pose_refinement_parser()
    assert _dests(p) == REF_FLAGS
    a = p.parse_args([])
    assert a.refinement_types == ["linear_interpolation"]
    assert a.body_part_lengths_individual_name_yaml == "my_lengths"


def test_prepare_kwargs_reference_semantics():
    def f(a=1, betas=(0.9, 0.999), max_iter=10, flag=False):
        return a
    kw = cli.prepare_kwargs(f, {"betas": [0.8, 0.99], "max_iter": ".inf"})
    assert kw == {"a": 1, "betas": (0.8, 0.99), "max_iter": np.inf, "flag": False}
    assert cli.prepare_kwargs(f, None) == {"a": 1, "betas": (0.9, 0.999), "max_iter": 10, "flag": False}


@pytest.mark.parametrize("kw", [dict(configuration_number=None, recording_paths=["x.npy"], synchronize_video=False),
                                dict(configuration_number=1, recording_paths=None, synchronize_video=False),
                                dict(configuration_number=1, recording_paths=["x.npy"], synchronize_video=True)])
def test_out_of_scope_steps_fail_loudly(kw):
    with pytest.raises(NotImplementedError):
        cli.record_and_estimate_pose(["c0", "c1"], **kw)
