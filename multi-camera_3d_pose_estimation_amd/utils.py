"""Drop-in for the reference utils.py functions on the hot path (triangulate_points,
calibration readers, frame loading) on the GPU.  See mvpose/utils.py."""
from mvpose.utils import (calculate_projection_matrix, get_params_from_name, load_frames,  # noqa: F401
                          read_camera_parameters, read_rotation_translation, to_numpy, triangulate_points)
