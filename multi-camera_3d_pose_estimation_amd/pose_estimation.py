"""Drop-in for the reference's pose_estimation.py module surface (get_pose_3D, get_pose_2D,
run_pose_est, estimate_pose_from_video) on the GPU.  See mvpose/pose_estimation.py."""
from mvpose.pose_estimation import (estimate_pose_from_video, get_pose_2D, get_pose_3D, load_frames,  # noqa: F401
                                    run_pose_est)
