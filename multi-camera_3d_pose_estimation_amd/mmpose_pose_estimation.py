"""Drop-in for the reference's mmpose_pose_estimation.py (PoseEstimator with the same
constructor and per-frame predict contract) on the GPU.  See mvpose/mmpose_pose_estimation.py."""
from mvpose.mmpose_pose_estimation import PoseEstimator, select_person_bbox  # noqa: F401
