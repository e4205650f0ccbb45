"""Drop-in for the reference's record_and_estimate_pose.py (same flags and outputs);
the 2D->3D hot path runs on the GPU through libmvpose.  See mvpose/cli.py."""
from mvpose.cli import record_and_estimate_pose, record_and_estimate_pose_main  # noqa: F401

if __name__ == "__main__":
    record_and_estimate_pose_main()
