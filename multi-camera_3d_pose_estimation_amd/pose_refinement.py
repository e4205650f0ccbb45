"""Drop-in for the reference's pose_refinement.py command line (same flags, YAML and
outputs); linear_interpolation and the SGD refinement run on the GPU.  See mvpose/cli.py."""
from mvpose.cli import pose_refinement_main
from mvpose.refine import (Optimized_3d_Pose_Estimation, linear_interpolation,  # noqa: F401
                           project_points_torch)

if __name__ == "__main__":
    pose_refinement_main()
