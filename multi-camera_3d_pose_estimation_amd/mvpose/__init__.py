"""mvpose — MI355X-native (gfx950) multi-view 3D pose hot path.

Drop-in for the per-frame 2D-detect -> DLT-triangulate loop and the
reprojection SGD of sashapersonxyz/Multi-camera_3D_Pose_Estimation
(see DESIGN.md).  All compute runs in hand-written HIP kernels inside
libmvpose.so (C-ABI: include/mvpose.h); this package is the host side.
"""
__all__ = ["ops", "synthetic"]
