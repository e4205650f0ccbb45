"""CPU: pin the triangulation oracle (oracle/cv_ref.py) to the reference.

* dlt_kat.npz     — reference utils.DLT (utils.py:19-34) known answers; at zero
                    distortion the OpenCV-semantics path must agree to 1e-4.
* pose3d_select.npz — reference pose_estimation.get_pose_3D
                    (pose_estimation.py:11-65) run with the oracle's cv2 leaves:
                    pins selection / ordering / reshape / dtype bit-exactly.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import cv_ref
from mvpose import synthetic as syn


def _cams(d):
    return {i: [d["K"][i], d["R"][i], d["T"][i], d["dist"][i]] for i in range(d["K"].shape[0])}


def test_dlt_known_answers():
    d = np.load(os.path.join(GOLDEN, "dlt_kat.npz"))
    out = cv_ref.get_pose_3D(_cams(d), d["kpts"], camera_indices=[0, 1]).reshape(-1, 3)
    # float32 output of values ~350 cm: 1e-4 = ~3 ulp
    np.testing.assert_allclose(out, d["out"], rtol=0, atol=1e-4)


@pytest.mark.parametrize("tag,ci,ign", [("01", [0, 1], False), ("012", [0, 1, 2], False),
                                        ("12", [1, 2], False), ("01_nodist", [0, 1], True)])
def test_get_pose_3D_matches_reference(tag, ci, ign):
    d = np.load(os.path.join(GOLDEN, "pose3d_select.npz"))
    out = cv_ref.get_pose_3D(_cams(d), d["kpts"], camera_indices=ci, ignore_nonlinear_distortions=ign)
    ref = d["out_" + tag]
    assert out.dtype == ref.dtype == np.float32
    np.testing.assert_array_equal(out, ref)


def test_undistort_converges_on_reference_forward_model():
    cams = syn.make_rig(2, seed=5)
    poses = syn.make_poses(10, seed=6)
    k = syn.make_kpts_2d(poses, cams, seed=7, noise_px=0.0)
    out = cv_ref.get_pose_3D(syn.reference_camera_params(cams), k, camera_indices=[0, 1])
    np.testing.assert_allclose(out, poses, atol=1e-3)


def test_jacobi_svd_matches_numpy():
    rng = np.random.default_rng(0)
    for m in (4, 8, 16):
        A = rng.normal(size=(m, 4))
        w, Vt = cv_ref.jacobi_svd(A)
        w_np = np.linalg.svd(A, compute_uv=False)
        np.testing.assert_allclose(w, w_np, rtol=1e-12)
        # rows of Vt are right singular vectors (up to sign)
        _, _, Vt_np = np.linalg.svd(A)
        np.testing.assert_allclose(np.abs(np.sum(Vt * Vt_np, axis=1)), 1.0, rtol=1e-10)


def test_all_views_extension_consistent():
    cams = syn.make_rig(4, seed=8)
    poses = syn.make_poses(6, seed=9)
    k = syn.make_kpts_2d(poses, cams, seed=10, noise_px=0.0)
    cp = [(c["K"], c["R"], c["T"], c["dist"]) for c in cams]
    out = cv_ref.triangulate_all_views(cp, k, [0, 1, 2, 3])
    np.testing.assert_allclose(out, poses, atol=1e-3)


def test_hypot_restatement_matches_libm():
    """OpenCV's JacobiSVDImpl_ calls std::hypot = libm's (glibc 2.35 on this image and the GPU
    box).  The device's exact path restates glibc's algorithm (csrc/triangulate.hip hypot_glibc);
    the same text in C must equal libm on random pairs incl. near-equal magnitudes, wide exponent
    ranges, zeros and the rotation angles' typical (2p, a - b) pairs."""
    rng = np.random.default_rng(3)
    n = 400_000
    x = rng.uniform(-1, 1, n) * 10.0 ** rng.uniform(-30, 30, n)
    y = rng.uniform(-1, 1, n) * 10.0 ** rng.uniform(-30, 30, n)
    y[::3] = x[::3] * (1 + rng.uniform(-1e-3, 1e-3, n)[::3])
    y[1::7] = 0.0
    x[2::11] = rng.uniform(-1, 1, len(x[2::11])) * 1e300
    assert cv_ref.hypot_restatement_mismatches(x, y) == 0
