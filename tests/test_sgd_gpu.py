"""GPU parity: HIP refinement (mvp_sgd_refine, mvp_project_points) vs the
reference's golden vectors and the oracle (oracle/sgd_ref.py, itself pinned
bit-exactly to those vectors by test_oracle_sgd.py).

Tolerances (written here, float32 path):
* projection: |Δuv| <= 2e-3 px on ~1e3 px values (a few f32 ulp; the
  reference's [R|T] product goes through BLAS in an order we do not reproduce);
* refinement: trajectories within SGD_ATOL = 1e-4 cm after the golden runs' 5-60
  Adam steps (measured <= 6.1e-5 cm, profiles/r01_sgd_bench.log: f32 rounding of the
  gradient in a different summation order than torch's autograd; Adam normalises the
  gradient, so such differences move a step by far less than lr);
  running-mean cost histories within rtol 1e-4; identical iteration counts
  (early stop) and identical history lengths.
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import sgd_ref
from test_oracle_sgd import C5_CASES, SGD_CASES, c5_problem, sgd_cams, sgd_kwargs

pytestmark = pytest.mark.gpu
SGD_ATOL = 1e-4

with open(os.path.join(GOLDEN, "body_part_lengths.json")) as _f:
    MY_LENGTHS = json.load(_f)["my_lengths"]


@pytest.fixture(scope="module")
def refine():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mvpose import refine as _refine
    return _refine


def test_project_points_golden(refine):
    d = np.load(os.path.join(GOLDEN, "project.npz"))
    pts = torch.tensor(d["points"])
    for v in range(3):
        for ign in (0, 1):
            out = refine.project_points_torch(pts, d["K"][v], d["R"][v], d["T"][v], d["dist"][v],
                                              ignore_distortions=bool(ign))
            np.testing.assert_allclose(out.numpy(), d[f"out_c{v}_{ign}"], rtol=0, atol=2e-3)
    out = refine.project_points_torch(pts.cuda(), d["K"][1], torch.tensor(d["rvec"], dtype=torch.float32),
                                      d["T"][1], d["dist"][1])
    assert out.is_cuda
    np.testing.assert_allclose(out.cpu().numpy(), d["out_axisangle"], rtol=0, atol=2e-3)
    out = refine.project_points_torch(pts, d["K"][0], d["R"][0], d["T"][0], d["dist"][0], indicies=[4, 1])
    np.testing.assert_allclose(out.numpy(), d["out_c0_0"][[4, 1]], rtol=0, atol=2e-3)


@pytest.mark.parametrize("case", SGD_CASES)
def test_sgd_matches_reference_golden(refine, case):
    d = np.load(os.path.join(GOLDEN, case + ".npz"))
    cams = {i: c for i, c in enumerate(sgd_cams(d))}
    opt = refine.Optimized_3d_Pose_Estimation(d["gauss"], d["init"], decomposed_cam_params_initial=cams,
                                              body_lengths=dict(MY_LENGTHS))
    opt.sgd_optimize(print_frequency=10 ** 9, **sgd_kwargs(d))
    assert opt.best_trajectory.shape == d["best"].shape
    np.testing.assert_allclose(opt.best_trajectory.numpy(), d["best"], rtol=0, atol=SGD_ATOL)
    np.testing.assert_allclose(opt.trajectory.numpy(), d["final"], rtol=0, atol=SGD_ATOL)
    for k, v in opt.all_costs_total.items():
        ref = d["hist_" + k]
        assert len(v) == len(ref), k
        np.testing.assert_allclose(np.array(v, np.float64), ref, rtol=1e-4, atol=1e-7, err_msg=k)


@pytest.mark.parametrize("case", C5_CASES)
def test_sgd_config5_matches_reference_golden(refine, case):
    """BASELINE config 5 at its own size (V=8, T=400 -> 399 rows after time_interval [0, -1]):
    T*J = 6,783 > 1024 runs sgd_kernel<1024, false> (the bench's kernel), trajectory in LDS.
    One window (8 iterations), overlapping windows of 100 (7 windows), early stop (64
    iterations, patience 3)."""
    from mvpose import refine as _r
    d = np.load(os.path.join(GOLDEN, case + ".npz"))
    cams, gauss, init = c5_problem(d)
    opt = _r.Optimized_3d_Pose_Estimation(gauss, init, decomposed_cam_params_initial=dict(enumerate(cams)),
                                          body_lengths=dict(MY_LENGTHS))
    opt.sgd_optimize(print_frequency=10 ** 9, **sgd_kwargs(d))
    np.testing.assert_allclose(opt.best_trajectory.numpy(), d["best"], rtol=0, atol=SGD_ATOL)
    np.testing.assert_allclose(opt.trajectory.numpy(), d["final"], rtol=0, atol=SGD_ATOL)
    for k, v in opt.all_costs_total.items():
        ref = d["hist_" + k]
        assert len(v) == len(ref), k
        np.testing.assert_allclose(np.array(v, np.float64), ref, rtol=1e-4, atol=1e-7, err_msg=k)


def test_sgd_long_trajectory_outside_lds_matches_oracle(refine):
    """T = 700 rows: the trajectory (142 KB) exceeds the kernel's 120 KB LDS budget, so the
    Adam state and the trajectory live in the global workspace (traj_in_lds == false,
    csrc/sgd.hip sgd_launch) — against the oracle, windows of 140 and one window."""
    for V, T, kw in ((2, 701, dict(batch_size=140, lr=0.02, lambda_smooth=1e-3, lambda_body_length=0.5,
                                     max_iter=4)),
                     (3, 701, dict(batch_size=None, lr=0.01, lambda_smooth=1e-6, lambda_body_length=1.0,
                                   max_iter=6))):
        cams, gauss, init = _problem(V, T, seed=300 + V)
        ref = sgd_ref.refine(gauss, init, cams, body_lengths=dict(MY_LENGTHS), **kw)
        opt = refine.Optimized_3d_Pose_Estimation(gauss, init, decomposed_cam_params_initial=dict(enumerate(cams)),
                                                  body_lengths=dict(MY_LENGTHS))
        opt.sgd_optimize(print_frequency=10 ** 9, **kw)
        np.testing.assert_allclose(opt.best_trajectory.numpy(), ref.best_trajectory.numpy(), rtol=0, atol=SGD_ATOL)
        np.testing.assert_allclose(opt.trajectory.numpy(), ref.trajectory.numpy(), rtol=0, atol=SGD_ATOL)
        for k in ref.all_costs_total:
            np.testing.assert_allclose(np.array(opt.all_costs_total[k], np.float64),
                                       np.array([float(x) for x in ref.all_costs_total[k]]), rtol=1e-4, atol=1e-7)


def _problem(V, T, seed):
    from mvpose import synthetic as syn
    rng = np.random.default_rng(seed)
    cams = syn.make_rig(V, seed=seed)
    poses = syn.make_poses(T, seed=seed + 1)
    gauss = np.zeros((T, V, 17, 6))
    for v, c in enumerate(cams):
        gauss[:, v, :, 0:2] = syn.project(poses, c) + rng.normal(0, 2.0, (T, 17, 2))
        s = rng.uniform(2.0, 6.0, (T, 17, 2))
        rho = rng.uniform(-0.4, 0.4, (T, 17))
        gauss[:, v, :, 2] = s[..., 0] ** 2
        gauss[:, v, :, 3] = gauss[:, v, :, 4] = rho * s[..., 0] * s[..., 1]
        gauss[:, v, :, 5] = s[..., 1] ** 2
    init = (poses + rng.normal(0, 3.0, poses.shape)).astype(np.float32)
    return [[c["K"], c["R"], c["T"], c["dist"]] for c in cams], gauss, init


@pytest.mark.parametrize("V,T,kw", [
    (3, 50, dict(batch_size=16, lr=0.02, lambda_smooth=1e-3, lambda_body_length=0.5, max_iter=8)),
    (4, 33, dict(batch_size=None, lr=0.01, lambda_smooth=0.0, lambda_body_length=1.0, max_iter=12,
                 ignore_distortions=True)),
    (2, 41, dict(batch_size=10, lr=0.01, lambda_smooth=1e-6, lambda_body_length=0.0, max_iter=6,
                 time_interval=[3, -2])),
])
def test_sgd_matches_oracle(refine, V, T, kw):
    cams, gauss, init = _problem(V, T, seed=100 + V + T)
    ref = sgd_ref.refine(gauss, init, cams, body_lengths=dict(MY_LENGTHS), **kw)
    opt = refine.Optimized_3d_Pose_Estimation(gauss, init, decomposed_cam_params_initial=dict(enumerate(cams)),
                                              body_lengths=dict(MY_LENGTHS))
    opt.sgd_optimize(print_frequency=10 ** 9, **kw)
    np.testing.assert_allclose(opt.best_trajectory.numpy(), ref.best_trajectory.numpy(), rtol=0, atol=SGD_ATOL)
    np.testing.assert_allclose(opt.trajectory.numpy(), ref.trajectory.numpy(), rtol=0, atol=SGD_ATOL)
    assert list(opt.all_costs_total) == list(ref.all_costs_total)
    for k in ref.all_costs_total:
        np.testing.assert_allclose(np.array(opt.all_costs_total[k], np.float64),
                                   np.array([float(x) for x in ref.all_costs_total[k]]), rtol=1e-4, atol=1e-7)


def test_batched_trajectories_equal_single_runs(refine):
    """M independent trajectories in one launch == M separate launches (bitwise)."""
    cams, g0, x0 = _problem(2, 48, seed=7)
    _, g1, x1 = _problem(2, 48, seed=8)
    kw = dict(batch_size=12, lr=0.01, lambda_smooth=1e-4, lambda_body_length=1.0, max_iter=20,
              body_lengths=dict(MY_LENGTHS))
    both = refine.refine_trajectories(np.stack([g0, g1]), np.stack([x0, x1]), cams, **kw)
    for i, (g, x) in enumerate(((g0, x0), (g1, x1))):
        one = refine.refine_trajectories(g[None], x[None], cams, **kw)
        for key in ("best", "final", "iter_means", "iters"):
            assert torch.equal(both[key][i], one[key][0]), key


def test_sgd_argument_errors(refine):
    from mvpose._lib import MvposeError
    cams, g, x = _problem(2, 10, seed=3)
    with pytest.raises(ValueError):
        refine.refine_trajectories(g[None], x[None], cams, batch_size=1, body_lengths=dict(MY_LENGTHS))
    with pytest.raises(ValueError):
        refine.refine_trajectories(g[None], x[None], cams, body_lengths=None, lambda_body_length=1.0)
    with pytest.raises(KeyError):
        refine.refine_trajectories(g[None], x[None], cams, body_lengths={"left_nose_right_toe": 3.0})
    assert issubclass(MvposeError, RuntimeError)


@pytest.mark.parametrize("case,kw", [("default", {}), ("rolling", dict(use_rolling_average=True)),
                                     ("nomedian", dict(filter_distance_from_median=False)),
                                     ("k7", dict(k=7, k_std=1.5, median_std=3))])
def test_linear_interpolation_golden(refine, case, kw):
    """mvp_linear_interpolation vs the reference's output (interp.npz): the f32 window
    statistics decide the same kept set, the f64 line fit rounds to the same f32."""
    d = np.load(os.path.join(GOLDEN, "interp.npz"))
    out = refine.linear_interpolation(d["points"], **kw)
    assert out.dtype == np.float32 and out.shape == d["points"].shape
    np.testing.assert_allclose(out, d["out_" + case], rtol=2e-7, atol=1e-6)


def test_linear_interpolation_matches_oracle_large(refine):
    from oracle import interp_ref
    rng = np.random.default_rng(5)
    pts = (np.cumsum(rng.normal(0, 1, (120, 17, 3)), axis=0) + rng.normal(0, 0.2, (120, 17, 3))).astype(np.float32)
    pts[rng.integers(0, 120, 60), rng.integers(0, 17, 60), rng.integers(0, 3, 60)] += 30
    ref = interp_ref.linear_interpolation(pts)
    out = refine.linear_interpolation(torch.tensor(pts, device="cuda"))
    assert out.is_cuda
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=2e-7, atol=1e-6)
    two_d = refine.linear_interpolation(pts[:, :, 0])
    np.testing.assert_allclose(two_d, ref[:, :, 0], rtol=2e-7, atol=1e-6)
