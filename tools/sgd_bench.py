"""Refinement kernel timing + parity deviations (BASELINE config 5: V=8, T=400 SGD)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mvpose import refine  # noqa: E402
from test_oracle_sgd import SGD_CASES, sgd_cams, sgd_kwargs  # noqa: E402
from test_sgd_gpu import MY_LENGTHS, _problem  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")
res = {}
for case in SGD_CASES:
    d = np.load(os.path.join(GOLDEN, case + ".npz"))
    opt = refine.Optimized_3d_Pose_Estimation(d["gauss"], d["init"], decomposed_cam_params_initial=dict(
        enumerate(sgd_cams(d))), body_lengths=dict(MY_LENGTHS))
    opt.sgd_optimize(print_frequency=10 ** 9, **sgd_kwargs(d))
    h = np.array(opt.all_costs_total["total_cost"], np.float64)
    res[case] = dict(best=float(np.abs(opt.best_trajectory.numpy() - d["best"]).max()),
                     final=float(np.abs(opt.trajectory.numpy() - d["final"]).max()),
                     hist_rel=float(np.max(np.abs(h - d["hist_total_cost"]) / np.abs(d["hist_total_cost"]))))
print(json.dumps({"golden_max_dev": res}))

V, T, iters = 8, 400, int(sys.argv[1]) if len(sys.argv) > 1 else 200
cams, g, x = _problem(V, T, seed=5)
kw = dict(lr=0.01, lambda_smooth=1e-6, lambda_body_length=1.0, patience=10 ** 9, tolerance=1e-5,
          max_iter=iters - 1, body_lengths=dict(MY_LENGTHS))
for M, bsz in ((1, None), (1, 40), (256, None)):
    G = np.broadcast_to(g, (M,) + g.shape).copy()
    X = np.broadcast_to(x, (M,) + x.shape).copy()
    refine.refine_trajectories(G, X, cams, batch_size=bsz, **kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = refine.refine_trajectories(G, X, cams, batch_size=bsz, **kw)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n_win = r["batch_costs"].shape[2]
    print(json.dumps({"M": M, "V": V, "T": T, "batch_size": bsz or T, "windows": n_win, "iterations": iters,
                      "ms_per_iteration": dt * 1e3 / iters, "us_per_window_step": dt * 1e6 / iters / n_win,
                      "trajectory_iterations_per_s": M * iters / dt}))
