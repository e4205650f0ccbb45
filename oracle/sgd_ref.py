"""ORACLE (test infrastructure only) — reprojection-error SGD refinement.

torch-CPU (autograd) restatement of the reference's trajectory-only refinement
path, pinned by tests/golden/sgd_*.npz / project.npz / bodylen.npz (generated
by importing the reference itself, tests/golden/make_golden.py):

* ``project_points``      pose_refinement.py:94-179 (project_points_torch)
* ``rotation_matrix``     utils.py:1219-1268 (rotation_conversion, to_vector=False)
* ``body_part_lengths``   utils.py:1164-1208 with CONNECTIVITY_DICT['coco'] (:1067)
* ``nan_mean``            pose_refinement.py:221-229
* ``refine``              Optimized_3d_Pose_Estimation.__init__ (:579-668) +
                          sgd_optimize (:894-1096) with optimize_trajectory=True,
                          no extrinsic learning, no NN — what the CLI runs
                          (:1210-1214).  Quirks kept: every camera is scored
                          against the CAMERA-0 Gaussian (:663, :885); the cost
                          history list doubles as the running-mean list (F6,
                          ``all_costs_total = all_costs.copy()`` :987); the
                          trajectory keeps moving outside the window (Adam
                          momentum, whole tensor); the loop runs while
                          ``iteration <= max_iter``.
"""
from __future__ import annotations

import numpy as np
import torch

# utils.py:1067 CONNECTIVITY_DICT['coco'] and the COCO joint names (utils.py:1071-1155)
COCO_EDGES = [(0, 1), (0, 2), (1, 3), (2, 4), (5, 7), (7, 9), (6, 8), (8, 10), (11, 13), (13, 15),
              (12, 14), (14, 16), (5, 6), (5, 11), (6, 12), (11, 12)]
COCO_NAMES = ["nose", "left_eye", "right_eye", "left_ear", "right_ear", "left_shoulder", "right_shoulder",
              "left_elbow", "right_elbow", "left_wrist", "right_wrist", "left_hip", "right_hip", "left_knee",
              "right_knee", "left_ankle", "right_ankle"]
EDGE_NAMES = [f"{COCO_NAMES[a]}_{COCO_NAMES[b]}" for a, b in COCO_EDGES]


def rotation_matrix(r, dtype=torch.float32):
    """(3,3) passes through; (3,) axis-angle -> Rodrigues (utils.py:1242-1262)."""
    r = torch.as_tensor(r, dtype=dtype)
    if r.shape == (3, 3):
        return r
    theta = torch.norm(r)
    if torch.abs(theta - torch.tensor(0.0)) < 1e-6:
        return torch.eye(3)
    ux, uy, uz = r / theta
    k = torch.tensor([[0, -uz, uy], [uz, 0, -ux], [-uy, ux, 0]])
    return torch.eye(3) + torch.sin(theta) * k + (1 - torch.cos(theta)) * torch.mm(k, k)


def project_points(points, K, R, T, dist, rows=None, ignore_distortions=False, dtype=torch.float32):
    """(Time, N, 3) -> (len(rows), N, 2) pixels; pose_refinement.py:94-179."""
    cast = (lambda a: a.to(dtype) if isinstance(a, torch.Tensor) else torch.tensor(a, dtype=dtype))
    K, T, points, dist = cast(K), cast(T), cast(points), cast(dist)
    R = rotation_matrix(cast(R), dtype)
    n_t, n_p, _ = points.shape
    rows = list(range(n_t)) if rows is None else rows
    X = points[rows].reshape(len(rows) * n_p, 3)
    Xh = torch.cat([X, torch.ones(X.shape[0], 1, dtype=dtype)], dim=-1)
    cam = Xh @ torch.cat([R, T.squeeze().unsqueeze(-1)], dim=-1).T
    x = cam[:, 0] / cam[:, 2]
    y = cam[:, 1] / cam[:, 2]
    if not ignore_distortions:
        r2 = x ** 2 + y ** 2
        k1, k2, p1, p2, k3 = dist.squeeze()
        radial = 1 + k1 * r2 + k2 * r2 ** 2 + k3 * r2 ** 3
        xd = x * radial
        yd = y * radial
        xd += 2 * p1 * x * y + p2 * (r2 + 2 * x ** 2)
        yd += p1 * (r2 + 2 * y ** 2) + 2 * p2 * x * y
        uv = torch.stack([xd, yd], dim=-1)
    else:
        uv = torch.stack([x, y], dim=-1)
    pix = torch.cat([uv, torch.ones(uv.shape[0], 1, dtype=dtype)], dim=-1) @ K.T
    pix = pix[:, :2] / pix[:, 2].unsqueeze(-1)
    return pix.reshape(len(rows), n_p, 2)


def body_part_lengths(pose):
    """{edge name: (T,) lengths}; utils.py:1164-1208 (torch branch)."""
    return {n: torch.norm(pose[:, b, :] - pose[:, a, :], dim=1) for n, (a, b) in zip(EDGE_NAMES, COCO_EDGES)}


def nan_mean(xs):
    """pose_refinement.py:221-229: mean over the finite entries of the stack."""
    s = torch.stack(xs)
    keep = ~(torch.isnan(s) | torch.isinf(s))
    return torch.sum(s[keep]) / len(s[keep])


def windows(n_t, batch):
    """create_batch_indices (pose_refinement.py:786-796): stride batch//2."""
    return [list(range(s, s + batch)) for s in range(0, n_t - batch + 1, batch // 2)]


class RefineResult:
    def __init__(self, best, final, history, iterations):
        self.best_trajectory = best
        self.trajectory = final
        self.all_costs_total = history
        self.iterations = iterations


def refine(gaussians, initial_trajectory, cams, body_lengths=None, lr=0.001, betas=(0.9, 0.999),
           lambda_smooth=1.0, lambda_body_length=1.0, patience=100, tolerance=1e-5, max_iter=1000,
           batch_size=None, ignore_distortions=False, time_interval=(0, -1), dtype=torch.float32):
    """Trajectory-only Optimized_3d_Pose_Estimation(...).sgd_optimize(...).

    gaussians (T,V,J,6), initial_trajectory (T,J,3), cams = list of V
    [K(3,3), R(3,3) or axis-angle(3), T(3,1), dist(1,5)] (camera order = camera IDs 0..V-1),
    body_lengths = {edge name: length} in the YAML's key order.
    """
    G = torch.as_tensor(np.asarray(gaussians), dtype=dtype)
    n_j = G.shape[2]
    cams = [[torch.as_tensor(np.asarray(p), dtype=dtype) for p in c] for c in cams]
    cov = G[:, 0, :, 2:].reshape(G.shape[0], n_j, 2, 2)
    cov = cov + 1e-6 * torch.eye(2).expand_as(cov)
    cov_inv = torch.linalg.inv(cov).to(dtype)                         # same for every camera (:663)
    a, b = time_interval
    Gs, Cs = G[a:b], cov_inv[a:b]
    n_t = len(Gs)
    batch = n_t if batch_size is None else int(batch_size)
    n_t = int(np.floor(n_t / batch) * batch)
    Gs = Gs[:n_t]
    traj = torch.as_tensor(np.asarray(initial_trajectory), dtype=dtype)[a:b].clone().detach()
    traj.requires_grad_(True)
    bl_keys = list(body_lengths.keys()) if body_lengths is not None else []
    a_vec = torch.tensor(list(body_lengths.values()), dtype=dtype).unsqueeze(1) if body_lengths else None
    if a_vec is not None:
        a_vec = a_vec.repeat_interleave(batch, dim=0).view(batch * len(bl_keys), 1).squeeze()
    opt = torch.optim.Adam([traj], lr=lr, betas=betas)
    names = ["total_cost", "likelihood_cost"]
    if lambda_smooth > 0:
        names.append("smoothness_cost")
    if lambda_body_length > 0:
        names.append("body_length_cost")
    hist = {n: [] for n in names}          # per-batch costs AND running means (F6)
    best_total, best, no_imp, it = float("inf"), None, 0, 0
    wins = windows(n_t, batch)
    while no_imp < patience and it <= max_iter:
        for rows in wins:
            opt.zero_grad()
            costs = {}
            like = []
            mean = Gs[rows, 0, :, :2].squeeze()
            for cam in cams:
                uv = project_points(traj, *cam, rows=rows, ignore_distortions=ignore_distortions, dtype=dtype)
                d = uv - mean
                like.append(-(-0.5 * torch.einsum("...i,...ij,...j->...", d, Cs[rows], d)))
            costs["likelihood_cost"] = nan_mean(like)
            if lambda_smooth > 0:
                sm = [torch.norm((traj[rows[i]] - traj[rows[i] - 1]) - (traj[rows[i] - 1] - traj[rows[i] - 2])) ** 2
                      for i in range(2, len(rows))]
                costs["smoothness_cost"] = lambda_smooth * nan_mean(sm)
            if lambda_body_length > 0:
                L = body_part_lengths(traj[rows])
                bvec = torch.hstack([L[k] for k in bl_keys]).squeeze()
                mu = torch.dot(a_vec, bvec) / torch.dot(bvec, bvec)
                costs["body_length_cost"] = (lambda_body_length * torch.norm(a_vec - mu * bvec) ** 2
                                             / torch.norm(a_vec) ** 2)
            total = torch.sum(torch.stack(list(costs.values())))
            costs["total_cost"] = total
            total.backward()
            torch.nn.utils.clip_grad_norm_([traj], max_norm=1.0)
            opt.step()
            for n in names:
                hist[n].append(costs[n].clone().detach())
        for n in names:
            hist[n].append(np.mean(hist[n], 0))
        cur = hist["total_cost"][-1]
        if cur < best_total - tolerance:
            best_total = cur
            best = traj.clone().detach()
            no_imp = 0
        else:
            no_imp += 1
        if no_imp >= patience:
            break
        it += 1
    return RefineResult(best, traj.detach().clone(), hist, it)
