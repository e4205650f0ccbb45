"""Reprojection-error trajectory refinement on the GPU (mvp_sgd_refine).

Host mirror of the reference's refinement API (pose_refinement.py):

* ``Optimized_3d_Pose_Estimation(gaussians, initial_trajectory,
  decomposed_cam_params_initial, body_lengths, camera_IDs, ...)`` (:579) and
  its ``sgd_optimize(**kwargs)`` (:894) with the same keywords and defaults;
  afterwards ``best_trajectory``, ``trajectory``, ``all_costs_total`` and
  ``best_decomposed_cam_params`` read like the reference's.  The whole
  optimisation (every iteration and window) is ONE kernel launch.
* ``refine_trajectories(...)``: M independent trajectories (same rig) in one
  launch, one workgroup each — the throughput form (SGD shards as replicas).
* ``project_points_torch`` (:94-179) and ``linear_interpolation`` (:15-84) on the GPU.

* Extrinsic learning from samples (``sgd_optimize(extrinsic_optimization_IDs=[id],
  optimize_trajectory=False, GT_camera_IDs=[a, b])``, :684-706, :800-831, :915-943):
  the per-step cost and R/T gradient over every triangulated Gaussian sample is one
  HIP launch (mvp_extrinsic_sample_grad); the 12 learnable numbers, Adam and
  clip_grad_norm_ stay torch CPU tensors exactly as in the reference.

* Joint trajectory + extrinsic optimisation (``sgd_optimize(extrinsic_optimization_IDs=ids,
  optimize_trajectory=True)``, :931-954 + :894-1096): the listed cameras' R (3x3) and T
  learn inside the same single-launch optimisation (mvp_sgd_refine_cams: their likelihood
  gradient, their own Adam state, one clip_grad_norm_ over [R, T, ..., trajectory]).

Scope: the NN trajectory parameterisation (``use_NN``) and ``randomize_params`` raise
NotImplementedError.  A joint call that would learn an axis-angle R raises it too: the
reference converts each learnable camera's INITIAL R to axis-angle (:935), so a second joint
call with ``reset_camera_params=True`` restarts from that vector and learns its 3 numbers;
the kernel learns R as a 3x3 matrix only.  A trajectory-only call after such a reset runs
(the fixed axis-angle R is converted to its matrix, as project_points_torch does).
"""
from __future__ import annotations

import ctypes
import math
import random
import threading

import numpy as np
import torch

from . import _lib
from . import ops
from ._lib import call

CAM_FLOATS = 26
N_COSTS = 4
COST_NAMES = ("total_cost", "likelihood_cost", "smoothness_cost", "body_length_cost")

# reference utils.py:1067 CONNECTIVITY_DICT['coco'], joint names utils.py:1071-1155;
# segment names are generate_connectivity_names' "<start>_<end>" (utils.py:1055-1062).
COCO_JOINTS = ("nose", "left_eye", "right_eye", "left_ear", "right_ear", "left_shoulder", "right_shoulder",
               "left_elbow", "right_elbow", "left_wrist", "right_wrist", "left_hip", "right_hip", "left_knee",
               "right_knee", "left_ankle", "right_ankle")
COCO_CONNECTIONS = ((0, 1), (0, 2), (1, 3), (2, 4), (5, 7), (7, 9), (6, 8), (8, 10), (11, 13), (13, 15),
                    (12, 14), (14, 16), (5, 6), (5, 11), (6, 12), (11, 12))
SEGMENTS = {f"{COCO_JOINTS[a]}_{COCO_JOINTS[b]}": (a, b) for a, b in COCO_CONNECTIONS}


class SgdParams(ctypes.Structure):
    """mvp_sgd_params (include/mvpose.h)."""
    _fields_ = [("lr", ctypes.c_double), ("beta1", ctypes.c_double), ("beta2", ctypes.c_double),
                ("adam_eps", ctypes.c_double), ("lambda_smooth", ctypes.c_double),
                ("lambda_body_length", ctypes.c_double), ("tolerance", ctypes.c_double),
                ("max_grad_norm", ctypes.c_double), ("patience", ctypes.c_int), ("max_iter", ctypes.c_int),
                ("batch_size", ctypes.c_int), ("ignore_distortions", ctypes.c_int),
                ("own_camera_gaussians", ctypes.c_int)]


_lib.lib.mvp_sgd_refine.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                    ctypes.POINTER(SgdParams), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


_PINNED = {}
_PINNED_LOCK = threading.Lock()


def _h2d_words(words, dev):
    """A small int32 host array on the device through a reused pinned staging buffer and an
    asynchronous copy (a pageable copy synchronises the stream: tens of microseconds of idle
    device per call).  The buffer is rewritten only after its previous copy has completed."""
    n = int(words.size)
    with _PINNED_LOCK:
        buf, ev = _PINNED.get(dev, (None, None))
        if buf is None or buf.numel() < n:
            buf, ev = torch.empty(max(n, 4096), dtype=torch.int32).pin_memory(), None
        if ev is not None:
            ev.synchronize()
        buf[:n].numpy()[:] = words
        out = buf[:n].to(dev, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        _PINNED[dev] = (buf, ev)
    return out


def _on_device_f32(a, dev):
    """a as a contiguous float32 tensor on dev (device-resident float32 inputs pass through
    without a .to() call, which costs tens of microseconds even when it is a no-op)."""
    if isinstance(a, torch.Tensor) and a.dtype == torch.float32 and a.device == dev and a.is_contiguous():
        return a
    return torch.as_tensor(a).to(device=dev, dtype=torch.float32).contiguous()


def _device(device):
    dev = torch.device(device if device is not None else "cuda")
    if dev.type != "cuda":
        raise ValueError("mvpose refinement runs on the GPU only (no CPU fallback)")
    if dev.index is None and torch.cuda.is_available():
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev


def rotation_conversion(rotation_rep, to_vector=True):
    """utils.py:1219-1268: axis-angle <-> matrix (host, float32 torch like the reference)."""
    was_np = isinstance(rotation_rep, np.ndarray)
    r = torch.as_tensor(rotation_rep)
    if r.shape == (3, 3) and to_vector:
        theta = torch.acos((torch.trace(r) - 1) / 2)
        if torch.abs(theta) < 1e-6:
            return torch.zeros(3)
        s = 2 * torch.sin(theta)
        out = theta * torch.tensor([(r[2, 1] - r[1, 2]) / s, (r[0, 2] - r[2, 0]) / s, (r[1, 0] - r[0, 1]) / s])
    elif r.shape != (3, 3) and not to_vector:
        theta = torch.norm(r)
        if torch.abs(theta) < 1e-6:
            return torch.eye(3)
        ux, uy, uz = r / theta
        k = torch.tensor([[0, -uz, uy], [uz, 0, -ux], [-uy, ux, 0]])
        out = torch.eye(3) + torch.sin(theta) * k + (1 - torch.cos(theta)) * torch.mm(k, k)
    else:
        out = r
    return np.array(out) if was_np else out


def camera_record(K, R, T, dist) -> np.ndarray:
    """One MVP_SGD_CAM_FLOATS f32 record [K | R (matrix) | T | dist] from the reference's
    decomposed parameters (R may be a 3x3 matrix or an axis-angle vector)."""
    if not any(isinstance(a, torch.Tensor) for a in (K, R, T, dist)) and np.size(R) == 9:
        # numpy in, R a matrix: the float32 casts alone (what the torch path below computes for
        # it, without its per-camera tensor round trips)
        d = np.asarray(dist, dtype=np.float32).reshape(-1)
        if d.size != 5:
            raise ValueError("dist_coeffs must have shape (1, 5)")
        return np.concatenate([np.asarray(K, dtype=np.float32).reshape(9), np.asarray(R, dtype=np.float32).reshape(9),
                               np.asarray(T, dtype=np.float32).reshape(3), d])
    f32 = (lambda a: torch.as_tensor(np.asarray(a) if not isinstance(a, torch.Tensor) else a).to(torch.float32))
    Rm = rotation_conversion(f32(R), to_vector=False)
    d = f32(dist).reshape(-1)
    if d.numel() != 5:
        raise ValueError("dist_coeffs must have shape (1, 5)")
    rec = np.concatenate([f32(K).reshape(9).numpy(), torch.as_tensor(Rm, dtype=torch.float32).reshape(9).numpy(),
                          f32(T).reshape(3).numpy(), d.numpy()]).astype(np.float32)
    return rec


def segments_for(body_lengths):
    """body_lengths {segment name: length} (YAML order) -> (pairs int32 (n,2), lengths f32 (n,))."""
    names = list(body_lengths.keys())
    unknown = [n for n in names if n not in SEGMENTS]
    if unknown:
        raise KeyError(f"unknown body segment(s) {unknown}; expected names from {list(SEGMENTS)}")
    pairs = np.array([SEGMENTS[n] for n in names], np.int32).reshape(-1, 2)
    lens = np.array([float(body_lengths[n]) for n in names], np.float32)
    return pairs, lens


def project_points_torch(points, K, R, T, dist_coeffs, indicies=None, torch_dtype=torch.float32,
                         ignore_distortions=False, device=None):
    """pose_refinement.py:94-179 on the GPU: (Time, N, 3) -> (len(indicies), N, 2) f32.
    Returned on the device the points came from (CPU points are copied over and back)."""
    if torch_dtype != torch.float32:
        raise NotImplementedError("float32 only (the reference's default)")
    pts = torch.as_tensor(points).to(torch.float32)
    if pts.dim() != 3 or pts.shape[2] != 3:
        raise ValueError("points must have shape (Time, N, 3)")
    home = pts.device
    dev = _device(device if device is not None else (home if home.type == "cuda" else "cuda"))
    rows = list(range(pts.shape[0])) if indicies is None else list(indicies)
    sel = pts[rows].reshape(-1, 3).to(dev).contiguous()
    cam = torch.from_numpy(camera_record(K, R, T, dist_coeffs)).to(dev)
    uv = torch.empty((sel.shape[0], 2), dtype=torch.float32, device=dev)
    call("mvp_project_points", _ptr(sel), sel.shape[0], _ptr(cam), int(bool(ignore_distortions)), _ptr(uv),
         _stream(dev))
    return uv.reshape(len(rows), pts.shape[1], 2).to(home)


def linear_interpolation(points, k=5, k_std=2, median_std=2, use_rolling_average=False,
                         filter_distance_from_median=True, device=None):
    """pose_refinement.py:15-84 on the GPU (mvp_linear_interpolation).  points (T, P, D) or
    (T, P); returns a float32 array of the same shape (numpy in, numpy out; tensors stay tensors)."""
    was_tensor = isinstance(points, torch.Tensor)
    x = points if was_tensor else torch.from_numpy(np.ascontiguousarray(np.asarray(points)))
    home = x.device
    dev = _device(device if device is not None else (home if home.type == "cuda" else "cuda"))
    squeeze = x.dim() == 2
    x = (x[..., None] if squeeze else x).to(device=dev, dtype=torch.float32).contiguous()
    if x.dim() != 3:
        raise ValueError("points must be (time, n_points, dim) or (time, n_points)")
    out = torch.empty_like(x)
    T, P, D = x.shape
    call("mvp_linear_interpolation", _ptr(x), T, P, D, int(k), float(k_std), float(median_std),
         int(bool(use_rolling_average)), int(bool(filter_distance_from_median)), _ptr(out), _stream(dev))
    out = out[..., 0] if squeeze else out
    return out.to(home) if was_tensor else out.cpu().numpy()


EXT_SUMS = 14


def extrinsic_sample_grad(samples, targets, cam, n_samples, ignore_distortions=False, n_blocks=None):
    """One mvp_extrinsic_sample_grad pass.  samples (T, J, N, 3) f32 and targets (T, J, 6) f32
    [mean x, mean y, Σ⁻¹ 00, 01, 10, 11] on the GPU, cam = one MVP_SGD_CAM_FLOATS f32 record on
    the GPU.  Returns the reduced fp64 sums (14,) on the device:
    [Σ 0.5 dᵀΣ⁻¹d, finite count, Σ dq/dR (9), Σ dq/dT (3)]."""
    n_pts = samples.numel() // 3
    if samples.dtype != torch.float32 or targets.dtype != torch.float32 or cam.dtype != torch.float32:
        raise TypeError("samples, targets and cam must be float32")
    if not (samples.is_contiguous() and targets.is_contiguous() and cam.numel() == CAM_FLOATS):
        raise ValueError("samples/targets must be contiguous, cam one 26-float record")
    if targets.numel() * n_samples != 6 * n_pts:
        raise ValueError(f"targets {tuple(targets.shape)} do not match {n_pts} samples of {n_samples} per target")
    if n_blocks is None:
        n_blocks = max(1, min(1024, (n_pts + 255) // 256))
    part = torch.empty((n_blocks, EXT_SUMS), dtype=torch.float64, device=samples.device)
    call("mvp_extrinsic_sample_grad", _ptr(samples), _ptr(targets), int(n_samples), int(n_pts), _ptr(cam),
         int(bool(ignore_distortions)), int(n_blocks), _ptr(part), _stream(samples.device))
    return part.sum(0)


def refine_trajectories(gaussians, initial_trajectories, cameras, body_lengths=None, lr=0.001, betas=(0.9, 0.999),
                        lambda_smooth=1.0, lambda_body_length=1.0, patience=100, tolerance=1e-5, max_iter=1000,
                        batch_size=None, ignore_distortions=False, own_camera_gaussians=False, max_grad_norm=1.0,
                        adam_eps=1e-8, device=None, learn_cams=None):
    """M trajectories in one launch.  gaussians (M,T,V,J,6), initial_trajectories (M,T,J,3)
    (already time-sliced), cameras = V x (K, R, T, dist).  Returns device tensors:
    best (M,T,J,3) (NaN rows if never improved), final, batch_costs (M,max_iter+1,n_win,4),
    iter_means (M,max_iter+1,4), iters (M,).
    learn_cams: camera slots (<= 2) whose R (3x3) and T are learned jointly with the trajectory
    (mvp_sgd_refine_cams); adds cams_final / cams_best (M, n_learn, 12) = [R row-major | T]
    (best NaN if never improved)."""
    dev = _device(device)
    G = _on_device_f32(gaussians, dev)
    X0 = _on_device_f32(initial_trajectories, dev)
    if G.dim() != 5 or G.shape[-1] != 6 or X0.dim() != 4 or X0.shape[-1] != 3:
        raise ValueError("gaussians must be (M,T,V,J,6) and initial_trajectories (M,T,J,3)")
    M, T, V, J = G.shape[:4]
    if X0.shape[:3] != (M, T, J):
        raise ValueError(f"initial_trajectories {tuple(X0.shape)} does not match gaussians {tuple(G.shape)}")
    if len(cameras) != V:
        raise ValueError(f"{len(cameras)} cameras for V={V}")
    B = T if batch_size is None else int(batch_size)
    if B < 2 or B > T:
        raise ValueError(f"batch_size {B} must be in [2, T={T}]")
    if lambda_body_length > 0 and not body_lengths:
        raise ValueError("lambda_body_length > 0 needs body_lengths (reference create_body_length_vect)")
    # the constant tables (camera records, segment pairs and lengths: all 4-byte words) in one
    # host-to-device copy
    recs = np.stack([camera_record(*c) for c in cameras]).astype(np.float32).reshape(-1)
    if body_lengths:
        pairs, lens = segments_for(body_lengths)
        n_seg = len(lens)
        words = np.concatenate([recs.view(np.int32), pairs.astype(np.int32).reshape(-1), lens.view(np.int32)])
    else:
        n_seg = 0
        words = recs.view(np.int32)
    tab = _h2d_words(words, dev)
    cams = tab[:recs.size].view(torch.float32).view(V, -1)
    seg = tab[recs.size:recs.size + 2 * n_seg] if n_seg else None
    seg_len = tab[recs.size + 2 * n_seg:].view(torch.float32) if n_seg else None
    p = SgdParams(lr=float(lr), beta1=float(betas[0]), beta2=float(betas[1]), adam_eps=float(adam_eps),
                  lambda_smooth=float(lambda_smooth), lambda_body_length=float(lambda_body_length),
                  tolerance=float(tolerance), max_grad_norm=float(max_grad_norm), patience=int(patience),
                  max_iter=int(max_iter), batch_size=B, ignore_distortions=int(bool(ignore_distortions)),
                  own_camera_gaussians=int(bool(own_camera_gaussians)))
    t_win = (T // B) * B
    n_win = (t_win - B) // (B // 2) + 1
    nws = ctypes.c_int64()
    call("mvp_sgd_workspace_floats", M, T, V, J, ctypes.byref(nws))
    ws = torch.empty(nws.value, dtype=torch.float32, device=dev)
    best = torch.empty_like(X0)
    final = torch.empty_like(X0)
    n_it = int(max_iter) + 1
    # the three zero-initialised outputs: one fill
    n_bc, n_im = M * n_it * n_win * N_COSTS, M * n_it * N_COSTS
    zero = torch.zeros(n_bc + n_im + M, dtype=torch.int32, device=dev)
    batch_costs = zero[:n_bc].view(torch.float32).view(M, n_it, n_win, N_COSTS)
    iter_means = zero[n_bc:n_bc + n_im].view(torch.float32).view(M, n_it, N_COSTS)
    iters = zero[n_bc + n_im:]
    out = {"best": best, "final": final, "batch_costs": batch_costs, "iter_means": iter_means, "iters": iters}
    if learn_cams:
        nl = len(learn_cams)
        slots = (ctypes.c_int * nl)(*[int(c) for c in learn_cams])
        cf = torch.empty((M, nl, 12), dtype=torch.float32, device=dev)
        cb = torch.full((M, nl, 12), float("nan"), dtype=torch.float32, device=dev)
        call("mvp_sgd_refine_cams", _ptr(G), _ptr(X0), _ptr(cams), M, T, V, J, _ptr(seg), _ptr(seg_len), n_seg,
             ctypes.byref(p), _ptr(ws), _ptr(final), _ptr(best), _ptr(batch_costs), _ptr(iter_means), _ptr(iters),
             slots, nl, _ptr(cf), _ptr(cb), _stream(dev))
        out["cams_final"], out["cams_best"] = cf, cb
    else:
        call("mvp_sgd_refine", _ptr(G), _ptr(X0), _ptr(cams), M, T, V, J, _ptr(seg), _ptr(seg_len), n_seg,
             ctypes.byref(p), _ptr(ws), _ptr(final), _ptr(best), _ptr(batch_costs), _ptr(iter_means), _ptr(iters),
             _stream(dev))
    return out


class Optimized_3d_Pose_Estimation:
    """GPU drop-in for pose_refinement.Optimized_3d_Pose_Estimation (:579-668)."""

    # extrinsic-from-samples branch: Adam steps on the device (mvp_extrinsic_adam_step) when the
    # learnable R is a 3x3 matrix; False = the host loop (torch CPU Adam per step), kept for
    # axis-angle R and as the tests' comparison
    device_adam = True

    def __init__(self, gaussians, initial_trajectory, decomposed_cam_params_initial=None, body_lengths=None,
                 camera_IDs=None, R_initial=None, T_initial=None, N_sample_points=100, torch_dtype=torch.float32,
                 device=None):
        if torch_dtype != torch.float32:
            raise NotImplementedError("float32 only (the reference's default)")
        if decomposed_cam_params_initial is None:
            raise ValueError("decomposed_cam_params_initial is required")
        for cid, prm in decomposed_cam_params_initial.items():   # :601-606
            if prm[1] is None:
                prm[1] = torch.eye(3)
            if prm[2] is None:
                prm[2] = torch.zeros(3, 1)
        self.device = _device(device)
        self.torch_dtype = torch_dtype
        self.gaussians = torch.as_tensor(np.asarray(gaussians) if not isinstance(gaussians, torch.Tensor)
                                         else gaussians).to(torch.float32)
        self.initial_trajectory = torch.as_tensor(np.asarray(initial_trajectory) if not isinstance(
            initial_trajectory, torch.Tensor) else initial_trajectory).to(torch.float32)
        self.decomposed_cam_params_initial = {
            k: [torch.as_tensor(np.asarray(c) if not isinstance(c, torch.Tensor) else c).to(torch.float32)
                for c in v] for k, v in decomposed_cam_params_initial.items()}
        self.decomposed_cam_params = {k: [c.clone() for c in v] for k, v in self.decomposed_cam_params_initial.items()}
        self.n_cams = self.gaussians.shape[1]
        self.n_joints = self.gaussians.shape[2]
        self.n_dims = self.initial_trajectory.shape[2]
        self.N_sample_points = N_sample_points
        self.body_lengths = body_lengths
        self.camera_IDs = camera_IDs if camera_IDs is not None else list(decomposed_cam_params_initial.keys())
        keys = list(self.decomposed_cam_params.keys())
        self.camera_indices = [keys.index(i) for i in self.camera_IDs]
        self.best_trajectory = None
        self.best_decomposed_cam_params = None

    def sgd_optimize(self, extrinsic_optimization_IDs=[], optimize_trajectory=True, lr=0.001, betas=(0.9, 0.999),
                     lambda_smooth=1.0, lambda_body_length=1.0, patience=100, tolerance=1e-5, max_iter=1000,
                     print_frequency=100, batch_size=None, N_sample_points=100, GT_camera_IDs=None,
                     ignore_distortions=False, reset_camera_params=False, print_compute_times=False,
                     time_interval=[0, -1], randomize_params=False, use_NN=False, own_camera_gaussians=False):
        if use_NN or randomize_params:
            raise NotImplementedError("use_NN / randomize_params are not part of the GPU path")
        if extrinsic_optimization_IDs is not None and optimize_trajectory is False:
            return self._sgd_extrinsic(list(extrinsic_optimization_IDs), GT_camera_IDs, lr, betas, lambda_smooth,
                                       lambda_body_length, patience, tolerance, max_iter, print_frequency,
                                       batch_size, N_sample_points, ignore_distortions, reset_camera_params,
                                       time_interval)
        if self.n_dims != 3:
            raise NotImplementedError("3D trajectories only")
        if reset_camera_params:   # :907-908, on every path (the cameras an earlier call learned are dropped)
            self.decomposed_cam_params = {k: [c.clone().detach() for c in v]
                                          for k, v in self.decomposed_cam_params_initial.items()}
        ext_ids = list(extrinsic_optimization_IDs or [])
        learn = []
        if ext_ids:
            # joint trajectory + extrinsic optimisation (:931-954): per listed camera the initial R
            # becomes axis-angle (used only by reset_camera_params), zero R / T entries of the
            # working copy become random.random()/1e6 (one draw each, the reference's order), and
            # R (3x3) and T join the trajectory in one Adam / clip_grad_norm_
            if len(ext_ids) > 2:
                raise NotImplementedError("at most 2 learnable cameras in the joint optimisation")
            for ID in ext_ids:
                if ID not in self.camera_IDs:
                    raise ValueError(f"extrinsic camera {ID!r} is not in camera_IDs {self.camera_IDs}")
                self.decomposed_cam_params_initial[ID][1] = rotation_conversion(
                    self.decomposed_cam_params_initial[ID][1], to_vector=True)
                Rp, Tp = self.decomposed_cam_params[ID][1], self.decomposed_cam_params[ID][2]
                if tuple(Rp.shape) != (3, 3):
                    raise NotImplementedError("joint optimisation learns R as a 3x3 matrix (the reference's "
                                              "decomposed parameters); an axis-angle R is not supported")
                with torch.no_grad():
                    Rp[Rp == 0] = random.random() / 10 ** 6
                    Tp[Tp == 0] = random.random() / 10 ** 6
                learn.append(self.camera_IDs.index(ID))
        a, b = time_interval
        G = self.gaussians[a:b]
        X0 = self.initial_trajectory[a:b]
        n_t = min(len(G), len(X0))
        G, X0 = G[:n_t], X0[:n_t]
        B = n_t if batch_size is None else int(batch_size)
        cams = [self.decomposed_cam_params[i] for i in self.camera_IDs]
        G = G[:, self.camera_indices] if own_camera_gaussians else G
        r = refine_trajectories(G[None], X0[None], cams, body_lengths=self.body_lengths, lr=lr, betas=betas,
                                lambda_smooth=lambda_smooth, lambda_body_length=lambda_body_length,
                                patience=patience, tolerance=tolerance, max_iter=max_iter, batch_size=B,
                                ignore_distortions=ignore_distortions, own_camera_gaussians=own_camera_gaussians,
                                device=self.device, learn_cams=learn)
        iters = int(r["iters"][0].item())
        best = r["best"][0].cpu()
        self.trajectory = r["final"][0].cpu()
        self.best_trajectory = None if torch.isnan(best).any() else best
        best_cams = {}
        if learn:
            cf, cb = r["cams_final"][0].cpu(), r["cams_best"][0].cpu()
            for li, ID in enumerate(ext_ids):
                prm = self.decomposed_cam_params[ID]
                best_cams[ID] = (cb[li, :9].reshape(3, 3).clone(), cb[li, 9:].reshape(prm[2].shape).clone())
                prm[1] = cf[li, :9].reshape(3, 3).clone()
                prm[2] = cf[li, 9:].reshape(prm[2].shape).clone()
        if self.best_trajectory is not None:
            self.best_decomposed_cam_params = {k: [p.detach().clone() for p in v]
                                               for k, v in self.decomposed_cam_params.items()}
            for ID, (bR, bT) in best_cams.items():
                self.best_decomposed_cam_params[ID][1] = bR
                self.best_decomposed_cam_params[ID][2] = bT
        names = ["total_cost", "likelihood_cost"]
        if lambda_smooth > 0:
            names.append("smoothness_cost")
        if lambda_body_length > 0:
            names.append("body_length_cost")
        bc = r["batch_costs"][0, :iters].cpu().numpy()
        im = r["iter_means"][0, :iters].cpu().numpy()
        hist = {n: [] for n in names}
        for it in range(iters):           # the reference's shared cost / running-mean list (F6)
            for n in names:
                k = COST_NAMES.index(n)
                hist[n].extend(np.float32(v) for v in bc[it, :, k])
                hist[n].append(np.float32(im[it, k]))
        self.all_costs_total = hist
        self.iterations = iters
        if print_frequency and print_frequency < 10 ** 8:
            for it in range(0, iters, print_frequency):
                print(f"Iteration {it}: " + ", ".join(f"{n}: {im[it, COST_NAMES.index(n)]:.2e}" for n in names))
        return self

    # ---- extrinsic learning from samples (pose_refinement.py:894-1096 with
    # optimize_trajectory=False): sample_gaussians (:684-706), construct_sample_cost
    # (:800-831), the Adam loop (:1000-1089).
    def sample_gaussians(self, G, GT, N):
        """:684-706 — np.random.multivariate_normal per (t, GT camera, joint) on the global numpy
        RNG, vectorised: the reference's T·2·J calls each draw N·2 standard normals in loop order
        (an even count, so the legacy Gaussian cache never carries over) and map them by its own
        svd(cov) -> x @ (sqrt(s)[:, None] * v) + mean; one standard_normal draw of the whole
        (T, 2, J, N, 2) block and the same per-matrix LAPACK SVD / BLAS products on the stacked
        covariances give bit-identical samples.  Returns (T, J, N, 2 cams, 2) float64."""
        T, J = G.shape[0], G.shape[2]
        means = G[:, GT, :, :2].numpy().astype(np.float64)
        covs = G[:, GT, :, 2:].reshape(T, 2, J, 2, 2).numpy().astype(np.float64)
        x = np.random.standard_normal((T, 2, J, N, 2))
        _, s, v = np.linalg.svd(covs)
        samples = np.matmul(x, np.sqrt(s)[..., :, None] * v) + means[..., None, :]
        return np.transpose(samples, (0, 2, 3, 1, 4))

    def _window_costs(self, G, X, B, lambda_smooth, lambda_body_length):
        """The smoothness / body-length costs of each window (:836-860) for the fixed trajectory
        X (T, J, 3): one mvp_sgd_refine launch with max_iter=0 and lr=0 (the trajectory does not
        move), its per-window cost rows.  Returns {name: [f32 per window]}."""
        cam0 = [c.detach() for c in self.decomposed_cam_params[self.camera_IDs[0]]]
        r = refine_trajectories(G[:, :1][None], X[None], [cam0], body_lengths=self.body_lengths,
                                lr=0.0, lambda_smooth=lambda_smooth, lambda_body_length=lambda_body_length,
                                patience=1, max_iter=0, batch_size=B, device=self.device)
        bc = r["batch_costs"][0, 0].cpu().numpy()
        out = {}
        if lambda_smooth > 0:
            out["smoothness_cost"] = [np.float32(v) for v in bc[:, COST_NAMES.index("smoothness_cost")]]
        if lambda_body_length > 0:
            out["body_length_cost"] = [np.float32(v) for v in bc[:, COST_NAMES.index("body_length_cost")]]
        return out

    def _sgd_extrinsic(self, ext_ids, GT, lr, betas, lambda_smooth, lambda_body_length, patience, tolerance,
                       max_iter, print_frequency, batch_size, N_sample_points, ignore_distortions,
                       reset_camera_params, time_interval):
        if self.n_dims != 3:
            raise NotImplementedError("3D trajectories only")
        a, b = time_interval
        G_sub = self.gaussians[a:b]
        n_sub = len(G_sub)
        B = n_sub if batch_size is None else int(batch_size)
        T = int(np.floor(n_sub / B) * B)
        if T != n_sub:
            # the reference's cov_invs_subset keeps all n_sub rows (:898) and its einsum fails
            raise ValueError(f"batch_size {B} must divide the {n_sub} frames of time_interval {time_interval} "
                             "when learning extrinsics from samples (the reference fails here too)")
        G = G_sub[:T]
        if reset_camera_params:
            self.decomposed_cam_params = {k: [c.clone().detach() for c in v]
                                          for k, v in self.decomposed_cam_params_initial.items()}
        if GT is None:          # the reference's branch for this iterates over None (:918-919)
            raise TypeError("GT_camera_IDs is required when learning extrinsics from samples")
        assert len(ext_ids) == 1
        assert len(GT) == 2
        assert min(i in self.decomposed_cam_params for i in GT)
        assert ext_ids[0] in self.decomposed_cam_params
        if self.n_cams <= 2:
            raise ValueError("construct_sample_cost reads camera index 2's Gaussians (:802-805): need >= 3 cameras")
        if not self.body_lengths:
            raise ValueError("body_lengths is required (create_body_length_vect, :767-779)")
        ID = ext_ids[0]
        # :935-945 — axis-angle of the initial R (not the learnable one), non-zero R / T entries
        self.decomposed_cam_params_initial[ID][1] = rotation_conversion(self.decomposed_cam_params_initial[ID][1],
                                                                        to_vector=True)
        Rp, Tp = self.decomposed_cam_params[ID][1], self.decomposed_cam_params[ID][2]
        Rp[Rp == 0] = random.random() / 10 ** 6
        Tp[Tp == 0] = random.random() / 10 ** 6
        Rp.requires_grad_(True)
        Tp.requires_grad_(True)
        learnable = [Rp, Tp]
        trajectory = self.initial_trajectory[a:b].clone().detach()
        self.trajectory = trajectory
        self.best_trajectory = None
        self.best_decomposed_cam_params = None
        n_win = (T - B) // (B // 2) + 1
        optimizer = torch.optim.Adam(learnable, lr=lr, betas=betas)

        dev = self.device
        N = int(self.N_sample_points)
        samples = self.sample_gaussians(G, GT, N)                    # (T, J, N, 2, 2) f64
        self.samples = samples
        J = G.shape[2]
        # construct_sample_cost (:808-812): utils.triangulate_points on the float64 samples with the
        # GT pair's float32 parameters — OpenCV keeps CV_64F throughout (mvp_triangulate_points_f64;
        # P = np.dot in float32 as the reference computes it), then .to(float32)
        p1, p2 = self.decomposed_cam_params[GT[0]], self.decomposed_cam_params[GT[1]]
        pair = ops.pack_cameras([[p.detach().numpy() for p in (p1[0], p1[1], p1[2], p1[3])],
                                 [p.detach().numpy() for p in (p2[0], p2[1], p2[2], p2[3])]])
        kd = torch.from_numpy(np.ascontiguousarray(samples.reshape(-1, 2, 2))).to(dev)
        samples_3d = ops.triangulate_points_f64(kd, torch.from_numpy(pair).to(dev)).to(torch.float32)
        samples_3d = samples_3d.reshape(T, J, N, 3).contiguous()
        self.samples_3d = samples_3d
        # targets: camera index 2's means (:802, hard-coded) with camera 0's Σ⁻¹ (quirk F5, :663)
        g2 = G[:, 2, :, :2].to(dev)
        cv = G[:, 0, :, 2:].to(dev)
        c00, c01, c10, c11 = cv[..., 0] + 1e-6, cv[..., 1], cv[..., 2], cv[..., 3] + 1e-6
        det = c00 * c11 - c01 * c10
        targets = torch.stack([g2[..., 0], g2[..., 1], c11 / det, -c01 / det, -c10 / det, c00 / det], -1)
        targets = targets.contiguous()
        K, dist = self.decomposed_cam_params[ID][0], self.decomposed_cam_params[ID][3]

        const = self._window_costs(G, trajectory[:T], B, lambda_smooth, lambda_body_length)
        names = ["total_cost"] + list(const.keys()) + ["extrinsic_param_sample_cost"]
        hist = {n: [] for n in names}          # all_costs and all_costs_total share these lists (F6)
        best_total = float("inf")
        no_improve = 0
        it = 0
        if self.device_adam and Rp.shape == (3, 3) and tuple(Tp.shape) in ((3, 1), (3,)):
            it, _ = self._sgd_extrinsic_device(samples_3d, targets, K, dist, Rp, Tp, const, names, hist, lr, betas,
                                               patience, tolerance, max_iter, n_win, N, ignore_distortions,
                                               trajectory, print_frequency)
            self.all_costs_total = hist
            self.iterations = it
            return self
        while no_improve < patience and it <= max_iter:
            for w in range(n_win):
                optimizer.zero_grad()
                Rm = rotation_conversion(Rp, to_vector=False)
                cam = torch.cat([K.detach().reshape(9), Rm.detach().reshape(9), Tp.detach().reshape(3),
                                 dist.detach().reshape(5)]).to(torch.float32).to(dev, non_blocking=True)
                sums = extrinsic_sample_grad(samples_3d, targets, cam, N, ignore_distortions).cpu()
                cnt = sums[1]
                ext_cost = (sums[0] / cnt).to(torch.float32)
                gR = (sums[2:11] / cnt).to(torch.float32).reshape(3, 3)
                gT = (sums[11:14] / cnt).to(torch.float32)
                # chain through the (possibly axis-angle) parameterisation exactly as autograd would
                surrogate = (Rm * gR).sum() + (Tp.reshape(3) * gT).sum()
                surrogate.backward()
                costs = {n: torch.tensor(const[n][w]) for n in const}
                costs["extrinsic_param_sample_cost"] = ext_cost
                total = torch.sum(torch.stack(list(costs.values())))
                torch.nn.utils.clip_grad_norm_(learnable, max_norm=1.0)
                optimizer.step()
                hist["total_cost"].append(np.float32(total))
                for n in costs:
                    hist[n].append(np.float32(costs[n]))
            for n in names:
                hist[n].append(np.mean(hist[n], 0))
            cur = hist["total_cost"][-1]
            if cur < best_total - tolerance:
                best_total = cur
                self.best_trajectory = trajectory.clone().detach()
                self.best_decomposed_cam_params = {k: [p.clone().detach() for p in v]
                                                   for k, v in self.decomposed_cam_params.items()}
                no_improve = 0
            else:
                no_improve += 1
            if no_improve >= patience:
                break
            if print_frequency and it % print_frequency == 0 and print_frequency < 10 ** 8:
                print(f"Iteration {it}: " + ", ".join(f"{n}: {hist[n][-1]:.2e}" for n in names))
            it += 1
        self.all_costs_total = hist
        self.iterations = it
        return self

    def _sgd_extrinsic_device(self, samples_3d, targets, K, dist, Rp, Tp, const, names, hist, lr, betas, patience,
                              tolerance, max_iter, n_win, N, ignore_distortions, trajectory, print_frequency,
                              chunk_iters=8):
        """The Adam loop of _sgd_extrinsic with every step on the device (learnable R a 3x3
        matrix, the reference's default): per window one mvp_extrinsic_sample_grad pass and one
        mvp_extrinsic_adam_step (clip + Adam, camera record updated in place) — no host round
        trip per step.  Every `chunk_iters` iterations one read-back of the per-step costs and
        parameters replays the reference's shared-list running means and early stop (F6) on the
        host; the best / final parameters are taken from the parameter history (iterations the
        device ran past the stopping point are discarded)."""
        dev = self.device
        cam = torch.cat([K.detach().reshape(9), Rp.detach().reshape(9), Tp.detach().reshape(3),
                         dist.detach().reshape(5)]).to(torch.float32).to(dev).contiguous()
        state = torch.zeros(25, dtype=torch.float32, device=dev)
        max_steps = (int(max_iter) + 1) * n_win
        cost_hist = torch.zeros(max_steps, dtype=torch.float32, device=dev)
        param_hist = torch.zeros((max_steps, 12), dtype=torch.float32, device=dev)
        n_pts = samples_3d.numel() // 3
        n_blocks = max(1, min(1024, (n_pts + 255) // 256))
        part = torch.empty((n_blocks, EXT_SUMS), dtype=torch.float64, device=dev)
        s = _stream(dev)

        def launch_step(step):
            call("mvp_extrinsic_sample_grad", _ptr(samples_3d), _ptr(targets), int(N), int(n_pts), _ptr(cam),
                 int(bool(ignore_distortions)), int(n_blocks), _ptr(part), s)
            call("mvp_extrinsic_adam_step", _ptr(part), int(n_blocks), _ptr(cam), _ptr(state), float(lr),
                 float(betas[0]), float(betas[1]), 1e-8, 1.0, _ptr(cost_hist), _ptr(param_hist), s)

        best_total = float("inf")
        no_improve = 0
        it = 0
        launched = 0          # iterations launched on the device
        done = False
        final_params = None
        while not done:
            n_new = min(chunk_iters, int(max_iter) + 1 - launched)
            for _ in range(n_new * n_win):
                launch_step(None)
            launched += n_new
            costs_h = cost_hist[:launched * n_win].cpu().numpy()
            params_h = param_hist[:launched * n_win].cpu()
            while it < launched:
                for w in range(n_win):
                    k = it * n_win + w
                    costs = {n: torch.tensor(const[n][w]) for n in const}
                    costs["extrinsic_param_sample_cost"] = torch.tensor(costs_h[k])
                    total = torch.sum(torch.stack(list(costs.values())))
                    hist["total_cost"].append(np.float32(total))
                    for n in costs:
                        hist[n].append(np.float32(costs[n]))
                for n in names:
                    hist[n].append(np.mean(hist[n], 0))
                last = params_h[(it + 1) * n_win - 1]
                final_params = last
                cur = hist["total_cost"][-1]
                if cur < best_total - tolerance:
                    best_total = cur
                    self.best_trajectory = trajectory.clone().detach()
                    self.best_decomposed_cam_params = {k2: [p.clone().detach() for p in v]
                                                       for k2, v in self.decomposed_cam_params.items()}
                    ID = [k2 for k2, v in self.decomposed_cam_params.items() if v[1] is Rp][0]
                    self.best_decomposed_cam_params[ID][1] = last[:9].reshape(3, 3).clone()
                    self.best_decomposed_cam_params[ID][2] = last[9:].reshape(Tp.shape).clone()
                    no_improve = 0
                else:
                    no_improve += 1
                if no_improve >= patience:
                    done = True
                    break
                if print_frequency and it % print_frequency == 0 and print_frequency < 10 ** 8:
                    print(f"Iteration {it}: " + ", ".join(f"{n}: {hist[n][-1]:.2e}" for n in names))
                it += 1
                if it > max_iter:
                    done = True
                    break
        with torch.no_grad():
            Rp.copy_(final_params[:9].reshape(3, 3))
            Tp.copy_(final_params[9:].reshape(Tp.shape))
        return it, final_params
