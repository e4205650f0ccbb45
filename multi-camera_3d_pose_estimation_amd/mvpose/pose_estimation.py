"""GPU mirror of the reference's pose_estimation.py module surface.

* ``get_pose_3D(camera_params, all_kpts_2d, world_trans_rot=None, camera_indices=None,
  ignore_nonlinear_distortions=False)`` (pose_estimation.py:11-65): one batched
  ``mvp_triangulate`` launch instead of T·J ``utils.triangulate_points`` calls;
  same selection quirks, float32 output, optional inv(R_W0) rotation.
* ``get_pose_2D(frames, model, confidence=0.5, pose_keypoints=range(17))`` (:71-151):
  the V cameras' frames of one time step -> ((17, 3, V) f32 [x, y, score], list of V
  (17, 6) heatmap Gaussians); with a GPU estimator the V frames are one batched run.
* ``load_frames(recording_paths, start_end_frames)`` (utils.py:849-909): decoded
  frame stacks, one per camera, sliced ``[start:end]`` (the default ``[0, -1]``
  drops the last frame, quirk F4).  A recording is a ``.npy`` (T, H, W, 3) uint8
  array of frames as a video decoder (BGR) returns them, an MJPEG / uncompressed AVI
  or a directory of frame<N>.jpg files (``mvpose.video``).
* ``run_pose_est`` (:157-244) and ``estimate_pose_from_video`` (:259-327): every
  frame of every camera through the batched GPU pipeline (RTMDet-m person box ->
  crop, HRNet-W32 with flip test, decode, heatmap moments), then get_pose_3D over
  ``camera_indices=[0, 1]`` as the reference hard-codes (:319).  A model name builds
  PoseEstimator(detector, pose model) from model_yaml exactly as :290-297 does.
"""
from __future__ import annotations

import os

import numpy as np
import torch
import yaml

from . import geometry, ops
from .estimator import BatchPoseEstimator
from .hrnet import N_JOINTS


def get_pose_3D(camera_params, all_kpts_2d, world_trans_rot=None, camera_indices=None,
                ignore_nonlinear_distortions=False, device=None):
    """camera_params {key: [K, R, T, dist]} (get_params_from_name order), all_kpts_2d
    (T, J, 3, V) -> (T, J, 3) float32 numpy (float64 if world_trans_rot is given)."""
    dev = torch.device(device if device is not None else "cuda")
    keys = list(camera_params.keys())
    params = {}
    for k in keys:
        K, R, T, dist = camera_params[k]
        params[k] = [K, R, T, np.asarray(dist) * 0 if ignore_nonlinear_distortions else dist]
    if camera_indices is None:
        camera_indices = keys
    positions = [keys.index(c) for c in camera_indices]
    kp = torch.as_tensor(np.ascontiguousarray(np.asarray(all_kpts_2d, dtype=np.float32)), device=dev)
    cams = torch.tensor(ops.pack_cameras(params), device=dev)
    out = ops.triangulate(kp, cams, positions, mode=ops.TRI_REFERENCE).cpu().numpy()
    if world_trans_rot is not None:
        R_W0, _ = world_trans_rot
        out = np.einsum("ij,tpj->tpi", np.linalg.inv(R_W0), out)
    return out


def get_pose_2D(frames, model, confidence=0.5, pose_keypoints=range(17)):
    """pose_estimation.py:71-151.  frames: V frames (H, W, 3) uint8 of one time step.

    model: a BatchPoseEstimator / mvpose PoseEstimator or one's bound predict (the V frames
    go through the GPU in ONE batched run, detector included), or any per-frame callable with the reference's contract
    (model(frame) -> (pred_instances, heatmaps); an onepose-style model's dict output
    with 'points' / 'confidence' is parsed as the reference does, :99-101).
    Returns (results_stacked (17, 3, V) float32, heatmaps list of V arrays).
    confidence and pose_keypoints select only the keypoints the reference DRAWS on the
    frames (:117-131, then discarded with the GUI window), so they do not change the
    output — as in the reference."""
    est = resolve_estimator(model)
    if est is not None:
        batch = np.ascontiguousarray(np.stack([np.asarray(f) for f in frames]))
        r = est.run(torch.from_numpy(batch).to(est.device).contiguous())
        pts = r["keypoints"].cpu().numpy()
        conf = r["scores"].cpu().numpy()
        heat = list(r["gaussians"].cpu().numpy())
    else:
        results = [model(frame) for frame in frames]
        if getattr(model, "__module__", "").startswith("onepose"):
            pts = [np.asarray(res["points"]) for res in results]
            conf = [np.asarray(res["confidence"]).squeeze() for res in results]
        else:
            pts = [np.asarray(res[0]["keypoints"]).squeeze() for res in results]
            conf = [np.asarray(res[0]["keypoint_scores"]).squeeze() for res in results]
        try:
            heat = [res[1] for res in results]
        except (IndexError, KeyError, TypeError):
            heat = []
    stacked = np.stack([np.concatenate((p, np.expand_dims(c, 1)), axis=1) for p, c in zip(pts, conf)], axis=2)
    return stacked, heat


def video_device():
    """Where load_frames reconstructs MPEG-4 Part 2 recordings: the GPU (split decode, frames land
    in HBM) unless MVPOSE_VIDEO_DECODE=host or no GPU is visible."""
    if os.environ.get("MVPOSE_VIDEO_DECODE", "device") == "host" or not torch.cuda.is_available():
        return None
    return torch.device("cuda", torch.cuda.current_device())


def load_frames(recording_paths, start_end_frames=(0, -1), device=None):
    """{camera: (T', H, W, 3) uint8 BGR} sliced [start:end] (utils.py:903-909 ->
    frame_generator :849-900).  A recording is a .npy stack (memory-mapped), an MPEG-4 Part 2
    ('mp4v') MP4 / AVI / raw stream, an MJPEG or uncompressed AVI, a directory of frame<N>.jpg
    files (mvpose.video), or an in-memory array / tensor; other codecs raise
    NotImplementedError (no decoder in this image).  device: mp4v recordings are then
    split-decoded onto it (host entropy decoding, GPU reconstruction) and come back as device
    tensors, bit-identical to the host decoder's frames."""
    from . import video
    if isinstance(recording_paths, (list, tuple)):
        recording_paths = dict(enumerate(recording_paths))
    if not isinstance(recording_paths, dict):
        return None
    a, b = (0, -1) if start_end_frames is None else start_end_frames
    out = {}
    for k, path in recording_paths.items():
        if isinstance(path, (np.ndarray, torch.Tensor)):  # already-decoded frames in memory
            out[k] = path[a:b]
            continue
        out[k] = video.read_recording(path, a, b, device=device)
    return out


def resolve_estimator(model):
    """The GPU estimator behind the reference's `model` argument, or None: a BatchPoseEstimator
    or mvpose PoseEstimator, or one's bound predict (what estimate_pose_from_video passes,
    `model = model_structure.predict`, pose_estimation.py:297)."""
    from .mmpose_pose_estimation import PoseEstimator
    obj = getattr(model, "__self__", model)
    return obj if isinstance(obj, (BatchPoseEstimator, PoseEstimator)) else None


def build_estimator(model, detector_model="coco_base", model_yaml="", frame_hw=(720, 1280), max_frames=256,
                    device=None):
    """The estimator estimate_pose_from_video builds for a model NAME (pose_estimation.py:
    290-297): PoseEstimator(det_cfg, det_ckpt, pose_cfg, pose_ckpt) from model_yaml's
    detectors[detector_model] and pose_estimators[model] entries — a detector always sits in
    front, as in the reference.  Checkpoints must be LOCAL files (weights_only loads);
    MVPOSE_RANDOM_WEIGHTS=1 / MVPOSE_RANDOM_DETECTOR=1 select seeded synthetic weights (the yaml
    may then be absent), MVPOSE_NO_DETECTOR=1 opts out of the detector (whole-image crops).
    An estimator object (or its bound predict) is returned as is.  frame_hw is accepted for
    compatibility: the estimator sizes itself to the first frames it sees."""
    from .mmpose_pose_estimation import PoseEstimator
    est = resolve_estimator(model)
    if est is not None:
        return est
    dev = torch.device(device if device is not None else "cuda")
    det_cfg = det_ckpt = pose_cfg = pose_ckpt = None
    if model_yaml and os.path.exists(model_yaml):
        with open(model_yaml) as f:
            paths = yaml.safe_load(f) or {}
        det_cfg, det_ckpt = paths.get("detectors", {}).get(detector_model, (None, None))
        if model not in paths.get("pose_estimators", {}) and os.environ.get("MVPOSE_RANDOM_WEIGHTS") != "1":
            raise KeyError(f"pose estimator {model!r} not in {model_yaml}'s pose_estimators")
        pose_cfg, pose_ckpt = paths.get("pose_estimators", {}).get(model, (None, None))
    elif os.environ.get("MVPOSE_RANDOM_WEIGHTS") != "1":
        raise FileNotFoundError(f"model_yaml {model_yaml!r} not found (set MVPOSE_RANDOM_WEIGHTS=1 for random "
                                "weights)")
    return PoseEstimator(det_cfg, det_ckpt, pose_cfg, pose_ckpt, device=dev, max_frames=max_frames)


class FrameStreamer:
    """Overlapped host -> GPU frame supply for recorded videos (the reference decodes and
    holds whole videos on the host, utils.py:849-909, then loops frame by frame).

    Per chunk of `batch_frames` synchronised frames: a host thread gathers the V cameras'
    frames into a PINNED staging buffer (numpy copies release the GIL), the H2D copy runs
    on a dedicated copy stream, and the estimator consumes the device buffer on the
    compute stream — so chunk i+1's gather and copy overlap chunk i's kernels.  Two pinned
    and two device buffers (each capped at `max_staging_bytes`); every hand-off is an event
    (no host synchronisation inside the loop).  With a PoseEstimator the detector runs on
    each chunk on the device and its boxes crop the frames (mmpose_pose_estimation.py:
    234-253).  Outputs accumulate on the device and come back with one copy at the end.
    Use as a context manager (or call close()) to release the gather threads."""

    def __init__(self, est, n_views: int, frame_hw, batch_frames: int = 128, gather_threads: int = 8,
                 max_staging_bytes: int = 512 << 20):
        from concurrent.futures import ThreadPoolExecutor
        self.est = est
        self.pool = ThreadPoolExecutor(max_workers=max(1, min(int(gather_threads), os.cpu_count() or 1)))
        self.V = int(n_views)
        self.H, self.W = (int(v) for v in frame_hw)
        per_frame = self.V * self.H * self.W * 3
        self.step = max(1, min(int(batch_frames), est.max_frames // self.V, int(max_staging_bytes) // per_frame))
        shape = (self.step, self.V, self.H, self.W, 3)
        self.device = est.device
        self.host = [torch.empty(shape, dtype=torch.uint8).pin_memory() for _ in range(2)]
        self.dev = [torch.empty(shape, dtype=torch.uint8, device=self.device) for _ in range(2)]
        self.copy_stream = torch.cuda.Stream(self.device)
        self.copied = [None, None]     # copy-stream event: H2D of buffer k done (host buffer reusable)
        self.consumed = [None, None]   # compute-stream event: kernels done reading device buffer k

    def close(self):
        self.pool.shutdown(wait=True)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _gather(self, stacks, t0, t1, k):
        """Chunk [t0, t1) of every camera into pinned buffer k, in pieces of 4 frames over the
        gather threads (numpy releases the GIL for the copies)."""
        h = self.host[k].numpy()
        jobs = [(v, a, min(t1, a + 4)) for v in range(self.V) for a in range(t0, t1, 4)]

        def cp(job):
            v, a, b = job
            np.copyto(h[a - t0:b - t0, v], stacks[v][a:b])
        for _ in self.pool.map(cp, jobs):
            pass

    def run(self, stacks, n_frames=None):
        """stacks: V arrays (T, H, W, 3) uint8 (memory-mapped .npy or in memory).  Returns
        device tensors kpts_2d (T, 17, 3, V) f32 and heatmaps (T, V, 17, 6) f64."""
        from concurrent.futures import ThreadPoolExecutor
        T = min(len(s) for s in stacks) if n_frames is None else int(n_frames)
        dev = self.device
        kp = torch.empty((T, N_JOINTS, 3, self.V), dtype=torch.float32, device=dev)
        hm = torch.empty((T, self.V, N_JOINTS, 6), dtype=torch.float64, device=dev)
        chunks = [(t, min(T, t + self.step)) for t in range(0, T, self.step)]
        main = torch.cuda.current_stream(dev)
        if any(isinstance(s, torch.Tensor) and s.is_cuda for s in stacks):
            # frames already in device memory (split-decoded recordings): no host staging or H2D,
            # each chunk's views interleaved (t, v)-major on the device
            dstacks = [s.to(dev) if isinstance(s, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(s)).to(dev)
                       for s in stacks]
            for t0, t1 in chunks:
                n = t1 - t0
                fr = self.dev[0][:n]
                for v, s in enumerate(dstacks):
                    fr[:, v].copy_(s[t0:t1])
                r = self.est.run(fr.reshape(n * self.V, self.H, self.W, 3), n_views=self.V, kpts_tkv=kp[t0:t1])
                hm[t0:t1] = r["gaussians"].reshape(n, self.V, N_JOINTS, 6)
            return kp, hm
        with ThreadPoolExecutor(max_workers=1) as pool:
            fut = pool.submit(self._gather, stacks, *chunks[0], 0) if chunks else None
            for i, (t0, t1) in enumerate(chunks):
                k = i & 1
                fut.result()                                   # chunk i is in pinned buffer k
                if i + 1 < len(chunks):                        # gather chunk i+1 meanwhile
                    kn = k ^ 1
                    if self.copied[kn] is not None:
                        self.copied[kn].synchronize()          # its previous H2D has left buffer kn
                    fut = pool.submit(self._gather, stacks, *chunks[i + 1], kn)
                n = t1 - t0
                with torch.cuda.stream(self.copy_stream):
                    if self.consumed[k] is not None:
                        self.copy_stream.wait_event(self.consumed[k])
                    self.dev[k][:n].copy_(self.host[k][:n], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.copy_stream)
                    self.copied[k] = ev
                main.wait_event(ev)
                fr = self.dev[k][:n].reshape(n * self.V, self.H, self.W, 3)
                r = self.est.run(fr, n_views=self.V, kpts_tkv=kp[t0:t1])
                hm[t0:t1] = r["gaussians"].reshape(n, self.V, N_JOINTS, 6)
                ce = torch.cuda.Event()
                ce.record(main)
                self.consumed[k] = ce
        return kp, hm


def run_pose_est(model, confidence=0.5, camera_indices=None, recording_paths=None, start_end_frames=(0, -1),
                 frame_shape=(1080, 1920), batch_frames=128):
    """pose_estimation.py:157-244 -> kpts_2d (T, 17, 3, V) float32, heatmaps (T, V, 17, 6)
    float64 (numpy).  recording_paths values may also be in-memory (T, H, W, 3) uint8 arrays.

    model: a PoseEstimator (detector in front) / BatchPoseEstimator or one's bound predict ->
    every frame through the batched GPU path (FrameStreamer); a model name -> build_estimator;
    any other per-frame callable with the reference's contract -> get_pose_2D frame by frame,
    as the reference loops (:184-190).  confidence does not change the output (it only
    selects what the reference draws, :117-131)."""
    gpu_model = isinstance(model, str) or resolve_estimator(model) is not None
    frames = load_frames(recording_paths, start_end_frames, device=video_device() if gpu_model else None)
    cams = list(frames.keys()) if camera_indices is None else list(camera_indices)
    stacks = [frames[c] for c in cams]
    V = len(stacks)
    H, W = stacks[0].shape[1:3]
    est = build_estimator(model, frame_hw=(H, W)) if isinstance(model, str) else resolve_estimator(model)
    if est is None:                                   # a generic per-frame callable
        stacks = [s.cpu().numpy() if isinstance(s, torch.Tensor) else s for s in stacks]
        T = min(len(s) for s in stacks)
        res = [get_pose_2D([s[t] for s in stacks], model, confidence) for t in range(T)]
        return (np.array([r[0] for r in res], dtype=np.float32).reshape(T, N_JOINTS, 3, V),
                np.array([r[1] for r in res]))
    with FrameStreamer(est, V, (H, W), batch_frames) as fs:
        kp, hm = fs.run(stacks)
    return kp.cpu().numpy(), hm.cpu().numpy()


def estimate_pose_from_video(camera_names, recording_paths, model, detector_model="coco_base", model_yaml="",
                             start_end_frames=(0, -1), confidence=0, extrinsic_params_dir="",
                             recompute_kpts_2d=True):
    """pose_estimation.py:259-327.  recompute_kpts_2d replaces the reference's interactive
    y/n prompt when kpts_2d.npy already exists (:287-289)."""
    index_name, _origin = geometry.load_camera_names(extrinsic_params_dir)
    name_index = {v: k for k, v in index_name.items()}
    camera_indices = [name_index[n] for n in camera_names]
    camera_params = {}
    for i, name in enumerate(camera_names):
        _, camera_params[i] = geometry.get_params_from_name(name, extrinsic_params_dir=extrinsic_params_dir)
    folder = os.path.dirname(recording_paths[0])
    existing = os.path.join(folder, "kpts_2d.npy")
    heatmaps = None
    if os.path.exists(existing) and not recompute_kpts_2d:
        kpts_2d = np.load(existing)
    else:
        paths = {i: recording_paths[i] for i in camera_indices}   # as :281 indexes them
        gpu_model = isinstance(model, str) or resolve_estimator(model) is not None
        frames = load_frames(paths, start_end_frames,           # decoded once (mp4v: onto the GPU)
                             device=video_device() if gpu_model else None)
        if isinstance(model, str):                             # :290-297: detector + pose model from the yaml
            model = build_estimator(model, detector_model, model_yaml,
                                    frame_hw=tuple(frames[camera_indices[0]].shape[1:3]))
        kpts_2d, heatmaps = run_pose_est(model, confidence=confidence, camera_indices=camera_indices,
                                         recording_paths=frames, start_end_frames=(0, None))
    kpts_3d = get_pose_3D(camera_params, kpts_2d, camera_indices=[0, 1])
    return kpts_2d, heatmaps, kpts_3d
