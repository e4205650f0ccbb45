"""GPU drop-in for the reference's mmpose_pose_estimation.PoseEstimator
(mmpose_pose_estimation.py:81-272): same constructor signature, the same per-frame
callable contract `model(frame) -> (pred_instances, heatmaps)` that get_pose_2D uses
(pose_estimation.py:88, :104-110), plus a batched form.

Behind it: BatchPoseEstimator (crop + normalise, HRNet-W32 bf16 with flip test,
MSRA decode, revert + heatmap moments, all HIP kernels in libmvpose.so).

* pose_checkpoint: a LOCAL mmpose HRNet-W32 checkpoint (.pth, loaded with
  torch.load(weights_only=True); its 'state_dict' if present).  The reference's
  model_paths.yaml holds download URLs; there is no network here, so a URL or a
  missing file raises, unless MVPOSE_RANDOM_WEIGHTS=1 selects seeded random weights.
* The person detector (RTMDet-m through mmdet's inference_detector, :234-241) is
  mvpose.rtmdet.RTMDetector (HIP, libmvpose): built from det_checkpoint when that is a
  LOCAL mmdet checkpoint (.pth, weights_only load), or with seeded synthetic weights
  under MVPOSE_RANDOM_DETECTOR=1; any other det_checkpoint raises FileNotFoundError
  (the reference always builds its detector, :98-99) — whole-image crops only by an
  explicit using_detector=False or MVPOSE_NO_DETECTOR=1.  `detector=` also takes any callable
  frame -> detections (M, 6) [x1, y1, x2, y2, score, label] (mmdet pred_instances'
  bboxes | scores | labels).  The reference's selection rule then applies (first box
  with label == det_cat_id and score > bbox_thr, :242-250); with an RTMDetector the
  batched path takes it on the device (the per-frame argmax = the first detection after
  NMS) and mvp_bbox_geometry turns it into the crop geometry there, so a batch never
  synchronises with the host.  When no box passes, the crop is the whole image, the
  reference's own fallback.
* device: the model runs on the GPU whatever is passed (the reference's default
  'cpu' is accepted); there is no CPU path.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .estimator import BatchPoseEstimator


def select_person_bbox(detections, det_cat_id=0, bbox_thr=0.3):
    """The reference's detector hand-off (mmpose_pose_estimation.py:242-250): the first
    detection with label == det_cat_id and score > bbox_thr, as xyxy, or None."""
    if detections is None:
        return None
    d = np.asarray(detections, dtype=np.float64).reshape(-1, 6)
    keep = d[(d[:, 5] == det_cat_id) & (d[:, 4] > bbox_thr)]
    return keep[0, :4].astype(np.float32) if len(keep) else None


def build_detector(det_checkpoint, device="cuda", max_batch=64, seed=0):
    """RTMDetector for the reference's det_checkpoint (model_paths.yaml's detectors entry, which
    PoseEstimator always builds, mmpose_pose_estimation.py:98-99): a LOCAL mmdet RTMDet-m
    checkpoint (safe loader, its 'state_dict' if present), or seeded synthetic weights under
    MVPOSE_RANDOM_DETECTOR=1.  Anything else (a download URL, a missing file) raises
    FileNotFoundError, like a missing pose checkpoint — whole-image crops are an explicit
    choice (using_detector=False, or MVPOSE_NO_DETECTOR=1), never a silent fallback."""
    from .rtmdet import RTMDetector
    if det_checkpoint and os.path.exists(str(det_checkpoint)):
        blob = torch.load(det_checkpoint, map_location="cpu", weights_only=True)
        return RTMDetector(blob.get("state_dict", blob), max_batch=max_batch, device=device)
    if os.environ.get("MVPOSE_RANDOM_DETECTOR") == "1":
        return RTMDetector(seed=seed, max_batch=max_batch, device=device)
    raise FileNotFoundError(f"detector checkpoint {det_checkpoint!r} is not a local file (no network here): pass "
                            "a local mmdet RTMDet-m .pth, set MVPOSE_RANDOM_DETECTOR=1 for synthetic detector "
                            "weights, or opt out of the detector (using_detector=False / MVPOSE_NO_DETECTOR=1)")


def load_pose_checkpoint(pose_checkpoint):
    """State dict of a local mmpose HRNet-W32 checkpoint (safe loader), or None for
    MVPOSE_RANDOM_WEIGHTS=1 (seeded random weights)."""
    if os.environ.get("MVPOSE_RANDOM_WEIGHTS") == "1":
        return None
    if not pose_checkpoint or not os.path.exists(str(pose_checkpoint)):
        raise FileNotFoundError(f"pose checkpoint {pose_checkpoint!r} is not a local file (no network here; "
                                "set MVPOSE_RANDOM_WEIGHTS=1 for random weights)")
    blob = torch.load(pose_checkpoint, map_location="cpu", weights_only=True)
    return blob.get("state_dict", blob)


class PoseEstimator:
    """mmpose_pose_estimation.PoseEstimator on the GPU (constructor :82-113)."""

    def __init__(self, det_config, det_checkpoint, pose_config, pose_checkpoint, device="cpu", det_cat_id=0,
                 bbox_thr=0.3, nms_thr=0.3, using_detector=True, *, detector=None, max_frames=256,
                 state_dict=None, seed=0, swap_rb=False):
        """swap_rb=False: frames arrive as the reference hands them to mmpose (cvtColor(RGB2BGR)
        of decoded BGR video frames, utils.py:860/864 — so the data preprocessor's bgr_to_rgb
        flip and that swap cancel, as BatchPoseEstimator documents)."""
        self.det_config, self.det_checkpoint = det_config, det_checkpoint
        self.pose_config, self.pose_checkpoint = pose_config, pose_checkpoint
        self.device = torch.device("cuda" if str(device).startswith("cpu") else device)
        self.det_cat_id = det_cat_id
        self.bbox_thr = bbox_thr
        self.nms_thr = nms_thr
        if using_detector and detector is None and os.environ.get("MVPOSE_NO_DETECTOR") == "1":
            using_detector = False
        self.using_detector = using_detector
        if detector is None and using_detector:
            detector = build_detector(det_checkpoint, self.device)
        self.detector = detector if using_detector else None
        self._state_dict = state_dict if state_dict is not None else load_pose_checkpoint(pose_checkpoint)
        self._seed = seed
        self._swap_rb = swap_rb
        self._max_frames = int(max_frames)
        self._est = None
        self._best = None   # device (max_frames, 6) per-frame best detections (RTMDetector path)

    # ---- the batched GPU estimator, built for the first frame size seen
    def estimator(self, frame_hw) -> BatchPoseEstimator:
        hw = tuple(int(v) for v in frame_hw)
        if self._est is None or (self._est.frame_h, self._est.frame_w) != hw:
            self._est = BatchPoseEstimator(self._state_dict, seed=self._seed, max_frames=self._max_frames,
                                           frame_hw=hw, swap_rb=self._swap_rb, device=self.device)
        return self._est

    @property
    def max_frames(self) -> int:
        return self._max_frames

    def bboxes_for(self, frames):
        """Per-frame person boxes for BatchPoseEstimator.run(bboxes=...).

        RTMDetector: the detector's per-frame best rows as a DEVICE tensor (N, 6) {x1, y1, x2,
        y2, score, prior} (score > bbox_thr is applied on the device by mvp_bbox_geometry: no
        host synchronisation).  With det_cat_id != 0 no RTMDet-m (person-only) box qualifies:
        NaN rows.  Any other detector callable: per frame, its (M, 6) detections
        through the reference's rule (select_person_bbox) -> host (N, 4), NaN rows = none."""
        from .rtmdet import RTMDetector
        if isinstance(self.detector, RTMDetector) and self.det_cat_id == 0:
            f = frames if isinstance(frames, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(frames))
            f = f.to(self.device).contiguous()
            n = f.shape[0]
            if self._best is None or self._best.shape[0] < n:
                self._best = torch.empty((max(n, self._max_frames), 6), dtype=torch.float32, device=self.device)
            mb = self.detector.max_batch
            for i in range(0, n, mb):
                self.detector.detect(f[i:i + mb], best_out=self._best[i:min(n, i + mb)])
            return self._best[:n]
        out = np.full((len(frames), 4), np.nan)
        if isinstance(frames, torch.Tensor):
            frames = frames.cpu().numpy()
        if self.detector is not None and not isinstance(self.detector, RTMDetector):
            for i, f in enumerate(frames):
                b = select_person_bbox(self.detector(f), self.det_cat_id, self.bbox_thr)
                if b is not None:
                    out[i] = b
        return out

    def run(self, frames: torch.Tensor, n_views: int = 1, kpts_tkv: torch.Tensor | None = None,
            overlap_moments: bool = False, argmax: bool = False, bboxes=None) -> dict:
        """Batched predict on device-resident frames (N, H, W, 3) uint8 ordered (t, v): the
        detector (when enabled) and the reference's hand-off on every camera-frame, then
        BatchPoseEstimator.run with those boxes; stream-ordered, no host synchronisation on
        the RTMDetector path.  bboxes overrides the detector."""
        est = self.estimator(frames.shape[1:3])
        if bboxes is None and self.detector is not None:
            bboxes = self.bboxes_for(frames)
        thr = self.bbox_thr if isinstance(bboxes, torch.Tensor) and bboxes.is_cuda else None
        return est.run(frames, n_views=n_views, kpts_tkv=kpts_tkv, overlap_moments=overlap_moments, argmax=argmax,
                       bboxes=bboxes, bbox_thr=thr)

    def predict_batch(self, frames, bboxes=None, overlap_moments=False):
        """frames (N, H, W, 3) uint8 (numpy or a CUDA tensor) -> BatchPoseEstimator.run's dict
        (device tensors: keypoints (N,17,2), scores (N,17), gaussians (N,17,6) f64, ...)."""
        f = frames if isinstance(frames, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(frames))
        f = f.to(self.device, non_blocking=True).contiguous()
        return self.run(f, bboxes=bboxes, overlap_moments=overlap_moments)

    def predict(self, input_file, return_full_heatmaps=False):
        """(pred_instances, heatmaps) for one frame (:222-272): pred_instances['keypoints']
        (1,17,2) f32 and ['keypoint_scores'] (1,17) f32; heatmaps = get_heatmap_means_cov
        (17,6) f64, or with return_full_heatmaps the flip-averaged 64x48 maps reverted to
        the image, (17, H, W) f32 (mmpose merge_data_samples' revert_heatmap)."""
        frame = np.asarray(input_file)
        f = torch.from_numpy(np.ascontiguousarray(frame)).to(self.device).reshape(1, *frame.shape)
        r = self.run(f)
        inst = {"keypoints": r["keypoints"].cpu().numpy(), "keypoint_scores": r["scores"].cpu().numpy()}
        if return_full_heatmaps:
            return inst, self._est.revert_heatmaps(0)
        return inst, r["gaussians"][0].cpu().numpy()

    __call__ = predict

    @staticmethod
    def get_heatmap_means_cov(heatmaps):
        """get_heatmap_means_cov (mmpose_pose_estimation.py:163-215) for full-image heatmaps
        (17, H, W) (or a list of them): h[h < 0.01] = 0, normalised mean / covariance per
        joint, zero-sum -> zeros.  Like the reference it zeroes the caller's array in place.
        (The hot path never materialises these maps: mvp_heatmap_moments fuses the revert
        and the moments.)  float32 on the GPU, the reference's dtype."""
        if isinstance(heatmaps, list):
            return np.array([PoseEstimator.get_heatmap_means_cov(h) for h in heatmaps])
        heatmaps[heatmaps < 0.01] = 0
        h = torch.as_tensor(np.asarray(heatmaps), dtype=torch.float32, device="cuda")
        K, H, W = h.shape
        ys = torch.arange(H, device=h.device, dtype=torch.float32).view(1, H, 1)
        xs = torch.arange(W, device=h.device, dtype=torch.float32).view(1, 1, W)
        s = h.sum(dim=(1, 2))
        p = h / torch.where(s == 0, torch.ones_like(s), s).view(K, 1, 1)
        mx = (xs * p).sum(dim=(1, 2))
        my = (ys * p).sum(dim=(1, 2))
        dx, dy = xs - mx.view(K, 1, 1), ys - my.view(K, 1, 1)
        vx = (dx ** 2 * p).sum(dim=(1, 2))
        vy = (dy ** 2 * p).sum(dim=(1, 2))
        cxy = (dx * dy * p).sum(dim=(1, 2))
        out = torch.stack([mx, my, vx, cxy, cxy, vy], 1).double().cpu().numpy()
        out[(s == 0).cpu().numpy()] = 0.0
        return out
