"""Batched GPU top-down 2D pose estimation (the reference's PoseEstimator.predict,
mmpose_pose_estimation.py:222-272, for all cameras x frames of a batch at once).

Per batch of N camera-frames (uint8, device-resident):
    mvp_preprocess      crop (per-crop bbox, default the whole image) + normalise, original + flipped
    mvp_graph_forward   HRNet-W32 + HeatmapHead on 2N crops (bf16 MFMA)
    mvp_heatmap_decode  flip-test average + MSRAHeatmap decode + restore
    mvp_heatmap_moments revert_heatmap + get_heatmap_means_cov
No host synchronisation inside `run`.  By default everything runs on the current
stream; with overlap_moments=True the moments kernel (whose output nothing else
on the path reads: triangulation uses the decoded keypoints) is issued on a side
stream so that it runs beside the next batch's backbone.  The flip-averaged
heatmaps it reads are double-buffered for that, and the returned
"moments_done" event orders any consumer of "gaussians" (wait_moments()).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import geometry
from ._lib import call
from .hrnet import HEATMAP_HW, INPUT_HW, N_JOINTS, HRNetBackbone

MEAN = np.array([123.675, 116.28, 103.53], np.float32)   # PoseDataPreprocessor (RGB order)
STD = np.array([58.395, 57.12, 57.375], np.float32)
COCO_FLIP_INDICES = [0, 2, 1, 4, 3, 6, 5, 8, 7, 10, 9, 12, 11, 14, 13, 16, 15]
HEATMAP_THR = 0.01  # get_heatmap_means_cov threshold (mmpose_pose_estimation.py:166)


def warp_is_separable(minv, img_h, img_w) -> bool:
    """mvp_warp_is_separable on a (6,) image -> heatmap map (enables the fast moments path)."""
    m = np.ascontiguousarray(minv, dtype=np.float64)
    out = ctypes.c_int()
    call("mvp_warp_is_separable", m.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), int(img_h), int(img_w),
         ctypes.byref(out))
    return bool(out.value)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


class BatchPoseEstimator:
    """GPU equivalent of PoseEstimator (mmpose_pose_estimation.py:81-272) from the
    person bbox on: each crop takes its bbox from `run(..., bboxes=)` (the detector's
    first person box, :242-250) or, without one, the whole image — what the reference
    falls back to when RTMDet finds no person (:246-250)."""

    def __init__(self, state_dict=None, seed: int = 0, max_frames: int = 256, frame_hw=(720, 1280),
                 flip_test: bool = True, swap_rb: bool = True, device="cuda"):
        """swap_rb: PoseDataPreprocessor(bgr_to_rgb=True) on frames as handed to the model.  The
        reference hands mmpose cvtColor(RGB2BGR) of the decoded (BGR) frame (utils.py:860/864), so
        for decoded frames the two swaps cancel: pass swap_rb=False."""
        self.device = torch.device(device)
        self.flip_test = flip_test
        self.swap_rb = bool(swap_rb)
        self.max_frames = int(max_frames)
        self.frame_h, self.frame_w = frame_hw
        self.backbone = HRNetBackbone(state_dict, seed=seed,
                                      max_batch=self.max_frames * (2 if flip_test else 1), device=device)
        geo = geometry.CropGeometry.whole_image(self.frame_w, self.frame_h)
        self.geometry = geo
        self.separable = warp_is_separable(geo.revert_minv, self.frame_h, self.frame_w)
        n = self.max_frames
        self.crop_minv = torch.tensor(np.tile(geo.crop_minv, (n, 1)), dtype=torch.float64, device=self.device)
        self.revert_minv = torch.tensor(np.tile(geo.revert_minv, (n, 1)), dtype=torch.float64, device=self.device)
        self.center_scale = torch.tensor(np.tile(geo.center_scale, (n, 1)), dtype=torch.float32, device=self.device)
        nc = n * (2 if flip_test else 1)
        self.crops = torch.empty((nc, INPUT_HW[0], INPUT_HW[1], 4), dtype=torch.bfloat16, device=self.device)
        self.heatmaps = torch.empty((nc, N_JOINTS) + HEATMAP_HW, dtype=torch.float32, device=self.device)
        # two flip-averaged heatmap buffers: decode of batch i+1 may start while the
        # side-stream moments of batch i still reads the other one
        self._avg = [torch.empty((n, N_JOINTS) + HEATMAP_HW, dtype=torch.float32, device=self.device)
                     for _ in range(2)]
        self._avg_busy = [None, None]   # side-stream event after the last moments read of each buffer
        self._avg_k = 1                 # buffer the last run wrote
        # per-crop bbox geometry (run(bboxes=...)), formed on the device by mvp_bbox_geometry and
        # double-buffered like the heatmaps: the side-stream moments of run i read revert_minv /
        # the separability flags while run i+1 writes its own.  Host boxes go up through pinned
        # staging.
        self._geo_dev = [(torch.empty((n, 6), dtype=torch.float64, device=self.device),
                          torch.empty((n, 6), dtype=torch.float64, device=self.device),
                          torch.empty((n, 4), dtype=torch.float32, device=self.device),
                          torch.empty((n,), dtype=torch.int32, device=self.device)) for _ in range(2)]
        self._box_dev = [torch.empty((n, 4), dtype=torch.float32, device=self.device) for _ in range(2)]
        self._box_host = [None, None]
        self._box_copied = [None, None]  # event after the last H2D copy out of each host buffer
        self._side = None
        self._last_revert = self.revert_minv
        self._mean = (ctypes.c_float * 3)(*MEAN)
        self._std = (ctypes.c_float * 3)(*STD)
        self._flip = (ctypes.c_int * N_JOINTS)(*COCO_FLIP_INDICES)

    @property
    def avg(self) -> torch.Tensor:
        """Flip-averaged heatmaps of the last run (valid until the run after next)."""
        return self._avg[self._avg_k]

    def _bbox_geometry(self, k: int, n: int, bboxes, bbox_thr):
        """Crop geometry of n person boxes into geometry buffer k, on the device
        (mvp_bbox_geometry): returns (crop_minv, revert_minv, center_scale, separable flags)
        device views.  bboxes: a CUDA float32 tensor (n, >=4) — e.g. RTMDetector.detect's
        per-frame best rows {x1, y1, x2, y2, score, prior}, used when score > bbox_thr — or
        host (n, 4) xyxy boxes (a row with a non-finite value = no detection = the whole
        image), uploaded through pinned staging."""
        if isinstance(bboxes, torch.Tensor) and bboxes.is_cuda:
            bx = bboxes
            if bx.dtype != torch.float32 or bx.dim() != 2 or bx.shape[1] < 4 or not bx.is_contiguous():
                raise ValueError("device bboxes must be a contiguous float32 (N, >=4) tensor")
            score_col = 4 if (bbox_thr is not None and bx.shape[1] >= 5) else -1
        else:
            bb = np.asarray(bboxes.cpu() if isinstance(bboxes, torch.Tensor) else bboxes,
                            dtype=np.float64).reshape(-1, 4).astype(np.float32)
            if self._box_host[k] is None:
                self._box_host[k] = torch.empty((self.max_frames, 4), dtype=torch.float32).pin_memory()
            if self._box_copied[k] is not None:  # the previous upload out of host buffer k is done
                self._box_copied[k].synchronize()
            if bb.shape[0] != n:
                raise ValueError(f"bboxes: {bb.shape[0]} boxes for {n} frames")
            self._box_host[k][:n].copy_(torch.from_numpy(bb))
            bx = self._box_dev[k][:n]
            bx.copy_(self._box_host[k][:n], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self._box_copied[k] = ev
            score_col = -1
        if bx.shape[0] != n:
            raise ValueError(f"bboxes: {bx.shape[0]} boxes for {n} frames")
        cm, rm, cs, sep = (t[:n] for t in self._geo_dev[k])
        call("mvp_bbox_geometry", _ptr(bx), int(bx.shape[1]), n, score_col,
             ctypes.c_float(0.0 if bbox_thr is None else float(bbox_thr)), self.frame_h, self.frame_w, _ptr(cm),
             _ptr(rm), _ptr(cs), _ptr(sep), _stream(self.device))
        return cm, rm, cs, sep

    def run(self, frames: torch.Tensor, n_views: int = 1, kpts_tkv: torch.Tensor | None = None,
            argmax: bool = False, overlap_moments: bool = False, bboxes=None, bbox_thr: float | None = None):
        """frames: (N, H, W, 3) uint8 on the GPU, ordered (t, v) when n_views > 1.
        bboxes: None (every crop = the whole image), (N, 4) host xyxy image boxes (a row of
        NaNs = no detection = the whole image), or a CUDA float32 (N, >=4) tensor such as the
        detector's per-frame best rows, whose score column 4 is held against bbox_thr — the
        reference's detector hand-off to inference_topdown (mmpose_pose_estimation.py:242-253).
        Device boxes keep the whole run free of host synchronisation.
        Returns dict: keypoints (N,17,2) f32 image px, scores (N,17) f32,
        gaussians (N,17,6) f64 [mx,my,vxx,vxy,vxy,vyy], and optionally argmax.
        overlap_moments: gaussians are produced on a side stream; read them only after
        wait_moments(out) (or a device synchronisation)."""
        if frames.dtype != torch.uint8 or not frames.is_cuda or not frames.is_contiguous():
            raise ValueError("frames must be a contiguous uint8 CUDA tensor (N, H, W, 3)")
        n, h, w, c = frames.shape
        if (h, w, c) != (self.frame_h, self.frame_w, 3):
            raise ValueError(f"frames must be (N, {self.frame_h}, {self.frame_w}, 3), got {tuple(frames.shape)}")
        if n > self.max_frames:
            raise ValueError(f"{n} frames > max_frames {self.max_frames}")
        dev, s = self.device, _stream(self.device)
        nc = n * (2 if self.flip_test else 1)
        crops = self.crops[:nc]
        k = self._avg_k ^ 1
        main = torch.cuda.current_stream(dev)
        if bboxes is None:
            crop_minv, revert_minv, center_scale = self.crop_minv, self.revert_minv, self.center_scale
            separable, sep_flags = int(self.separable), None
        else:
            if self._avg_busy[k] is not None:   # moments of two runs ago still reading geometry buffer k
                main.wait_event(self._avg_busy[k])
                self._avg_busy[k] = None
            crop_minv, revert_minv, center_scale, sep_flags = self._bbox_geometry(k, n, bboxes, bbox_thr)
            separable = 1
        call("mvp_preprocess", _ptr(frames), n, h, w, _ptr(crop_minv), INPUT_HW[0], INPUT_HW[1], self._mean,
             self._std, int(self.swap_rb), int(self.flip_test), _ptr(crops), s)
        hm = self.backbone.forward(crops, out=self.heatmaps[:nc])
        kp = torch.empty((n, N_JOINTS, 2), dtype=torch.float32, device=dev)
        sc = torch.empty((n, N_JOINTS), dtype=torch.float32, device=dev)
        am = torch.empty((n, N_JOINTS), dtype=torch.int32, device=dev) if argmax else None
        if self._avg_busy[k] is not None:       # moments of two runs ago still reading buffer k
            main.wait_event(self._avg_busy[k])
            self._avg_busy[k] = None
        self._avg_k = k
        avg = self._avg[k][:n]
        call("mvp_heatmap_decode", _ptr(hm[:n]), _ptr(hm[n:]) if self.flip_test else None, n, N_JOINTS,
             HEATMAP_HW[0], HEATMAP_HW[1], self._flip, 1, _ptr(center_scale), INPUT_HW[1], INPUT_HW[0],
             _ptr(avg), _ptr(kp), _ptr(sc), _ptr(am), _ptr(kpts_tkv), int(n_views), s)
        gauss = torch.empty((n, N_JOINTS, 6), dtype=torch.float64, device=dev)
        done = None
        if overlap_moments:
            if self._side is None:
                self._side = torch.cuda.Stream(dev)
            decoded = torch.cuda.Event()
            decoded.record(main)
            self._side.wait_event(decoded)
            ms = ctypes.c_void_p(self._side.cuda_stream)
            gauss.record_stream(self._side)
        else:
            ms = s
        call("mvp_heatmap_moments", _ptr(avg), n, N_JOINTS, HEATMAP_HW[0], HEATMAP_HW[1], _ptr(revert_minv),
             h, w, ctypes.c_float(HEATMAP_THR), separable, _ptr(sep_flags), _ptr(gauss), ms)
        if overlap_moments:
            done = torch.cuda.Event()
            done.record(self._side)
            self._avg_busy[k] = done
        self._last_revert = revert_minv
        out = {"keypoints": kp, "scores": sc, "gaussians": gauss, "heatmaps": avg, "moments_done": done}
        if argmax:
            out["argmax"] = am
        return out

    def revert_heatmaps(self, index: int = 0) -> np.ndarray:
        """The last run's flip-averaged maps of frame `index`, reverted to the image with that
        run's crop geometry (mvp_heatmap_revert): (17, H, W) f32 numpy — mmpose's
        _pred_heatmaps for that crop."""
        minv = self._last_revert[index:index + 1]
        src = self.avg[index:index + 1].contiguous()
        out = torch.empty((1, N_JOINTS, self.frame_h, self.frame_w), dtype=torch.float32, device=self.device)
        call("mvp_heatmap_revert", _ptr(src), 1, N_JOINTS, HEATMAP_HW[0], HEATMAP_HW[1], _ptr(minv), self.frame_h,
             self.frame_w, _ptr(out), _stream(self.device))
        return out[0].cpu().numpy()

    @staticmethod
    def wait_moments(out: dict) -> None:
        """Order the current stream after an overlapped run's moments (no-op otherwise)."""
        if out.get("moments_done") is not None:
            torch.cuda.current_stream().wait_event(out["moments_done"])

    # ---- the reference's per-frame callable contract (pose_estimation.py:88, :104-110)
    def predict(self, frame, return_full_heatmaps=False, bbox=None):
        """Single frame (H, W, 3) uint8 numpy/tensor -> (pred_instances, heatmaps (17,6) f64)
        with pred_instances['keypoints'] (1,17,2) f32 and ['keypoint_scores'] (1,17) f32;
        with return_full_heatmaps the maps reverted to the image, (17, H, W) f32.
        bbox: optional xyxy person box (None = the whole image)."""
        f = torch.as_tensor(np.ascontiguousarray(frame), device=self.device).reshape(1, *np.shape(frame))
        r = self.run(f.contiguous(), bboxes=None if bbox is None else [bbox])
        inst = {"keypoints": r["keypoints"].cpu().numpy(), "keypoint_scores": r["scores"].cpu().numpy()}
        if return_full_heatmaps:
            return inst, self.revert_heatmaps(0)
        return inst, r["gaussians"][0].cpu().numpy()

    __call__ = predict
