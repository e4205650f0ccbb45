"""ORACLE (test infrastructure only) — the reference's person detector, restated.

The reference builds its detector with mmdet's `init_detector` from
`examples/model_paths.yaml:2-4` (`detectors.coco_base` =
`rtmdet_m_640-8xb32_coco-person.py` + the `rtmdet_m_8xb32-100e_coco-obj365-person`
checkpoint) and calls it once per camera-frame in `PoseEstimator.predict`
(mmpose_pose_estimation.py:98-99, :234-250):

    det_result = inference_detector(self.detector, input_file)          # :236
    pred_instance = det_result.pred_instances.cpu().numpy()             # :241
    bboxes = concat(bboxes, scores)[labels == det_cat_id & scores > bbox_thr]   # :242-244
    bboxes = bboxes[0, :4] or None                                      # :246-250

mmdet (3.x), mmcv, mmengine and cv2 are absent from this image and the checkpoint
is a remote URL, so everything below is restated from those libraries' published
algorithms and **parity is unpinned** (no fixture in the reference covers it):

* test pipeline (rtmdet_l config's `test_pipeline`, inherited by rtmdet_m / the
  person config): `Resize(scale=(640, 640), keep_ratio=True)` = mmcv
  `imrescale` (scale factor min(640/long, 640/short), size int(x*s + 0.5)) with
  cv2.resize INTER_LINEAR (`opencv_resize_linear_u8`), `Pad(size=(640, 640),
  pad_val=114)` (bottom / right), `DetDataPreprocessor(mean=[103.53, 116.28,
  123.675], std=[57.375, 57.12, 58.395], bgr_to_rgb=False)`;
* model `RTMDet` with `CSPNeXt(arch='P5', deepen_factor=0.67, widen_factor=0.75,
  expand_ratio=0.5, channel_attention=True)`, `CSPNeXtPAFPN(in_channels=[192, 384,
  768], out_channels=192, num_csp_blocks=2)`, `RTMDetSepBNHead(num_classes=1,
  in_channels=192, feat_channels=192, stacked_convs=2, share_conv=True,
  pred_kernel_size=1, exp_on_reg=True)`; every ConvModule = conv (no bias) + BN
  (SyncBN at eval = BN, eps 1e-5) + SiLU.  Module / parameter names are mmdet's,
  so an mmdet checkpoint's state dict loads as is;
* `test_cfg` of the person config: nms_pre=1000, min_bbox_size=0, score_thr=0.05,
  nms iou_threshold=0.6, max_per_img=100; post-processing = mmdet
  `BaseDenseHead._predict_by_feat_single` (sigmoid scores,
  `filter_scores_and_topk`, `MlvlPointGenerator(offset=0)` priors,
  `DistancePointBBoxCoder` / `distance2bbox` clipped to img_shape (the padded
  640x640), rescale by 1/scale_factor, min-size filter, mmcv `batched_nms`).
"""
from __future__ import annotations


import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

BN_EPS = 1e-5
MEAN = (103.53, 116.28, 123.675)
STD = (57.375, 57.12, 58.395)
PAD_VAL = 114
STRIDES = (8, 16, 32)
TEST_CFG = dict(nms_pre=1000, min_bbox_size=0, score_thr=0.05, iou_threshold=0.6, max_per_img=100)
# CSPNeXt P5 arch (in, out, blocks, add_identity, use_spp) and the rtmdet_m factors
ARCH_P5 = ((64, 128, 3, True, False), (128, 256, 6, True, False), (256, 512, 6, True, False),
           (512, 1024, 3, False, True))
DEEPEN, WIDEN = 0.67, 0.75


# ---------------------------------------------------------------- modules --
class ConvModule(nn.Module):
    """mmcv ConvModule: conv (bias=False under a norm) -> BN -> SiLU."""

    def __init__(self, cin, cout, k, stride=1, groups=1, act=True):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, k, stride, k // 2, groups=groups, bias=False)
        self.bn = nn.BatchNorm2d(cout, eps=BN_EPS)
        self.act = act

    def forward(self, x):
        x = self.bn(self.conv(x))
        return F.silu(x) if self.act else x


class DepthwiseSeparableConvModule(nn.Module):
    def __init__(self, cin, cout, k):
        super().__init__()
        self.depthwise_conv = ConvModule(cin, cin, k, groups=cin)
        self.pointwise_conv = ConvModule(cin, cout, 1)

    def forward(self, x):
        return self.pointwise_conv(self.depthwise_conv(x))


class CSPNeXtBlock(nn.Module):
    """mmdet CSPNeXtBlock (expansion 1.0 inside CSPLayer): 3x3 ConvModule, then a
    5x5 depthwise-separable ConvModule, + identity when add_identity."""

    def __init__(self, c, add_identity):
        super().__init__()
        self.conv1 = ConvModule(c, c, 3)
        self.conv2 = DepthwiseSeparableConvModule(c, c, 5)
        self.add_identity = add_identity

    def forward(self, x):
        out = self.conv2(self.conv1(x))
        return out + x if self.add_identity else out


class ChannelAttention(nn.Module):
    """x * hardsigmoid(fc(avgpool(x))), fc = 1x1 conv with bias."""

    def __init__(self, c):
        super().__init__()
        self.fc = nn.Conv2d(c, c, 1, 1, 0, bias=True)

    def forward(self, x):
        out = F.adaptive_avg_pool2d(x, 1)
        return x * F.hardsigmoid(self.fc(out))


class CSPLayer(nn.Module):
    def __init__(self, cin, cout, n_blocks, add_identity, channel_attention, expand_ratio=0.5):
        super().__init__()
        mid = int(cout * expand_ratio)
        self.main_conv = ConvModule(cin, mid, 1)
        self.short_conv = ConvModule(cin, mid, 1)
        self.final_conv = ConvModule(2 * mid, cout, 1)
        self.blocks = nn.Sequential(*[CSPNeXtBlock(mid, add_identity) for _ in range(n_blocks)])
        self.channel_attention = channel_attention
        if channel_attention:
            self.attention = ChannelAttention(2 * mid)

    def forward(self, x):
        x_short = self.short_conv(x)
        x_main = self.blocks(self.main_conv(x))
        x_final = torch.cat((x_main, x_short), 1)
        if self.channel_attention:
            x_final = self.attention(x_final)
        return self.final_conv(x_final)


class SPPBottleneck(nn.Module):
    def __init__(self, cin, cout, kernel_sizes=(5, 9, 13)):
        super().__init__()
        mid = cin // 2
        self.conv1 = ConvModule(cin, mid, 1)
        self.kernel_sizes = kernel_sizes
        self.conv2 = ConvModule(mid * (len(kernel_sizes) + 1), cout, 1)

    def forward(self, x):
        x = self.conv1(x)
        x = torch.cat([x] + [F.max_pool2d(x, k, 1, k // 2) for k in self.kernel_sizes], 1)
        return self.conv2(x)


def stage_plan():
    """[(cin, cout, n_blocks, add_identity, use_spp)] of CSPNeXt-m and its stem widths."""
    stem = int(ARCH_P5[0][0] * WIDEN // 2)
    out = []
    for cin, cout, nb, add_id, spp in ARCH_P5:
        out.append((int(cin * WIDEN), int(cout * WIDEN), max(round(nb * DEEPEN), 1), add_id, spp))
    return stem, out


class CSPNeXt(nn.Module):
    def __init__(self):
        super().__init__()
        stem, plan = stage_plan()
        self.stem = nn.Sequential(ConvModule(3, stem, 3, 2), ConvModule(stem, stem, 3),
                                  ConvModule(stem, int(ARCH_P5[0][0] * WIDEN), 3))
        for i, (cin, cout, nb, add_id, spp) in enumerate(plan):
            layers = [ConvModule(cin, cout, 3, 2)]
            if spp:
                layers.append(SPPBottleneck(cout, cout))
            layers.append(CSPLayer(cout, cout, nb, add_id, channel_attention=True))
            self.add_module(f"stage{i + 1}", nn.Sequential(*layers))

    def forward(self, x):
        x = self.stem(x)
        outs = []
        for i in range(4):
            x = getattr(self, f"stage{i + 1}")(x)
            if i >= 1:
                outs.append(x)
        return tuple(outs)


class CSPNeXtPAFPN(nn.Module):
    def __init__(self, in_channels=(192, 384, 768), out_channels=192, n_blocks=2):
        super().__init__()
        self.in_channels = in_channels
        n = len(in_channels)
        self.reduce_layers = nn.ModuleList()
        self.top_down_blocks = nn.ModuleList()
        for idx in range(n - 1, 0, -1):
            self.reduce_layers.append(ConvModule(in_channels[idx], in_channels[idx - 1], 1))
            self.top_down_blocks.append(CSPLayer(in_channels[idx - 1] * 2, in_channels[idx - 1], n_blocks, False, False))
        self.downsamples = nn.ModuleList()
        self.bottom_up_blocks = nn.ModuleList()
        for idx in range(n - 1):
            self.downsamples.append(ConvModule(in_channels[idx], in_channels[idx], 3, 2))
            self.bottom_up_blocks.append(CSPLayer(in_channels[idx] * 2, in_channels[idx + 1], n_blocks, False, False))
        self.out_convs = nn.ModuleList([ConvModule(c, out_channels, 3) for c in in_channels])

    def forward(self, inputs):
        n = len(self.in_channels)
        inner = [inputs[-1]]
        for idx in range(n - 1, 0, -1):
            high = self.reduce_layers[n - 1 - idx](inner[0])
            inner[0] = high
            up = F.interpolate(high, scale_factor=2, mode="nearest")
            inner.insert(0, self.top_down_blocks[n - 1 - idx](torch.cat([up, inputs[idx - 1]], 1)))
        outs = [inner[0]]
        for idx in range(n - 1):
            down = self.downsamples[idx](outs[-1])
            outs.append(self.bottom_up_blocks[idx](torch.cat([down, inner[idx + 1]], 1)))
        return tuple(conv(o) for conv, o in zip(self.out_convs, outs))


class RTMDetSepBNHead(nn.Module):
    """Per-level ConvModules whose conv weights are shared (share_conv) while the BNs
    are separate; 1x1 rtm_cls / rtm_reg with bias; reg = exp(.) * stride."""

    def __init__(self, num_classes=1, in_channels=192, feat_channels=192, stacked_convs=2):
        super().__init__()
        self.cls_convs, self.reg_convs = nn.ModuleList(), nn.ModuleList()
        self.rtm_cls, self.rtm_reg = nn.ModuleList(), nn.ModuleList()
        for _ in STRIDES:
            cls, reg = nn.ModuleList(), nn.ModuleList()
            for i in range(stacked_convs):
                chn = in_channels if i == 0 else feat_channels
                cls.append(ConvModule(chn, feat_channels, 3))
                reg.append(ConvModule(chn, feat_channels, 3))
            self.cls_convs.append(cls)
            self.reg_convs.append(reg)
            self.rtm_cls.append(nn.Conv2d(feat_channels, num_classes, 1))
            self.rtm_reg.append(nn.Conv2d(feat_channels, 4, 1))
        for n in range(1, len(STRIDES)):
            for i in range(stacked_convs):
                self.cls_convs[n][i].conv = self.cls_convs[0][i].conv
                self.reg_convs[n][i].conv = self.reg_convs[0][i].conv

    def forward(self, feats):
        cls_scores, bbox_preds = [], []
        for idx, (x, stride) in enumerate(zip(feats, STRIDES)):
            c, r = x, x
            for layer in self.cls_convs[idx]:
                c = layer(c)
            for layer in self.reg_convs[idx]:
                r = layer(r)
            cls_scores.append(self.rtm_cls[idx](c))
            bbox_preds.append(self.rtm_reg[idx](r).exp() * stride)
        return cls_scores, bbox_preds


class RTMDet(nn.Module):
    def __init__(self):
        super().__init__()
        self.backbone = CSPNeXt()
        self.neck = CSPNeXtPAFPN()
        self.bbox_head = RTMDetSepBNHead()

    def forward(self, x):
        return self.bbox_head(self.neck(self.backbone(x)))


def build_model(state_dict) -> RTMDet:
    m = RTMDet().eval()
    sd = {k: v for k, v in state_dict.items()}
    # share_conv: levels 1..2 alias level 0's conv weights (a checkpoint stores them per level)
    m.load_state_dict(sd, strict=False)
    missing = set(m.state_dict().keys()) - set(sd.keys())
    assert not missing, f"state dict misses {sorted(missing)[:5]}"
    return m


# ------------------------------------------------------------ preprocessing --
def rescale_size(h, w, size=640):
    """mmcv.rescale_size for scale=(size, size), keep_ratio: (new_h, new_w, factor)."""
    s = min(size / max(h, w), size / min(h, w))
    return int(h * float(s) + 0.5), int(w * float(s) + 0.5), s


def opencv_resize_linear_u8(img: np.ndarray, new_h: int, new_w: int) -> np.ndarray:
    """cv2.resize(img, (new_w, new_h), interpolation=INTER_LINEAR) for uint8 HxWxC,
    OpenCV 4.x imgproc/resize.cpp semantics:
      * an exact 2x downscale in both axes is executed as INTER_AREA's fast path:
        (a + b + c + d + 2) >> 2 over each 2x2 block;
      * otherwise fixed-point bilinear: per-axis coefficients from
        fx = (dx + 0.5) * scale - 0.5 (clamped at the borders), quantised to short
        with INTER_RESIZE_COEF_SCALE = 2048; the horizontal pass is exact int32; the
        vertical pass rounds as the SIMD kernel (VResizeLinearVec_32s8u) does:
        (((S0 >> 4) * b0 >> 16) + ((S1 >> 4) * b1 >> 16) + 2) >> 2."""
    H, W, C = img.shape
    sx, sy = W / new_w, H / new_h
    if sx == 2.0 and sy == 2.0 and H == 2 * new_h and W == 2 * new_w:
        a = img.astype(np.int32)
        s = a[0::2, 0::2] + a[0::2, 1::2] + a[1::2, 0::2] + a[1::2, 1::2]
        return ((s + 2) >> 2).astype(np.uint8)

    def coeffs(n_dst, n_src, scale):
        d = np.arange(n_dst, dtype=np.float64)
        f = ((d + 0.5) * scale - 0.5).astype(np.float32)
        s0 = np.floor(f).astype(np.int64)
        f = (f - s0).astype(np.float32)
        lo = s0 < 0
        f[lo], s0[lo] = 0, 0
        hi = s0 >= n_src - 1
        f[hi], s0[hi] = 0, n_src - 1
        c1 = np.round(f.astype(np.float64) * 2048).astype(np.int32)  # saturate_cast<short>(x*2048)
        c0 = np.round((1.0 - f).astype(np.float32).astype(np.float64) * 2048).astype(np.int32)
        s1 = np.minimum(s0 + 1, n_src - 1)
        return s0, s1, c0, c1

    x0, x1, a0, a1 = coeffs(new_w, W, np.float64(sx))
    y0, y1, b0, b1 = coeffs(new_h, H, np.float64(sy))
    src = img.astype(np.int64)
    hrow = src[:, x0, :] * a0[None, :, None] + src[:, x1, :] * a1[None, :, None]  # (H, new_w, C)
    S0 = hrow[y0] >> 4
    S1 = hrow[y1] >> 4
    v = ((S0 * b0[:, None, None]) >> 16) + ((S1 * b1[:, None, None]) >> 16)
    return np.clip((v + 2) >> 2, 0, 255).astype(np.uint8)


def letterbox(frame: np.ndarray, size: int = 640):
    """Resize(keep_ratio) + Pad(114) of the rtmdet test pipeline: (padded uint8
    (size, size, 3), (w_scale, h_scale), (new_h, new_w))."""
    H, W = frame.shape[:2]
    nh, nw, _ = rescale_size(H, W, size)
    r = opencv_resize_linear_u8(frame, nh, nw)
    out = np.full((size, size, 3), PAD_VAL, np.uint8)
    out[:nh, :nw] = r
    return out, (nw / W, nh / H), (nh, nw)


def normalize(img_u8: np.ndarray) -> torch.Tensor:
    """DetDataPreprocessor: float, (x - mean) / std per channel (no channel swap) ->
    (1, 3, H, W) f32."""
    x = torch.from_numpy(np.ascontiguousarray(img_u8)).permute(2, 0, 1).float()
    m = torch.tensor(MEAN).view(3, 1, 1)
    s = torch.tensor(STD).view(3, 1, 1)
    return ((x - m) / s)[None]


# ----------------------------------------------------------- postprocessing --
def grid_priors(h, w, stride):
    """MlvlPointGenerator(offset=0).single_level_grid_priors: (h*w, 2) f32 (x, y), row-major."""
    sx = torch.arange(w, dtype=torch.float32) * stride
    sy = torch.arange(h, dtype=torch.float32) * stride
    return torch.stack([sx.repeat(h), sy.view(-1, 1).repeat(1, w).view(-1)], 1)


def distance2bbox(points, d, max_shape):
    x1 = points[:, 0] - d[:, 0]
    y1 = points[:, 1] - d[:, 1]
    x2 = points[:, 0] + d[:, 2]
    y2 = points[:, 1] + d[:, 3]
    b = torch.stack([x1, y1, x2, y2], -1)
    b[:, 0::2].clamp_(min=0, max=max_shape[1])
    b[:, 1::2].clamp_(min=0, max=max_shape[0])
    return b


def nms(boxes, scores, thr):
    """mmcv nms (offset 0): greedy in descending score order, drop IoU > thr."""
    order = torch.sort(scores, descending=True, stable=True)[1]
    x1, y1, x2, y2 = boxes.unbind(1)
    area = (x2 - x1) * (y2 - y1)
    keep, dead = [], torch.zeros(len(boxes), dtype=torch.bool)
    for oi in order.tolist():
        if dead[oi]:
            continue
        keep.append(oi)
        xx1 = torch.maximum(x1[oi], x1)
        yy1 = torch.maximum(y1[oi], y1)
        xx2 = torch.minimum(x2[oi], x2)
        yy2 = torch.minimum(y2[oi], y2)
        inter = (xx2 - xx1).clamp(min=0) * (yy2 - yy1).clamp(min=0)
        iou = inter / (area[oi] + area - inter)
        dead |= iou > thr
    return torch.tensor(keep, dtype=torch.long)


def candidates(cls_scores, bbox_preds, size=640):
    """Every prior of the three levels, level-major / row-major: (scores (P,), boxes (P,4)
    clipped to the padded img_shape, in network-input pixels)."""
    sc, bx = [], []
    for cs, bp, s in zip(cls_scores, bbox_preds, STRIDES):
        h, w = cs.shape[-2:]
        sc.append(cs[0].permute(1, 2, 0).reshape(-1).sigmoid())
        bx.append(distance2bbox(grid_priors(h, w, s), bp[0].permute(1, 2, 0).reshape(-1, 4), (size, size)))
    return torch.cat(sc), torch.cat(bx)


def predict_by_feat(cls_scores, bbox_preds, scale_factor, size=640, cfg=TEST_CFG):
    """mmdet _predict_by_feat_single + _bbox_post_process (rescale=True, with_nms):
    -> (bboxes (M,4) f32 in frame pixels, scores (M,), labels (M,) int64), score-descending."""
    mb, ms = [], []
    for cs, bp, s in zip(cls_scores, bbox_preds, STRIDES):
        h, w = cs.shape[-2:]
        scores = cs[0].permute(1, 2, 0).reshape(-1).sigmoid()
        pred = bp[0].permute(1, 2, 0).reshape(-1, 4)
        priors = grid_priors(h, w, s)
        valid = scores > cfg["score_thr"]  # filter_scores_and_topk
        idx = torch.nonzero(valid).view(-1)
        sv = scores[idx]
        k = min(cfg["nms_pre"], len(idx))
        sv, o = sv.sort(descending=True, stable=True)
        keep = idx[o[:k]]
        mb.append(distance2bbox(priors[keep], pred[keep], (size, size)))
        ms.append(sv[:k])
    boxes, scores = torch.cat(mb), torch.cat(ms)
    boxes = boxes * torch.tensor([1 / scale_factor[0], 1 / scale_factor[1]] * 2, dtype=torch.float32)
    w, h = boxes[:, 2] - boxes[:, 0], boxes[:, 3] - boxes[:, 1]
    ok = (w > cfg["min_bbox_size"]) & (h > cfg["min_bbox_size"])
    boxes, scores = boxes[ok], scores[ok]
    labels = torch.zeros(len(scores), dtype=torch.long)
    if len(scores):
        keep = nms(boxes, scores, cfg["iou_threshold"])[:cfg["max_per_img"]]
        boxes, scores, labels = boxes[keep], scores[keep], labels[keep]
    return boxes, scores, labels


def postprocess_candidates(scores, boxes, level_off, scale_factor, cfg=TEST_CFG):
    """predict_by_feat's post-processing starting from decoded per-prior candidates
    (scores (P,), boxes (P, 4) clipped, in network-input pixels; level l = rows
    [level_off[l], level_off[l+1])) -> (bboxes, scores, labels) as predict_by_feat.
    Decoding is elementwise, so decoding before filter_scores_and_topk changes nothing."""
    scores = torch.as_tensor(scores, dtype=torch.float32)
    boxes = torch.as_tensor(boxes, dtype=torch.float32)
    mb, ms = [], []
    for lo, hi in zip(level_off[:-1], level_off[1:]):
        s = scores[lo:hi]
        idx = torch.nonzero(s > cfg["score_thr"]).view(-1)
        sv, o = s[idx].sort(descending=True, stable=True)
        k = min(cfg["nms_pre"], len(idx))
        mb.append(boxes[lo:hi][idx[o[:k]]])
        ms.append(sv[:k])
    boxes, scores = torch.cat(mb), torch.cat(ms)
    boxes = boxes * torch.tensor([1 / scale_factor[0], 1 / scale_factor[1]] * 2, dtype=torch.float32)
    w, h = boxes[:, 2] - boxes[:, 0], boxes[:, 3] - boxes[:, 1]
    ok = (w > cfg["min_bbox_size"]) & (h > cfg["min_bbox_size"])
    boxes, scores = boxes[ok], scores[ok]
    labels = torch.zeros(len(scores), dtype=torch.long)
    if len(scores):
        keep = nms(boxes, scores, cfg["iou_threshold"])[:cfg["max_per_img"]]
        boxes, scores, labels = boxes[keep], scores[keep], labels[keep]
    return boxes, scores, labels


def select_bbox(boxes, scores, labels, det_cat_id=0, bbox_thr=0.3):
    """mmpose_pose_estimation.py:242-250: first detection with the category and a score
    above bbox_thr -> (4,) f32 xyxy, or None."""
    m = (labels == det_cat_id) & (scores > bbox_thr)
    if not bool(m.any()):
        return None
    return boxes[m][0].numpy().astype(np.float32)


@torch.no_grad()
def detect(model: RTMDet, frame: np.ndarray, size: int = 640):
    """inference_detector on one frame: (bboxes, scores, labels, raw (cls_scores, bbox_preds), scale_factor)."""
    img, sf, _ = letterbox(frame, size)
    cls_scores, bbox_preds = model(normalize(img))
    b, s, l = predict_by_feat(cls_scores, bbox_preds, sf, size)
    return b, s, l, (cls_scores, bbox_preds), sf
