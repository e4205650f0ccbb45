"""RTMDet-m person detector on the libmvpose detector runtime (csrc/detnet.cpp, det.hip).

The reference runs mmdet's RTMDet-m (`detectors.coco_base` in
examples/model_paths.yaml:2-4: rtmdet_m_640-8xb32_coco-person.py) through
`inference_detector` on every camera-frame inside PoseEstimator.predict
(mmpose_pose_estimation.py:98-99, :234-241) and keeps the first detection with
label 0 and score > bbox_thr (:242-250).  Here, per batch of frames:

    mvp_det_letterbox   Resize(640, keep_ratio) with cv2 INTER_LINEAR semantics,
                        Pad(114), (x - mean) / std            -> bf16 NHWC, 4 channels
    CSPNeXt-m           stem (3 ConvModules), 4 stages of s2 conv + CSPLayer (CSPNeXtBlocks:
                        3x3 conv, 5x5 depthwise + 1x1; channel attention), SPP in stage 4
    CSPNeXtPAFPN        reduce 1x1s, nearest 2x, CSP layers, s2 downsamples, out 3x3s
    RTMDetSepBNHead     per level: 2 x (3x3 cls, 3x3 reg) ConvModules (shared conv weights,
                        separate BN), 1x1 rtm_cls / rtm_reg, sigmoid, exp * stride,
                        distance2bbox
    select              per frame: the highest-scoring prior over score_thr with a positive
                        rescaled width / height = the first detection after mmdet's NMS
    (optional) NMS      mmdet's full post-processing (nms_pre per level, min size, IoU 0.6,
                        max 100) -> the `inference_detector` detection list

Every ConvModule's BatchNorm is folded into the conv on the host (fp64 -> bf16 weights,
f32 biases); channel counts that are not multiples of 32 (24, 48) are zero-padded in
storage (zero weights and biases, and SiLU(0) = 0, keep the padding exactly zero).
Parameter names are mmdet's, so a local mmdet checkpoint's state dict loads as is; without
one, `random_state_dict(seed)` gives seeded activation-stable weights.
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np
import torch

from . import _lib
from ._lib import call
from .hrnet import TensorDesc, to_bf16_bits

BN_EPS = 1e-5
SIZE = 640
STRIDES = (8, 16, 32)
ARCH_P5 = ((64, 128, 3, True, False), (128, 256, 6, True, False), (256, 512, 6, True, False),
           (512, 1024, 3, False, True))
DEEPEN, WIDEN = 0.67, 0.75
NECK_OUT = 192
FEAT = 192
TEST_CFG = dict(nms_pre=1000, min_bbox_size=0, score_thr=0.05, iou_threshold=0.6, max_per_img=100)
DET_STEM, DET_CONV, DET_DW, DET_CA, DET_SPP, DET_UP2, DET_HEAD, DET_DWPW = range(8)
# stored channel counts where the fused dw5 + pw kernel runs (the 160x160 / 80x80 planes: CSPNeXt
# stages 1-2 and the last top-down block); on the 40x40 / 20x20 planes it measured slower (det.hip)
DWPW_CHANNELS = (64, 96)
ACT_NONE, ACT_RELU, ACT_SILU = 0, 1, 2


class DetView(ctypes.Structure):
    _fields_ = [("t", ctypes.c_int), ("coff", ctypes.c_int), ("c", ctypes.c_int)]


class DetOp(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("in_", DetView), ("out", DetView), ("res", DetView), ("ks", ctypes.c_int),
                ("stride", ctypes.c_int), ("act", ctypes.c_int), ("w_off", ctypes.c_int64),
                ("b_off", ctypes.c_int64), ("aux", ctypes.c_int64)]


_lib.lib.mvp_det_create.argtypes = [ctypes.POINTER(TensorDesc), ctypes.c_int, ctypes.POINTER(DetOp), ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                                    ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
_lib.lib.mvp_det_arena_bytes.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]


def pad32(c: int) -> int:
    return (c + 31) // 32 * 32


cout_pad = pad32  # detector conv weights: [pad32(cout)][kh][kw][cin] (det_cout_pad in det.h)


def rescale_size(h: int, w: int, size: int = SIZE):
    """mmcv rescale_size for scale (size, size), keep_ratio -> (new_h, new_w)."""
    s = min(size / max(h, w), size / min(h, w))
    return int(h * float(s) + 0.5), int(w * float(s) + 0.5)


def stage_plan():
    stem = int(ARCH_P5[0][0] * WIDEN // 2)
    return stem, [(int(a * WIDEN), int(b * WIDEN), max(round(n * DEEPEN), 1), add_id, spp)
                  for a, b, n, add_id, spp in ARCH_P5]


# ------------------------------------------------------------------ parameters --
def conv_modules():
    """(name, cout, cin, k, groups) of every mmdet ConvModule of RTMDet-m, mmdet naming."""
    out = []
    stem, plan = stage_plan()
    s0 = int(ARCH_P5[0][0] * WIDEN)
    out += [("backbone.stem.0", stem, 3, 3, 1), ("backbone.stem.1", stem, stem, 3, 1),
            ("backbone.stem.2", s0, stem, 3, 1)]

    def csp(p, cin, cout, nb):
        mid = cout // 2
        r = [(f"{p}.main_conv", mid, cin, 1, 1), (f"{p}.short_conv", mid, cin, 1, 1)]
        for b in range(nb):
            q = f"{p}.blocks.{b}"
            r += [(f"{q}.conv1", mid, mid, 3, 1), (f"{q}.conv2.depthwise_conv", mid, 1, 5, mid),
                  (f"{q}.conv2.pointwise_conv", mid, mid, 1, 1)]
        return r + [(f"{p}.final_conv", cout, 2 * mid, 1, 1)]

    for i, (cin, cout, nb, _, spp) in enumerate(plan):
        p = f"backbone.stage{i + 1}"
        out.append((f"{p}.0", cout, cin, 3, 1))
        j = 1
        if spp:
            out += [(f"{p}.1.conv1", cout // 2, cout, 1, 1), (f"{p}.1.conv2", cout, 2 * cout, 1, 1)]
            j = 2
        out += csp(f"{p}.{j}", cout, cout, nb)
    ch = [plan[1][1], plan[2][1], plan[3][1]]  # 192, 384, 768
    nb = 2
    for i, idx in enumerate(range(len(ch) - 1, 0, -1)):
        out.append((f"neck.reduce_layers.{i}", ch[idx - 1], ch[idx], 1, 1))
        out += csp(f"neck.top_down_blocks.{i}", ch[idx - 1] * 2, ch[idx - 1], nb)
    for idx in range(len(ch) - 1):
        out.append((f"neck.downsamples.{idx}", ch[idx], ch[idx], 3, 1))
        out += csp(f"neck.bottom_up_blocks.{idx}", ch[idx] * 2, ch[idx + 1], nb)
    for i, c in enumerate(ch):
        out.append((f"neck.out_convs.{i}", NECK_OUT, c, 3, 1))
    for lvl in range(len(STRIDES)):
        for i in range(2):
            out.append((f"bbox_head.cls_convs.{lvl}.{i}", FEAT, NECK_OUT if i == 0 else FEAT, 3, 1))
            out.append((f"bbox_head.reg_convs.{lvl}.{i}", FEAT, NECK_OUT if i == 0 else FEAT, 3, 1))
    return out


def attention_modules():
    """(name, channels) of the backbone CSPLayers' ChannelAttention."""
    _, plan = stage_plan()
    return [(f"backbone.stage{i + 1}.{2 if spp else 1}.attention", cout) for i, (_, cout, _, _, spp) in enumerate(plan)]


SILU_GAIN = 2.0     # conv weights N(0, SILU_GAIN / fan_in)
RES_GAMMA = 0.5     # last BN of each CSPNeXtBlock (its identity add would double the variance)
CA_BIAS = 2.0       # hardsigmoid(~2 + 3) ~ 0.8: the attention keeps the activations O(1)
CLS_STD = 2.0       # rtm_cls weight std x sqrt(fan_in): logits ~N(CLS_BIAS, ~1)
CLS_BIAS = -3.0
REG_BIAS = 1.0
DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def random_state_dict(seed: int = 0, calibrated: bool = True):
    """Seeded synthetic weights in mmdet naming (no network: the reference's checkpoint is a
    remote URL).  Convs N(0, SILU_GAIN / fan_in); BN gamma ~ 1, beta ~ 0.1 (the residual
    branches' last BN scaled by RES_GAMMA); channel attention fc N(0, 1 / c) with bias
    CA_BIAS; rtm_cls N(0, CLS_STD^2 / 192) with bias CLS_BIAS (mmdet's prior-probability init
    is -4.6), rtm_reg bias REG_BIAS.

    BN running statistics: with calibrated=True (default) they are the activation
    statistics of these weights on the bench's synthetic frames, as a trained network's are
    (data/rtmdet_m_bn_seed<seed>.npz, written by tools/calibrate_rtmdet.py); fixed statistics
    make the ~110 SiLU layers blow up or fade out, leaving a detector that ignores its input.
    calibrated=False: mean ~ N(0, 0.1), var ~ 1 + U(0, 0.2)."""
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for name, cout, cin, k, groups in conv_modules():
        parts = name.split(".")
        if parts[0] == "bbox_head" and parts[2] != "0":
            parts[2] = "0"  # share_conv: levels 1, 2 use level 0's conv weights
            sd[name + ".conv.weight"] = sd[".".join(parts) + ".conv.weight"].clone()
        else:
            fan_in = cin * k * k
            sd[name + ".conv.weight"] = torch.randn((cout, cin, k, k), generator=g) * math.sqrt(SILU_GAIN / fan_in)
        gain = RES_GAMMA if name.endswith("conv2.pointwise_conv") else 1.0
        sd[name + ".bn.weight"] = gain * (1.0 + 0.1 * torch.randn(cout, generator=g))
        sd[name + ".bn.bias"] = gain * 0.1 * torch.randn(cout, generator=g)
        sd[name + ".bn.running_mean"] = 0.1 * torch.randn(cout, generator=g)
        sd[name + ".bn.running_var"] = 1.0 + 0.2 * torch.rand(cout, generator=g)
        sd[name + ".bn.num_batches_tracked"] = torch.tensor(0)
    for name, c in attention_modules():
        sd[name + ".fc.weight"] = torch.randn((c, c, 1, 1), generator=g) / math.sqrt(c)
        sd[name + ".fc.bias"] = CA_BIAS + 0.5 * torch.randn(c, generator=g)
    for lvl in range(len(STRIDES)):
        sd[f"bbox_head.rtm_cls.{lvl}.weight"] = torch.randn((1, FEAT, 1, 1), generator=g) * (CLS_STD / math.sqrt(FEAT))
        sd[f"bbox_head.rtm_cls.{lvl}.bias"] = CLS_BIAS + 0.1 * torch.randn(1, generator=g)
        sd[f"bbox_head.rtm_reg.{lvl}.weight"] = torch.randn((4, FEAT, 1, 1), generator=g) * (0.3 / math.sqrt(FEAT))
        sd[f"bbox_head.rtm_reg.{lvl}.bias"] = REG_BIAS + 0.3 * torch.randn(4, generator=g)
    if calibrated:
        path = os.path.join(DATA_DIR, f"rtmdet_m_bn_seed{seed}.npz")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path}: no BN calibration for seed {seed} (tools/calibrate_rtmdet.py {seed})")
        with np.load(path) as z:
            for k in z.files:
                sd[k] = torch.from_numpy(z[k].astype(np.float32))
    return sd


def peaked_state_dict():
    """random_state_dict(0) with the classification head fitted to a peaked person score on
    rendered skeleton frames (tools/train_peaked_rtmdet.py: every BN's statistics re-calibrated
    on those frames, then the cls BN affines and rtm_cls fitted; data/rtmdet_m_peaked.npz holds
    only those tensors).  Synthetic test weights with one clear best prior per frame, as a
    trained detector has on a visible person: the detector parity test's workload."""
    sd = random_state_dict(0)
    with np.load(os.path.join(DATA_DIR, "rtmdet_m_peaked.npz")) as z:
        for k in z.files:
            sd[k] = torch.from_numpy(z[k].astype(np.float32))
    return sd


def fold(sd, name):
    """ConvModule conv (cout, cin/g, k, k) + eval BN -> (w f64 same shape, bias f64 (cout,))."""
    w = sd[name + ".conv.weight"].double().numpy()
    gamma = sd[name + ".bn.weight"].double().numpy()
    beta = sd[name + ".bn.bias"].double().numpy()
    mean = sd[name + ".bn.running_mean"].double().numpy()
    var = sd[name + ".bn.running_var"].double().numpy()
    scale = gamma / np.sqrt(var + BN_EPS)
    return w * scale[:, None, None, None], beta - mean * scale


# ------------------------------------------------------------------ graph spec --
class View:
    """Channel slice of a tensor: store channels [coff, coff + c); cmap[i] = store channel
    (relative to coff) of the i-th real (reference) channel."""

    def __init__(self, t, coff, c, cmap):
        self.t, self.coff, self.c = t, coff, c
        self.cmap = np.asarray(cmap, dtype=np.int64)

    def sub(self, lo, hi, c=None):
        """The real channels [lo, hi) as a view of their own store range."""
        m = self.cmap[lo:hi]
        base = int(m.min())
        return View(self.t, self.coff + base, c if c is not None else int(m.max()) - base + 1, m - base)

    def c_struct(self):
        return DetView(self.t, self.coff, self.c)


NONE_VIEW = DetView(-1, 0, 0)


class DetSpec:
    def __init__(self, size=SIZE, keep_f32=False, fuse_dwpw=None):
        self.size = size
        # CSPNeXtBlock conv2 as one fused op (default); MVPOSE_DET_DWPW=0 keeps the depthwise
        # output as a tensor of its own (layer-by-layer parity tests, the fused-vs-unfused test)
        self.fuse_dwpw = os.environ.get("MVPOSE_DET_DWPW", "1") != "0" if fuse_dwpw is None else bool(fuse_dwpw)
        self.f32_weights = {} if keep_f32 else None  # w_off -> unrounded conv weights (tests)
        self.tensors: list[tuple[int, int, int, int]] = []
        self.ops: list[DetOp] = []
        self.names: list[str] = []
        self._w, self._f = [], []
        self._wn = self._fn = 0
        self.macs = 0
        self.n_priors = 0
        self.level_off = [0]

    def tensor(self, h, w, c) -> int:
        self.tensors.append((h, w, c, 0))
        return len(self.tensors) - 1

    def new(self, h, w, real) -> View:
        c = pad32(real)
        return View(self.tensor(h, w, c), 0, c, np.arange(real))

    def hw(self, v: View):
        return self.tensors[v.t][:2]

    def _push_w(self, bits):
        off = self._wn
        self._w.append(bits.ravel())
        self._wn += bits.size
        return off

    def _push_f(self, a):
        a = np.asarray(a, np.float32).ravel()
        pad = (-a.size) % 4
        if pad:
            a = np.concatenate([a, np.zeros(pad, np.float32)])
        off = self._fn
        self._f.append(a)
        self._fn += a.size
        return off

    def _op(self, name, kind, x, out=None, res=None, ks=0, stride=1, act=ACT_SILU, w_off=0, b_off=0, aux=0):
        self.ops.append(DetOp(kind, x.c_struct() if isinstance(x, View) else x,
                              out.c_struct() if out is not None else NONE_VIEW,
                              res.c_struct() if res is not None else NONE_VIEW, ks, stride, act, w_off, b_off, aux))
        self.names.append(name)

    def stem(self, sd, name, x: View) -> View:
        w, b = fold(sd, name)  # (24, 3, 3, 3)
        cout = w.shape[0]
        ws = np.zeros((32, 3, 3, 4))
        ws[:cout, :, :, :3] = w.transpose(0, 2, 3, 1)
        bs = np.zeros(32)
        bs[:cout] = b
        h, ww = self.hw(x)
        out = View(self.tensor(h // 2, ww // 2, 32), 0, 32, np.arange(cout))
        self._op(name, DET_STEM, x, out, ks=3, stride=2, w_off=self._push_f(ws), b_off=self._push_f(bs))
        self.macs += (h // 2) * (ww // 2) * cout * 27
        return out

    def conv(self, sd, names, x: View, k, stride=1, out: View | None = None, res: View | None = None) -> View:
        """One conv launch for the ConvModule(s) `names` on x (several = output-concatenated
        siblings on the same input)."""
        names = [names] if isinstance(names, str) else list(names)
        folded = [fold(sd, n) for n in names]
        w = np.concatenate([f[0] for f in folded])
        b = np.concatenate([f[1] for f in folded])
        cout, cin = w.shape[:2]
        assert cin == len(x.cmap), (names, cin, len(x.cmap))
        h, ww = self.hw(x)
        ho, wo = (h + 2 * (k // 2) - k) // stride + 1, (ww + 2 * (k // 2) - k) // stride + 1
        if out is None:
            out = self.new(ho, wo, cout)
        assert len(out.cmap) == cout and self.hw(out) == (ho, wo), names
        cp = cout_pad(out.c)
        ws = np.zeros((cp, k, k, x.c))
        ws[np.ix_(out.cmap, np.arange(k), np.arange(k), x.cmap)] = w.transpose(0, 2, 3, 1)
        bs = np.zeros(cp)
        bs[out.cmap] = b
        w_off = self._push_w(to_bf16_bits(ws))
        if self.f32_weights is not None:
            self.f32_weights[w_off] = ws.astype(np.float32)
        # aux: the live couts (stored channels past the last real one have zero weights and
        # bias, so their outputs are SiLU(0) = 0 and kernels may skip them)
        self._op("+".join(names), DET_CONV, x, out, res, ks=k, stride=stride, w_off=w_off, b_off=self._push_f(bs),
                 aux=int(out.cmap.max()) + 1)
        self.macs += ho * wo * cout * cin * k * k
        return out

    def dw(self, sd, name, x: View) -> View:
        w, b = fold(sd, name)  # (c, 1, 5, 5)
        h, ww = self.hw(x)
        out = View(self.tensor(h, ww, x.c), 0, x.c, x.cmap)
        ws = np.zeros((x.c, 25))
        ws[x.cmap] = w.reshape(w.shape[0], 25)
        ws = ws.reshape(x.c // 8, 8, 25).transpose(0, 2, 1)  # [C/8][25 taps][8]: wave-uniform chunks
        bs = np.zeros(x.c)
        bs[x.cmap] = b
        self._op(name, DET_DW, x, out, ks=5, w_off=self._push_f(ws), b_off=self._push_f(bs))
        self.macs += h * ww * w.shape[0] * 25
        return out

    def dwpw(self, sd, dw_name, pw_name, x: View, out: View, res: View | None = None):
        """DepthwiseSeparableConvModule (5x5 depthwise + BN + SiLU, then 1x1 + BN + SiLU) as ONE
        op (DET_DWPW, det.hip dwpw_kernel): the depthwise output stays in LDS.  w_off: the
        depthwise f32 weights [C/8][25][8]; b_off: [depthwise bias (C) | pointwise bias (C)] f32;
        aux: the pointwise bf16 weights [C][1][1][C]."""
        wd, bd = fold(sd, dw_name)          # (c, 1, 5, 5)
        wp, bp = fold(sd, pw_name)          # (cout, c, 1, 1)
        h, ww = self.hw(x)
        C = x.c
        cout, cin = wp.shape[:2]
        assert cin == len(x.cmap) and len(out.cmap) == cout and self.hw(out) == (h, ww), (dw_name, pw_name)
        cp = cout_pad(out.c)
        assert cp == C, (dw_name, cp, C)
        wsd = np.zeros((C, 25))
        wsd[x.cmap] = wd.reshape(wd.shape[0], 25)
        wsd = wsd.reshape(C // 8, 8, 25).transpose(0, 2, 1)
        bsd = np.zeros(C)
        bsd[x.cmap] = bd
        wsp = np.zeros((cp, 1, 1, C))
        wsp[np.ix_(out.cmap, [0], [0], x.cmap)] = wp.transpose(0, 2, 3, 1)
        bsp = np.zeros(cp)
        bsp[out.cmap] = bp
        aux = self._push_w(to_bf16_bits(wsp))
        if self.f32_weights is not None:
            self.f32_weights[aux] = wsp.astype(np.float32)
        self._op(dw_name + "+" + pw_name, DET_DWPW, x, out, res, ks=5, w_off=self._push_f(wsd),
                 b_off=self._push_f(np.concatenate([bsd, bsp])), aux=aux)
        self.macs += h * ww * wd.shape[0] * 25 + h * ww * cout * cin
        return out

    def attention(self, sd, name, x: View):
        wr = sd[name + ".fc.weight"].double().numpy()[:, :, 0, 0]  # (c_out, c_in)
        br = sd[name + ".fc.bias"].double().numpy()
        wt = np.zeros((x.c, x.c))
        wt[np.ix_(x.cmap, x.cmap)] = wr.T  # W^T[k][c]
        bs = np.zeros(x.c)
        bs[x.cmap] = br
        self._op(name, DET_CA, x, w_off=self._push_f(wt), b_off=self._push_f(bs))

    def csp(self, sd, p, x: View, cout, n_blocks, add_identity, attention, out: View | None = None) -> View:
        mid = cout // 2
        pm = pad32(mid)
        h, ww = self.hw(x)
        cat = View(self.tensor(h, ww, 2 * pm), 0, 2 * pm, np.concatenate([np.arange(mid), pm + np.arange(mid)]))
        self.conv(sd, [f"{p}.main_conv", f"{p}.short_conv"], x, 1, out=cat)
        main = cat.sub(0, mid, pm)
        for b in range(n_blocks):
            q = f"{p}.blocks.{b}"
            t1 = self.conv(sd, f"{q}.conv1", main, 3)
            if self.fuse_dwpw and t1.c in DWPW_CHANNELS:
                self.dwpw(sd, f"{q}.conv2.depthwise_conv", f"{q}.conv2.pointwise_conv", t1, main,
                          res=main if add_identity else None)
                continue
            t2 = self.dw(sd, f"{q}.conv2.depthwise_conv", t1)
            self.conv(sd, f"{q}.conv2.pointwise_conv", t2, 1, out=main, res=main if add_identity else None)
        if attention:
            self.attention(sd, f"{p}.attention", cat)
        return self.conv(sd, f"{p}.final_conv", cat, 1, out=out)

    def spp(self, sd, p, x: View) -> View:
        mid = len(x.cmap) // 2
        h, ww = self.hw(x)
        buf = View(self.tensor(h, ww, 4 * mid), 0, 4 * mid, np.arange(4 * mid))
        self.conv(sd, f"{p}.conv1", x, 1, out=buf.sub(0, mid))
        self._op(p + ".poolings", DET_SPP, buf.sub(0, mid))
        return self.conv(sd, f"{p}.conv2", buf, 1)

    def up2(self, x: View, out: View):
        self._op("upsample", DET_UP2, x, out, act=ACT_NONE)

    def head_level(self, sd, lvl, x: View, stride):
        h, ww = self.hw(x)
        h1 = self.conv(sd, [f"bbox_head.cls_convs.{lvl}.0", f"bbox_head.reg_convs.{lvl}.0"], x, 3)
        h2 = View(self.tensor(h, ww, 2 * FEAT), 0, 2 * FEAT, np.arange(2 * FEAT))
        self.conv(sd, f"bbox_head.cls_convs.{lvl}.1", h1.sub(0, FEAT), 3, out=h2.sub(0, FEAT))
        self.conv(sd, f"bbox_head.reg_convs.{lvl}.1", h1.sub(FEAT, 2 * FEAT), 3, out=h2.sub(FEAT, 2 * FEAT))
        w = np.concatenate([sd[f"bbox_head.rtm_cls.{lvl}.weight"].double().numpy().reshape(1, FEAT),
                            sd[f"bbox_head.rtm_reg.{lvl}.weight"].double().numpy().reshape(4, FEAT)])
        b = np.concatenate([sd[f"bbox_head.rtm_cls.{lvl}.bias"].double().numpy(),
                            sd[f"bbox_head.rtm_reg.{lvl}.bias"].double().numpy()])
        self._op(f"bbox_head.level{lvl}", DET_HEAD, h2, ks=1, stride=stride, act=ACT_NONE, w_off=self._push_f(w),
                 b_off=self._push_f(b), aux=self.n_priors)
        self.macs += h * ww * 5 * FEAT
        self.n_priors += h * ww
        self.level_off.append(self.n_priors)

    def blobs(self):
        return np.concatenate(self._w), np.concatenate(self._f)


def build_rtmdet_m(sd, size: int = SIZE, keep_f32: bool = False) -> tuple[DetSpec, int]:
    """The RTMDet-m forward (mmdet CSPNeXt -> CSPNeXtPAFPN -> RTMDetSepBNHead) as a DetSpec."""
    g = DetSpec(size, keep_f32)
    x = View(g.tensor(size, size, 4), 0, 4, np.arange(3))
    stem, plan = stage_plan()
    x = g.stem(sd, "backbone.stem.0", x)
    x = g.conv(sd, "backbone.stem.1", x, 3)
    x = g.conv(sd, "backbone.stem.2", x, 3)
    s = size
    c3, c4 = plan[1][1], plan[2][1]  # 192, 384
    # the neck's concatenations, written by their producers: td1 = [up(reduce0(C5)) | C4]
    # at s/16, td2 = [up(reduce1) | C3] at s/8, bu1 = [down0(P3) | reduce1] at s/16,
    # bu2 = [down1(P4) | reduce0(C5)] at s/32
    td1 = View(g.tensor(s // 16, s // 16, 2 * c4), 0, 2 * c4, np.arange(2 * c4))
    td2 = View(g.tensor(s // 8, s // 8, 2 * c3), 0, 2 * c3, np.arange(2 * c3))
    bu1 = View(g.tensor(s // 16, s // 16, 2 * c3), 0, 2 * c3, np.arange(2 * c3))
    bu2 = View(g.tensor(s // 32, s // 32, 2 * c4), 0, 2 * c4, np.arange(2 * c4))
    outs = {1: td2.sub(c3, 2 * c3), 2: td1.sub(c4, 2 * c4)}
    for i, (cin, cout, nb, add_id, spp) in enumerate(plan):
        p = f"backbone.stage{i + 1}"
        x = g.conv(sd, f"{p}.0", x, 3, stride=2)
        j = 1
        if spp:
            x = g.spp(sd, f"{p}.1", x)
            j = 2
        x = g.csp(sd, f"{p}.{j}", x, cout, nb, add_id, True, out=outs.get(i))
    c5 = x
    # top-down
    g.conv(sd, "neck.reduce_layers.0", c5, 1, out=bu2.sub(c4, 2 * c4))
    g.up2(bu2.sub(c4, 2 * c4), td1.sub(0, c4))
    p4_td = g.csp(sd, "neck.top_down_blocks.0", td1, c4, 2, False, False)
    g.conv(sd, "neck.reduce_layers.1", p4_td, 1, out=bu1.sub(c3, 2 * c3))
    g.up2(bu1.sub(c3, 2 * c3), td2.sub(0, c3))
    p3 = g.csp(sd, "neck.top_down_blocks.1", td2, c3, 2, False, False)
    # bottom-up
    g.conv(sd, "neck.downsamples.0", p3, 3, stride=2, out=bu1.sub(0, c3))
    p4 = g.csp(sd, "neck.bottom_up_blocks.0", bu1, c4, 2, False, False)
    g.conv(sd, "neck.downsamples.1", p4, 3, stride=2, out=bu2.sub(0, c4))
    p5 = g.csp(sd, "neck.bottom_up_blocks.1", bu2, plan[3][1], 2, False, False)
    feats = [g.conv(sd, f"neck.out_convs.{i}", f, 3) for i, f in enumerate((p3, p4, p5))]
    for lvl, (f, st) in enumerate(zip(feats, STRIDES)):
        g.head_level(sd, lvl, f, st)
    return g, 0


# ------------------------------------------------------------------ runtime --
class RTMDetector:
    """Device-resident RTMDet-m person detector.

    detect(frames (N, H, W, 3) uint8 CUDA tensor) -> dict of device tensors:
      best (N, 6) f32 {x1, y1, x2, y2, score, prior} of the frame's top detection
      (score -1 when no prior clears score_thr), cand (N, P, 6) per-prior
      {score, x1, y1, x2, y2, logit} in network-input pixels.
    bboxes_for(best) applies the reference's hand-off rule (score > bbox_thr) -> (N, 4)
    xyxy with NaN rows for "no detection" (BatchPoseEstimator.run's whole-image fallback).
    __call__(frame) -> (M, 6) [x1, y1, x2, y2, score, label] detections of one frame after
    mmdet's NMS (the PoseEstimator(detector=...) callable contract)."""

    def __init__(self, state_dict=None, seed: int = 0, max_batch: int = 64, size: int = SIZE, device="cuda",
                 test_cfg=None):
        if state_dict is None:
            state_dict = random_state_dict(seed)
        self.size = int(size)
        self.cfg = dict(TEST_CFG, **(test_cfg or {}))
        self.spec, input_id = build_rtmdet_m(state_dict, self.size)
        w, f = self.spec.blobs()
        self.device = torch.device(device)
        self.w_dev = torch.from_numpy(w.view(np.int16).copy()).to(self.device)
        self.f_dev = torch.from_numpy(f).to(self.device)
        self.max_batch = int(max_batch)
        self.n_priors = self.spec.n_priors
        tens = (TensorDesc * len(self.spec.tensors))(*[TensorDesc(*t) for t in self.spec.tensors])
        ops = (DetOp * len(self.spec.ops))(*self.spec.ops)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            call("mvp_det_create", tens, len(self.spec.tensors), ops, len(self.spec.ops), input_id, self.size,
                 self.n_priors, ctypes.c_void_p(self.w_dev.data_ptr()), self.w_dev.numel(),
                 ctypes.c_void_p(self.f_dev.data_ptr()), self.f_dev.numel(), self.max_batch, ctypes.byref(h))
        self._h = h
        self.cand = torch.empty((self.max_batch, self.n_priors, 6), dtype=torch.float32, device=self.device)
        self.best = torch.empty((self.max_batch, 6), dtype=torch.float32, device=self.device)

    @property
    def macs_per_frame(self) -> int:
        return self.spec.macs

    @property
    def arena_bytes(self) -> int:
        b = ctypes.c_int64()
        call("mvp_det_arena_bytes", self._h, ctypes.byref(b))
        return b.value

    def scale_factors(self, h: int, w: int):
        """mmdet _bbox_post_process' 1 / scale_factor as f32 (x, y)."""
        nh, nw = rescale_size(h, w, self.size)
        return float(np.float32(1.0 / (nw / w))), float(np.float32(1.0 / (nh / h)))

    def detect(self, frames: torch.Tensor, letterboxed: torch.Tensor | None = None,
               best_out: torch.Tensor | None = None) -> dict:
        """Stream-ordered detection of up to max_batch camera-frames.  The returned 'cand' (and
        'best', unless best_out is given) are VIEWS of this detector's persistent buffers:
        the next detect() overwrites them, so clone what must outlive it.  best_out: a
        caller-owned contiguous float32 (N, 6) CUDA tensor that receives the best rows."""
        if frames.dtype != torch.uint8 or not frames.is_cuda or frames.dim() != 4 or frames.shape[3] != 3:
            raise ValueError("frames must be a (N, H, W, 3) uint8 CUDA tensor")
        frames = frames.contiguous()
        n, h, w = frames.shape[:3]
        if n > self.max_batch:
            raise ValueError(f"batch {n} > max_batch {self.max_batch}")
        cand, best = self.cand[:n], self.best[:n]
        if best_out is not None:
            if (best_out.dtype != torch.float32 or tuple(best_out.shape) != (n, 6) or not best_out.is_contiguous()
                    or not best_out.is_cuda):
                raise ValueError(f"best_out must be a contiguous float32 ({n}, 6) CUDA tensor")
            best = best_out
        if letterboxed is not None and (letterboxed.dtype != torch.bfloat16 or not letterboxed.is_cuda or
                                        not letterboxed.is_contiguous() or
                                        tuple(letterboxed.shape) != (n, self.size, self.size, 4)):
            raise ValueError(f"letterboxed must be a contiguous bfloat16 ({n}, {self.size}, {self.size}, 4) CUDA tensor")
        lb = ctypes.c_void_p(letterboxed.data_ptr()) if letterboxed is not None else None
        call("mvp_det_forward", self._h, ctypes.c_void_p(frames.data_ptr()), n, h, w,
             ctypes.c_float(self.cfg["score_thr"]), ctypes.c_void_p(cand.data_ptr()),
             ctypes.c_void_p(best.data_ptr()), lb, ctypes.c_void_p(torch.cuda.current_stream(frames.device).cuda_stream))
        return {"best": best, "cand": cand, "frame_hw": (h, w)}

    # ---- layer-by-layer access (parity tests): mvp_det_run_ops / mvp_det_tensor_copy
    def run_ops(self, frames: torch.Tensor, begin: int, end: int) -> None:
        n, h, w = frames.shape[:3]
        call("mvp_det_run_ops", self._h, ctypes.c_void_p(frames.data_ptr()), n, h, w, begin, end,
             ctypes.c_void_p(self.cand.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream))

    def folded_ops(self) -> list[int]:
        """Per op: 1 when its pass runs inside its consumer conv (mvp_det_folded_ops)."""
        out = (ctypes.c_int * len(self.spec.ops))()
        call("mvp_det_folded_ops", self._h, out, len(self.spec.ops))
        return list(out)

    def tensor(self, t: int, n: int) -> torch.Tensor:
        """Copy of arena tensor t (first n images) as (n, h, w, c) bf16."""
        h, w, c, _ = self.spec.tensors[t]
        out = torch.empty((n, h, w, c), dtype=torch.bfloat16, device=self.device)
        call("mvp_det_tensor_copy", self._h, t, n, ctypes.c_void_p(out.data_ptr()), 0,
             ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream))
        return out

    @staticmethod
    def bboxes_for(best: torch.Tensor, bbox_thr: float = 0.3) -> np.ndarray:
        """The reference's hand-off (mmpose_pose_estimation.py:242-250) on the per-frame top
        detections: (N, 4) float64 xyxy, NaN rows where the score is not above bbox_thr."""
        b = best.detach().cpu().numpy().astype(np.float64)
        out = np.full((len(b), 4), np.nan)
        ok = b[:, 4] > bbox_thr
        out[ok] = b[ok, :4]
        return out

    def nms(self, det: dict):
        """mmdet's post-processing on detect()'s candidates -> list of (M, 6) numpy
        [x1, y1, x2, y2, score, label] per frame (score-descending, label 0 = person)."""
        cand = det["cand"]
        n = cand.shape[0]
        cap = self.cfg["max_per_img"]
        dets = torch.empty((n, cap, 5), dtype=torch.float32, device=cand.device)
        counts = torch.empty((n,), dtype=torch.int32, device=cand.device)
        fx, fy = self.scale_factors(*det["frame_hw"])
        offs = (ctypes.c_int * len(self.spec.level_off))(*self.spec.level_off)
        call("mvp_det_nms", ctypes.c_void_p(cand.data_ptr()), n, self.n_priors, offs, len(self.spec.level_off) - 1,
             int(self.cfg["nms_pre"]), ctypes.c_float(self.cfg["score_thr"]), ctypes.c_float(self.cfg["iou_threshold"]),
             cap, ctypes.c_float(fx), ctypes.c_float(fy), ctypes.c_void_p(dets.data_ptr()),
             ctypes.c_void_p(counts.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream(cand.device).cuda_stream))
        d, c = dets.cpu().numpy(), counts.cpu().numpy()
        out = []
        for i in range(n):
            m = int(c[i])
            out.append(np.concatenate([d[i, :m], np.zeros((m, 1), np.float32)], 1))
        return out

    def __call__(self, frame):
        f = frame if isinstance(frame, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(frame))
        f = f.to(self.device).reshape((1,) + tuple(f.shape[-3:]))
        return self.nms(self.detect(f))[0]

    def close(self):
        if getattr(self, "_h", None):
            call("mvp_det_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
