"""HRNet-W32 (COCO, 256x192) as a static op graph for the libmvpose backbone runtime.

The reference runs this network inside mmpose's inference_topdown
(mmpose_pose_estimation.py:253, config td-hm_hrnet-w32_8xb64-210e_coco-256x192,
built at pose_estimation.py:290-297) on the CPU at batch 1.  Here the host
walks the same topology (mmpose HRNet: stem, layer1 Bottlenecks, transitions,
HRModules with BasicBlock branches and multi-scale fuse layers, HeatmapHead),
folds every BatchNorm into its conv (fp64, then bf16 weights / f32 biases),
packs all weights into two device blobs and hands the graph to
mvp_graph_create.  Parameter names are mmpose's, so a converted mmpose
checkpoint (state dict) loads directly; without network access the bench uses
`random_state_dict(seed)` (He-normal convs, randomised BN statistics).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib
from ._lib import call

BN_EPS = 1e-5
STAGES = ((1, (32, 64)), (4, (32, 64, 128)), (3, (32, 64, 128, 256)))
N_JOINTS = 17
INPUT_HW = (256, 192)
HEATMAP_HW = (64, 48)
DT_BF16, DT_F32 = 0, 1
OP_STEM, OP_CONV, OP_FUSE = 0, 1, 2


class TensorDesc(ctypes.Structure):
    _fields_ = [("h", ctypes.c_int), ("w", ctypes.c_int), ("c", ctypes.c_int), ("dtype", ctypes.c_int)]


class OpDesc(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("out", ctypes.c_int), ("n_in", ctypes.c_int),
                ("in_", ctypes.c_int * 4), ("up", ctypes.c_int * 4), ("cin", ctypes.c_int),
                ("cout", ctypes.c_int), ("ks", ctypes.c_int), ("stride", ctypes.c_int), ("relu", ctypes.c_int),
                ("segment", ctypes.c_int), ("w_off", ctypes.c_int64), ("b_off", ctypes.c_int64)]


_lib.lib.mvp_graph_create.argtypes = [ctypes.POINTER(TensorDesc), ctypes.c_int, ctypes.POINTER(OpDesc), ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_void_p)]

# Micro-batch (crops) per graph segment: keeps a chain's intermediates inside the
# 256 MiB Infinity Cache (MI355X_MICROARCH.md) instead of round-tripping HBM.
#   stem    : stem + layer1 + transition1 (256-ch 64x48 tensors, 1.5 MB / crop)
#   branch0 : each HRModule's 4 BasicBlocks on the 64x48x32 branch
#   branch1 : same on the 32x24x64 branch
# 0 = whole batch.  Override: MVPOSE_MICRO_BATCH="stem:64,branch0:256,branch1:0".
DEFAULT_MICRO_BATCH = {"stem": 0, "branch0": 0, "branch1": 0}  # measured: no gain yet


def micro_batch_config():
    cfg = dict(DEFAULT_MICRO_BATCH)
    env = os.environ.get("MVPOSE_MICRO_BATCH", "")
    for item in filter(None, env.split(",")):
        k, v = item.split(":")
        cfg[k.strip()] = int(v)
    return cfg


_lib.lib.mvp_graph_arena_bytes.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]


def cout_pad(c: int) -> int:
    return 32 if c <= 32 else (c + 63) // 64 * 64


# ------------------------------------------------------------------ weights --
def _conv_shapes():
    """(conv_key, bn_key or None, cout, cin, k) for every conv, mmpose naming."""
    out = [("backbone.conv1", "backbone.bn1", 64, 3, 3), ("backbone.conv2", "backbone.bn2", 64, 64, 3)]
    cin = 64
    for b in range(4):
        p = f"backbone.layer1.{b}"
        out += [(f"{p}.conv1", f"{p}.bn1", 64, cin, 1), (f"{p}.conv2", f"{p}.bn2", 64, 64, 3),
                (f"{p}.conv3", f"{p}.bn3", 256, 64, 1)]
        if b == 0:
            out.append((f"{p}.downsample.0", f"{p}.downsample.1", 256, cin, 1))
        cin = 256
    pre = [256]
    for s, (n_mod, chans) in enumerate(STAGES):
        for i, c in enumerate(chans):
            if i < len(pre):
                if c != pre[i]:
                    out.append((f"backbone.transition{s + 1}.{i}.0", f"backbone.transition{s + 1}.{i}.1", c, pre[i], 3))
            else:
                out.append((f"backbone.transition{s + 1}.{i}.0.0", f"backbone.transition{s + 1}.{i}.0.1", c, pre[-1], 3))
        for m in range(n_mod):
            p = f"backbone.stage{s + 2}.{m}"
            for bi, c in enumerate(chans):
                for k in range(4):
                    q = f"{p}.branches.{bi}.{k}"
                    out += [(f"{q}.conv1", f"{q}.bn1", c, c, 3), (f"{q}.conv2", f"{q}.bn2", c, c, 3)]
            last = s == len(STAGES) - 1 and m == n_mod - 1
            n_out = 1 if last else len(chans)
            for i in range(n_out):
                for j in range(len(chans)):
                    if j > i:
                        out.append((f"{p}.fuse_layers.{i}.{j}.0", f"{p}.fuse_layers.{i}.{j}.1", chans[i], chans[j], 1))
                    elif j < i:
                        for k in range(i - j):
                            co = chans[i] if k == i - j - 1 else chans[j]
                            out.append((f"{p}.fuse_layers.{i}.{j}.{k}.0", f"{p}.fuse_layers.{i}.{j}.{k}.1", co,
                                        chans[j], 3))
        pre = list(chans)
    out.append(("head.final_layer", None, N_JOINTS, 32, 1))
    return out


RES_GAMMA = 0.25    # last BN of every residual branch (BasicBlock bn2, Bottleneck bn3)
FUSE_GAMMA = 0.5    # BNs of the HRModule fuse layers
HEAD_STD = 0.005    # head weight std relative to He-normal; bias ~ HEAD_BIAS + N(0, 0.01)
HEAD_BIAS = -0.15


def random_state_dict(seed: int = 0, stable: bool = True):
    """Seeded weights in mmpose naming: He-normal convs, BN with randomised affine
    and running statistics (so folding is exercised).

    stable=True (default) keeps the activations O(1) through the ~90 layers the way a
    trained network does: the residual branches' last BN and the fuse-layer BNs get
    scaled-down gammas (RES_GAMMA, FUSE_GAMMA; otherwise every residual add and every
    multi-branch fuse sum doubles the variance and the heatmaps reach ~1e8), and the head
    is scaled and biased (HEAD_STD, HEAD_BIAS) so the heatmaps are trained-model-like: O(0.1)
    values, a few per cent of cells above get_heatmap_means_cov's 0.01 threshold.
    stable=False: the round-1 weights (plain He-normal, gamma ~ 1, head bias ~ N(0, 0.1))."""
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for conv, bn, cout, cin, k in _conv_shapes():
        std = (2.0 / (cin * k * k)) ** 0.5
        if bn is None and stable:
            std *= HEAD_STD
        sd[conv + ".weight"] = torch.randn((cout, cin, k, k), generator=g) * std
        if bn is None:
            b = torch.randn((cout,), generator=g)
            sd[conv + ".bias"] = HEAD_BIAS + 0.01 * b if stable else 0.1 * b
        else:
            gain = 1.0
            if stable and (bn.endswith(".bn3") or (".branches." in bn and bn.endswith(".bn2"))):
                gain = RES_GAMMA
            elif stable and ".fuse_layers." in bn:
                gain = FUSE_GAMMA
            sd[bn + ".weight"] = gain * (1.0 + 0.1 * torch.randn((cout,), generator=g))
            sd[bn + ".bias"] = gain * 0.1 * torch.randn((cout,), generator=g)
            sd[bn + ".running_mean"] = 0.1 * torch.randn((cout,), generator=g)
            sd[bn + ".running_var"] = 1.0 + 0.2 * torch.rand((cout,), generator=g)
            sd[bn + ".num_batches_tracked"] = torch.tensor(0)
    return sd


PEAKED_BASE_SEED = 21
PEAKED_WEIGHTS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "hrnet_w32_peaked.npz")


def peaked_state_dict():
    """random_state_dict(PEAKED_BASE_SEED) with the last stage-4 module's high-resolution branch,
    its fuse projections and the HeatmapHead replaced by tensors fitted on rendered skeleton
    frames (tools/train_peaked_hrnet.py; data/hrnet_w32_peaked.npz, loaded without pickle):
    heatmaps with one clear, trained-model-like peak per joint on
    synthetic.make_skeleton_frames inputs, for parity tests that must not sit on near-ties."""
    sd = random_state_dict(PEAKED_BASE_SEED)
    with np.load(PEAKED_WEIGHTS, allow_pickle=False) as z:
        for k in z.files:
            if k not in sd or tuple(sd[k].shape) != z[k].shape:
                raise ValueError(f"{PEAKED_WEIGHTS}: unexpected tensor {k} {z[k].shape}")
            sd[k] = torch.from_numpy(z[k].copy())
    return sd


def fold_bn(sd, conv, bn):
    """conv weight (cout,cin,k,k) + eval BatchNorm -> (w (cout,k,k,cin) f64, b (cout,) f64)."""
    w = sd[conv + ".weight"].double().numpy()
    if bn is None:
        scale = np.ones(w.shape[0])
        shift = sd[conv + ".bias"].double().numpy()
    else:
        gamma = sd[bn + ".weight"].double().numpy()
        beta = sd[bn + ".bias"].double().numpy()
        mean = sd[bn + ".running_mean"].double().numpy()
        var = sd[bn + ".running_var"].double().numpy()
        scale = gamma / np.sqrt(var + BN_EPS)
        shift = beta - mean * scale
    w = w * scale[:, None, None, None]
    return np.ascontiguousarray(w.transpose(0, 2, 3, 1)), shift


def to_bf16_bits(a: np.ndarray) -> np.ndarray:
    """fp64/fp32 -> bf16 bit patterns, round to nearest even."""
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)


# ------------------------------------------------------------------ graph --
class GraphSpec:
    """Host-side description: tensors, ops, weight blobs (numpy)."""

    def __init__(self):
        self.tensors: list[tuple[int, int, int, int]] = []
        self.ops: list[dict] = []
        self.seg_micro_batch: list[int] = [0]
        self._seg = 0
        self._w: list[np.ndarray] = []
        self._f: list[np.ndarray] = []
        self._w_len = 0
        self._f_len = 0

    def segment(self, micro_batch: int = 0) -> None:
        """Start a new segment (contiguous ops run in micro-batches of `micro_batch` crops)."""
        if self.ops and self.ops[-1]["segment"] == self._seg:
            self.seg_micro_batch.append(int(micro_batch))
            self._seg += 1
        else:
            self.seg_micro_batch[self._seg] = int(micro_batch)

    def tensor(self, h, w, c, dtype=DT_BF16) -> int:
        self.tensors.append((h, w, c, dtype))
        return len(self.tensors) - 1

    def _push_w(self, a_bits: np.ndarray) -> int:
        off = self._w_len
        self._w.append(a_bits.ravel())
        self._w_len += a_bits.size
        return off

    def _push_f(self, a: np.ndarray) -> int:
        off = self._f_len
        a = np.asarray(a, np.float32).ravel()
        pad = (-a.size) % 4
        if pad:
            a = np.concatenate([a, np.zeros(pad, np.float32)])
        self._f.append(a)
        self._f_len += a.size
        return off

    def stem(self, sd, conv, bn, x) -> int:
        w, b = fold_bn(sd, conv, bn)  # (64, 3, 3, 3)
        w4 = np.zeros((64, 3, 3, 4))
        w4[..., :3] = w
        h, ww, _, _ = self.tensors[x]
        y = self.tensor((h - 1) // 2 + 1, (ww - 1) // 2 + 1, 64)
        self.ops.append(dict(kind=OP_STEM, segment=self._seg, out=y, ins=[x], up=[1], cin=4, cout=64, ks=3, stride=2, relu=1,
                             w_off=self._push_f(w4), b_off=self._push_f(b)))
        return y

    def conv(self, sd, conv, bn, x, stride, relu, res=None, out_dtype=DT_BF16) -> int:
        w, b = fold_bn(sd, conv, bn)
        cout, k, _, cin = w.shape
        cp = cout_pad(cout)
        wp = np.zeros((cp, k, k, cin))
        wp[:cout] = w
        bp = np.zeros(cp)
        bp[:cout] = b
        h, ww, c, _ = self.tensors[x]
        assert c == cin, (conv, c, cin)
        pad = k // 2
        y = self.tensor((h + 2 * pad - k) // stride + 1, (ww + 2 * pad - k) // stride + 1, cout, out_dtype)
        self.ops.append(dict(kind=OP_CONV, segment=self._seg, out=y, ins=[x] + ([res] if res is not None else []), up=[1, 1],
                             cin=cin, cout=cout, ks=k, stride=stride, relu=int(relu),
                             w_off=self._push_w(to_bf16_bits(wp)), b_off=self._push_f(bp)))
        return y

    def fuse(self, terms, relu=True) -> int:
        (x0, u0) = terms[0]
        h, w, c, _ = self.tensors[x0]
        y = self.tensor(h * u0, w * u0, c)
        self.ops.append(dict(kind=OP_FUSE, segment=self._seg, out=y, ins=[t for t, _ in terms], up=[u for _, u in terms], cin=c,
                             cout=c, ks=0, stride=0, relu=int(relu), w_off=0, b_off=0))
        return y

    def blobs(self):
        w = np.concatenate(self._w) if self._w else np.zeros(8, np.uint16)
        f = np.concatenate(self._f) if self._f else np.zeros(4, np.float32)
        return w, f


def build_hrnet_w32(sd, micro_batch=None) -> tuple[GraphSpec, int, int]:
    """Walk mmpose's HRNet-W32 + HeatmapHead forward order; returns (spec, input id, output id)."""
    mb = micro_batch_config() if micro_batch is None else micro_batch
    g = GraphSpec()
    g.segment(mb.get("stem", 0))
    x_in = g.tensor(INPUT_HW[0], INPUT_HW[1], 4)
    x = g.stem(sd, "backbone.conv1", "backbone.bn1", x_in)
    x = g.conv(sd, "backbone.conv2", "backbone.bn2", x, 2, True)
    for b in range(4):
        p = f"backbone.layer1.{b}"
        idn = g.conv(sd, f"{p}.downsample.0", f"{p}.downsample.1", x, 1, False) if b == 0 else x
        y = g.conv(sd, f"{p}.conv1", f"{p}.bn1", x, 1, True)
        y = g.conv(sd, f"{p}.conv2", f"{p}.bn2", y, 1, True)
        x = g.conv(sd, f"{p}.conv3", f"{p}.bn3", y, 1, True, res=idn)
    ys = [x]
    pre = [256]
    for s, (n_mod, chans) in enumerate(STAGES):
        if s > 0:
            g.segment(0)
        xs = []
        for i, c in enumerate(chans):
            if i < len(pre) and c == pre[i]:
                xs.append(ys[i])
            elif i < len(pre):
                xs.append(g.conv(sd, f"backbone.transition{s + 1}.{i}.0", f"backbone.transition{s + 1}.{i}.1",
                                 ys[-1], 1, True))
            else:
                xs.append(g.conv(sd, f"backbone.transition{s + 1}.{i}.0.0", f"backbone.transition{s + 1}.{i}.0.1",
                                 ys[-1], 2, True))
        for m in range(n_mod):
            p = f"backbone.stage{s + 2}.{m}"
            for bi in range(len(chans)):
                g.segment(mb.get(f"branch{bi}", 0))
                for k in range(4):
                    q = f"{p}.branches.{bi}.{k}"
                    y = g.conv(sd, f"{q}.conv1", f"{q}.bn1", xs[bi], 1, True)
                    xs[bi] = g.conv(sd, f"{q}.conv2", f"{q}.bn2", y, 1, True, res=xs[bi])
            g.segment(0)
            last = s == len(STAGES) - 1 and m == n_mod - 1
            n_out = 1 if last else len(chans)
            outs = []
            for i in range(n_out):
                terms = []
                for j in range(len(chans)):
                    if j == i:
                        terms.append((xs[j], 1))
                    elif j > i:
                        t = g.conv(sd, f"{p}.fuse_layers.{i}.{j}.0", f"{p}.fuse_layers.{i}.{j}.1", xs[j], 1, False)
                        terms.append((t, 2 ** (j - i)))
                    else:
                        t = xs[j]
                        for k in range(i - j):
                            t = g.conv(sd, f"{p}.fuse_layers.{i}.{j}.{k}.0", f"{p}.fuse_layers.{i}.{j}.{k}.1", t, 2,
                                       k != i - j - 1)
                        terms.append((t, 1))
                outs.append(g.fuse(terms))
            xs = outs
        ys = xs
        pre = list(chans)
    out = g.conv(sd, "head.final_layer", None, ys[0], 1, False, out_dtype=DT_F32)
    return g, x_in, out


def basic_block_spec(c: int, h: int, w: int, seed: int = 0, n_blocks: int = 1):
    """A chain of n_blocks HRNet BasicBlocks (conv3x3+BN+ReLU, conv3x3+BN, +x, ReLU)
    on one c-channel h x w plane, for kernel tests and per-layer benchmarks.
    Returns (spec, input id, output id, state dict)."""
    gen = torch.Generator().manual_seed(seed)
    sd = {}
    g = GraphSpec()
    x = g.tensor(h, w, c)
    y = x
    for k in range(n_blocks):
        for j in (1, 2):
            sd[f"b{k}.conv{j}.weight"] = torch.randn((c, c, 3, 3), generator=gen) * (2.0 / (9 * c)) ** 0.5
            sd[f"b{k}.bn{j}.weight"] = 1.0 + 0.1 * torch.randn((c,), generator=gen)
            sd[f"b{k}.bn{j}.bias"] = 0.1 * torch.randn((c,), generator=gen)
            sd[f"b{k}.bn{j}.running_mean"] = 0.1 * torch.randn((c,), generator=gen)
            sd[f"b{k}.bn{j}.running_var"] = 1.0 + 0.2 * torch.rand((c,), generator=gen)
        t = g.conv(sd, f"b{k}.conv1", f"b{k}.bn1", y, 1, True)
        y = g.conv(sd, f"b{k}.conv2", f"b{k}.bn2", t, 1, True, res=y)
    return g, x, y, sd


def projection_spec(cin: int, cout: int, h: int, w: int, k: int = 1, seed: int = 0):
    """Two k x k convs cin -> cout on one h x w plane: t = conv_a(x) (BN, no ReLU) and
    y = relu(conv_b(x) + t) (the Bottleneck conv3 + downsample pattern), for kernel
    tests.  Returns (spec, input id, output id, state dict)."""
    gen = torch.Generator().manual_seed(seed)
    sd = {}
    g = GraphSpec()
    x = g.tensor(h, w, cin)
    for j in ("a", "b"):
        sd[f"{j}.weight"] = torch.randn((cout, cin, k, k), generator=gen) * (2.0 / (k * k * cin)) ** 0.5
        sd[f"{j}bn.weight"] = 1.0 + 0.1 * torch.randn((cout,), generator=gen)
        sd[f"{j}bn.bias"] = 0.1 * torch.randn((cout,), generator=gen)
        sd[f"{j}bn.running_mean"] = 0.1 * torch.randn((cout,), generator=gen)
        sd[f"{j}bn.running_var"] = 1.0 + 0.2 * torch.rand((cout,), generator=gen)
    t = g.conv(sd, "a", "abn", x, 1, False)
    y = g.conv(sd, "b", "bbn", x, 1, True, res=t)
    return g, x, y, sd


def join_spec(h: int, w: int, seed: int = 0, cat: bool = False):
    """Layer1 Bottleneck join on an h x w plane: r = conv_r(x) (64 -> 256; ReLU unless
    `cat`, when it is the downsample that cat-fusion folds into conv_a), y = relu(conv_a(x)
    + r) (64 -> 256, the Bottleneck conv3) and out = relu(conv_b(y)) (256 -> 64, the next
    Bottleneck's conv1) — the pattern the graph's pair-fusion pass runs as one launch.
    Returns (spec, input id, output id, state dict)."""
    gen = torch.Generator().manual_seed(seed)
    sd = {}
    g = GraphSpec()
    x = g.tensor(h, w, 64)
    for j, (co, ci) in (("r", (256, 64)), ("a", (256, 64)), ("b", (64, 256))):
        sd[f"{j}.weight"] = torch.randn((co, ci, 1, 1), generator=gen) * (2.0 / ci) ** 0.5
        sd[f"{j}bn.weight"] = 1.0 + 0.1 * torch.randn((co,), generator=gen)
        sd[f"{j}bn.bias"] = 0.1 * torch.randn((co,), generator=gen)
        sd[f"{j}bn.running_mean"] = 0.1 * torch.randn((co,), generator=gen)
        sd[f"{j}bn.running_var"] = 1.0 + 0.2 * torch.rand((co,), generator=gen)
    r = g.conv(sd, "r", "rbn", x, 1, not cat)
    y = g.conv(sd, "a", "abn", x, 1, True, res=r)
    out = g.conv(sd, "b", "bbn", y, 1, True)
    return g, x, out, sd


def bottleneck_spec(seed: int = 0, n_blocks: int = 4, lead: bool = True):
    """HRNet-W32 layer1 on the 64x48 plane: n_blocks Bottlenecks (1x1 -> 64 + ReLU, 3x3 64 -> 64
    + ReLU, 1x1 -> 256 + identity + ReLU).  lead=True: the first block takes a 64-ch input with
    its 1x1 downsample as the identity (HRNet's layer1.0, whose conv3 the graph cat-fuses), the
    rest run on 256 ch; lead=False: every block on a 256-ch input.  For kernel tests.
    Returns (spec, input id, output id, state dict)."""
    gen = torch.Generator().manual_seed(seed)
    sd = {}

    def mk(name, co, ci, k):
        sd[f"{name}.weight"] = torch.randn((co, ci, k, k), generator=gen) * (2.0 / (k * k * ci)) ** 0.5
        sd[f"{name}bn.weight"] = 1.0 + 0.1 * torch.randn((co,), generator=gen)
        sd[f"{name}bn.bias"] = 0.1 * torch.randn((co,), generator=gen)
        sd[f"{name}bn.running_mean"] = 0.1 * torch.randn((co,), generator=gen)
        sd[f"{name}bn.running_var"] = 1.0 + 0.2 * torch.rand((co,), generator=gen)

    g = GraphSpec()
    x_in = x = g.tensor(64, 48, 64 if lead else 256)
    for b in range(n_blocks):
        first = lead and b == 0
        cin = 64 if first else 256
        mk(f"b{b}.conv1", 64, cin, 1)
        mk(f"b{b}.conv2", 64, 64, 3)
        mk(f"b{b}.conv3", 256, 64, 1)
        if first:
            mk(f"b{b}.ds", 256, 64, 1)
        idn = g.conv(sd, f"b{b}.ds", f"b{b}.dsbn", x, 1, False) if first else x
        y = g.conv(sd, f"b{b}.conv1", f"b{b}.conv1bn", x, 1, True)
        y = g.conv(sd, f"b{b}.conv2", f"b{b}.conv2bn", y, 1, True)
        x = g.conv(sd, f"b{b}.conv3", f"b{b}.conv3bn", y, 1, True, res=idn)
    return g, x_in, x, sd


def layer1_transition_spec(seed: int = 0, output: int = 0):
    """HRNet-W32 layer1 (bottleneck_spec, lead=True) followed by transition1 on its output: t0 =
    3x3/s1 -> 32 ch, t1 = 3x3/s2 -> 64 ch (BN + ReLU).  The graph output is t0 (output=0) or t1;
    the layer1 output then feeds only the transition, the case where the fused Bottleneck hands
    it to trans1 in chunk-planar layout.  Returns (spec, input id, output id, state dict)."""
    g, x, y, sd = bottleneck_spec(seed=seed, n_blocks=4, lead=True)
    gen = torch.Generator().manual_seed(seed + 1)
    for j, co in (("t0", 32), ("t1", 64)):
        sd[f"{j}.weight"] = torch.randn((co, 256, 3, 3), generator=gen) * (2.0 / (9 * 256)) ** 0.5
        sd[f"{j}bn.weight"] = 1.0 + 0.1 * torch.randn((co,), generator=gen)
        sd[f"{j}bn.bias"] = 0.1 * torch.randn((co,), generator=gen)
        sd[f"{j}bn.running_mean"] = 0.1 * torch.randn((co,), generator=gen)
        sd[f"{j}bn.running_var"] = 1.0 + 0.2 * torch.rand((co,), generator=gen)
    t0 = g.conv(sd, "t0", "t0bn", y, 1, True)
    t1 = g.conv(sd, "t1", "t1bn", y, 2, True)
    return g, x, (t0, t1)[output], sd


def stem_spec(seed: int = 0):
    """HRNet's stem on a 256x192 crop: conv1 (3x3/s2 4 -> 64) and conv2 (3x3/s2 64 -> 64),
    BN + ReLU each (the pattern the graph's stem-fusion pass runs as one launch), for
    kernel tests.  Returns (spec, input id, output id, state dict)."""
    sd = {k: v for k, v in random_state_dict(seed).items() if k.startswith(("backbone.conv", "backbone.bn"))}
    g = GraphSpec()
    x = g.tensor(INPUT_HW[0], INPUT_HW[1], 4)
    y = g.stem(sd, "backbone.conv1", "backbone.bn1", x)
    y = g.conv(sd, "backbone.conv2", "backbone.bn2", y, 2, True)
    return g, x, y, sd


def transition_spec(seed: int = 0, output: int = 0):
    """HRNet-W32 transition1 on the layer1 output (256 ch @ 64x48): t0 = 3x3/s1 -> 32 ch and
    t1 = 3x3/s2 -> 64 ch, both BN + ReLU (the pair the graph's transition-fusion pass runs
    as one launch); the graph output is t0 (output=0) or t1 (output=1).  For kernel tests.
    Returns (spec, input id, output id, state dict)."""
    gen = torch.Generator().manual_seed(seed)
    sd = {}
    for j, co in (("t0", 32), ("t1", 64)):
        sd[f"{j}.weight"] = torch.randn((co, 256, 3, 3), generator=gen) * (2.0 / (9 * 256)) ** 0.5
        sd[f"{j}bn.weight"] = 1.0 + 0.1 * torch.randn((co,), generator=gen)
        sd[f"{j}bn.bias"] = 0.1 * torch.randn((co,), generator=gen)
        sd[f"{j}bn.running_mean"] = 0.1 * torch.randn((co,), generator=gen)
        sd[f"{j}bn.running_var"] = 1.0 + 0.2 * torch.rand((co,), generator=gen)
    g = GraphSpec()
    x = g.tensor(64, 48, 256)
    t0 = g.conv(sd, "t0", "t0bn", x, 1, True)
    t1 = g.conv(sd, "t1", "t1bn", x, 2, True)
    return g, x, (t0, t1)[output], sd


SIBLINGS = (("s1", 64, False), ("s2", 32, True), ("s3", 32, True))


def sibling_spec(seed: int = 0, output: int = 0, n: int = 3):
    """A stage-4 HRModule fuse layer's 3x3/s2 convs on the branch-0 tensor (32 ch @ 64x48):
    s1 -> 64 ch (BN, no ReLU), s2 / s3 -> 32 ch (BN + ReLU) — the first n of them, the
    siblings the graph's sibling-fusion pass runs as one launch; the graph output is
    sibling `output`.  For kernel tests.  Returns (spec, input id, output id, state dict)."""
    gen = torch.Generator().manual_seed(seed)
    sd = {}
    for j, co, _ in SIBLINGS[:n]:
        sd[f"{j}.weight"] = torch.randn((co, 32, 3, 3), generator=gen) * (2.0 / (9 * 32)) ** 0.5
        sd[f"{j}bn.weight"] = 1.0 + 0.1 * torch.randn((co,), generator=gen)
        sd[f"{j}bn.bias"] = 0.1 * torch.randn((co,), generator=gen)
        sd[f"{j}bn.running_mean"] = 0.1 * torch.randn((co,), generator=gen)
        sd[f"{j}bn.running_var"] = 1.0 + 0.2 * torch.rand((co,), generator=gen)
    g = GraphSpec()
    x = g.tensor(64, 48, 32)
    outs = [g.conv(sd, j, j + "bn", x, 2, relu) for j, _, relu in SIBLINGS[:n]]
    return g, x, outs[output], sd


def conv_spec(cin: int, cout: int, h: int, w: int, k: int = 3, stride: int = 1, relu: bool = True, seed: int = 0):
    """One k x k conv (+ folded BN, optional ReLU) cin -> cout on an h x w plane, for
    kernel tests and per-conv benchmarks.  Returns (spec, input id, output id, state dict)."""
    gen = torch.Generator().manual_seed(seed)
    sd = {"c.weight": torch.randn((cout, cin, k, k), generator=gen) * (2.0 / (k * k * cin)) ** 0.5,
          "bn.weight": 1.0 + 0.1 * torch.randn((cout,), generator=gen),
          "bn.bias": 0.1 * torch.randn((cout,), generator=gen),
          "bn.running_mean": 0.1 * torch.randn((cout,), generator=gen),
          "bn.running_var": 1.0 + 0.2 * torch.rand((cout,), generator=gen)}
    g = GraphSpec()
    x = g.tensor(h, w, cin)
    y = g.conv(sd, "c", "bn", x, stride, relu)
    return g, x, y, sd


class ConvGraph:
    """A GraphSpec instantiated on the device (mvp_graph_create): one bf16 NHWC
    input tensor -> one output tensor, batch given per forward call."""

    def __init__(self, spec: GraphSpec, input_id: int, output_id: int, max_batch: int, device="cuda"):
        self.spec, self.input_id, self.output_id = spec, input_id, output_id
        w, f = spec.blobs()
        self.device = torch.device(device)
        self.w_dev = torch.from_numpy(w.view(np.int16).copy()).to(self.device)
        self.f_dev = torch.from_numpy(f).to(self.device)
        self.max_batch = int(max_batch)
        tens = (TensorDesc * len(spec.tensors))(*[TensorDesc(*t) for t in spec.tensors])
        ops = (OpDesc * len(spec.ops))()
        for k, op in enumerate(spec.ops):
            d = ops[k]
            d.kind, d.out, d.n_in = op["kind"], op["out"], len(op["ins"])
            for i in range(4):
                d.in_[i] = op["ins"][i] if i < len(op["ins"]) else -1
                d.up[i] = op["up"][i] if i < len(op["up"]) else 1
            d.cin, d.cout, d.ks, d.stride, d.relu = op["cin"], op["cout"], op["ks"], op["stride"], op["relu"]
            d.segment = op["segment"]
            d.w_off, d.b_off = op["w_off"], op["b_off"]
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            segs = (ctypes.c_int * len(spec.seg_micro_batch))(*spec.seg_micro_batch)
            call("mvp_graph_create", tens, len(spec.tensors), ops, len(spec.ops), segs, len(spec.seg_micro_batch),
                 self.input_id, self.output_id,
                 ctypes.c_void_p(self.w_dev.data_ptr()), self.w_dev.numel(), ctypes.c_void_p(self.f_dev.data_ptr()),
                 self.f_dev.numel(), self.max_batch, ctypes.byref(h))
        self._h = h

    def run(self, x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """x: [n][h][w][c] of the input tensor, out: the output tensor; stream-ordered on torch's stream."""
        n = x.shape[0]
        if n > self.max_batch:
            raise ValueError(f"batch {n} > max_batch {self.max_batch}")
        call("mvp_graph_forward", self._h, ctypes.c_void_p(x.data_ptr()), n, ctypes.c_void_p(out.data_ptr()),
             ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))
        return out

    def refresh_weights(self) -> None:
        """w_dev / f_dev were rewritten in place: re-derive the graph's own weight copies."""
        call("mvp_graph_refresh_weights", self._h)

    def sync_weights(self, src: int = 0) -> None:
        """Frame-sharded data parallelism: every rank takes rank `src`'s folded weights (one
        RCCL broadcast of the two blobs over xGMI), then re-derives its graph copies."""
        from . import dist as mdist
        world, _ = mdist.world_rank()
        if world > 1:
            mdist.broadcast_([self.w_dev, self.f_dev], src=src)
            torch.cuda.synchronize(self.device)
            self.refresh_weights()

    @property
    def arena_bytes(self) -> int:
        b = ctypes.c_int64()
        call("mvp_graph_arena_bytes", self._h, ctypes.byref(b))
        return b.value

    def launch_plan(self, batch: int) -> np.ndarray:
        """(n_launches, 4) int64 {launching op, route, crops, MACs} of one forward of `batch`
        crops in launch order (mvp_graph_plan; tools/fwd_breakdown.py pairs it with a trace)."""
        cap = 4096
        rec = np.zeros((cap, 4), np.int64)
        n, tot = ctypes.c_int(), ctypes.c_int64()
        call("mvp_graph_plan", self._h, int(batch), ctypes.c_void_p(rec.ctypes.data), cap, ctypes.byref(n),
             ctypes.byref(tot))
        if n.value > cap:
            raise RuntimeError(f"{n.value} launches > {cap}")
        rec = rec[:n.value].copy()
        assert int(rec[:, 3].sum()) == tot.value == self.macs_per_crop() * batch
        return rec

    def macs_per_crop(self) -> int:
        macs = 0
        for op in self.spec.ops:
            if op["kind"] in (OP_STEM, OP_CONV):
                h, w, _, _ = self.spec.tensors[op["out"]]
                cin = 3 if op["kind"] == OP_STEM else op["cin"]
                macs += h * w * op["cout"] * cin * op["ks"] ** 2
        return macs

    def close(self):
        if getattr(self, "_h", None):
            call("mvp_graph_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HRNetBackbone(ConvGraph):
    """Device-resident HRNet-W32 + head on the libmvpose graph runtime.

    forward(crops (N,256,192,4) bf16 on GPU) -> heatmaps (N,17,64,48) f32."""

    def __init__(self, state_dict=None, seed: int = 0, max_batch: int = 256, device="cuda", micro_batch=None):
        if state_dict is None:
            state_dict = random_state_dict(seed)
        spec, input_id, output_id = build_hrnet_w32(state_dict, micro_batch)
        super().__init__(spec, input_id, output_id, max_batch, device)

    def forward(self, crops: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        if crops.dtype != torch.bfloat16 or not crops.is_cuda or not crops.is_contiguous():
            raise ValueError("crops must be a contiguous bf16 CUDA tensor (N,256,192,4)")
        if tuple(crops.shape[1:]) != (INPUT_HW[0], INPUT_HW[1], 4):
            raise ValueError(f"crops must be (N,{INPUT_HW[0]},{INPUT_HW[1]},4), got {tuple(crops.shape)}")
        n = crops.shape[0]
        if n > self.max_batch:
            raise ValueError(f"batch {n} > max_batch {self.max_batch}")
        if out is None:
            out = torch.empty((n, N_JOINTS) + HEATMAP_HW, dtype=torch.float32, device=crops.device)
        return self.run(crops, out)
