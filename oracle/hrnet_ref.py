"""ORACLE (test infrastructure only) — torch fp32 HRNet-W32 + HeatmapHead.

Restates the 2D model the reference loads through mmpose
(pose_estimation.py:290-297 -> mmpose_pose_estimation.py:103-109; config
`td-hm_hrnet-w32_8xb64-210e_coco-256x192`): mmpose 1.x HRNet backbone (stem
2x conv3x3/s2 + BN + ReLU; layer1 = 4 Bottlenecks to 256 ch; stages 2/3/4 with
1/4/3 HRModules of 2/3/4 branches (32/64/128/256 ch, 4 BasicBlocks per branch)
and multi-scale fuse layers (1x1 conv + BN + nearest upsample; chains of
3x3/s2 conv + BN [+ ReLU]); the last stage-4 module returns only the
highest-resolution branch) and HeatmapHead (final 1x1 conv 32 -> 17 with bias,
no deconvs).  Module / parameter names follow mmpose's, so an mmpose
checkpoint's state dict loads as is.

mmpose is absent and its checkpoints are remote URLs, so parity of this
topology against mmpose is UNPINNED; this module is the fp32 reference the
bf16 HIP backbone (mvpose/hrnet.py + libmvpose) is checked against, on seeded
weights (mvpose.hrnet.random_state_dict).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

BN_EPS = 1e-5
STAGES = ((1, (32, 64)), (4, (32, 64, 128)), (3, (32, 64, 128, 256)))  # (modules, channels)


def _conv(cin, cout, k, s):
    return nn.Conv2d(cin, cout, k, s, k // 2, bias=False)


def _bn(c):
    return nn.BatchNorm2d(c, eps=BN_EPS)


class BasicBlock(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv1, self.bn1 = _conv(c, c, 3, 1), _bn(c)
        self.conv2, self.bn2 = _conv(c, c, 3, 1), _bn(c)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        return F.relu(self.bn2(self.conv2(y)) + x)


class Bottleneck(nn.Module):
    def __init__(self, cin, planes, downsample):
        super().__init__()
        self.conv1, self.bn1 = _conv(cin, planes, 1, 1), _bn(planes)
        self.conv2, self.bn2 = _conv(planes, planes, 3, 1), _bn(planes)
        self.conv3, self.bn3 = _conv(planes, planes * 4, 1, 1), _bn(planes * 4)
        self.downsample = nn.Sequential(_conv(cin, planes * 4, 1, 1), _bn(planes * 4)) if downsample else None

    def forward(self, x):
        identity = self.downsample(x) if self.downsample is not None else x
        y = F.relu(self.bn1(self.conv1(x)))
        y = F.relu(self.bn2(self.conv2(y)))
        return F.relu(self.bn3(self.conv3(y)) + identity)


class HRModule(nn.Module):
    def __init__(self, channels, multiscale_output=True):
        super().__init__()
        nb = len(channels)
        self.nb = nb
        self.branches = nn.ModuleList([nn.Sequential(*[BasicBlock(c) for _ in range(4)]) for c in channels])
        n_out = nb if multiscale_output else 1
        self.fuse_layers = nn.ModuleList()
        for i in range(n_out):
            row = []
            for j in range(nb):
                if j > i:
                    row.append(nn.Sequential(_conv(channels[j], channels[i], 1, 1), _bn(channels[i]),
                                             nn.Upsample(scale_factor=2 ** (j - i), mode="nearest")))
                elif j == i:
                    row.append(None)
                else:
                    chain = []
                    for k in range(i - j):
                        if k == i - j - 1:
                            chain.append(nn.Sequential(_conv(channels[j], channels[i], 3, 2), _bn(channels[i])))
                        else:
                            chain.append(nn.Sequential(_conv(channels[j], channels[j], 3, 2), _bn(channels[j]),
                                                       nn.ReLU()))
                    row.append(nn.Sequential(*chain))
            self.fuse_layers.append(nn.ModuleList(row))

    def forward(self, xs):
        xs = [b(x) for b, x in zip(self.branches, xs)]
        if self.nb == 1:
            return xs
        out = []
        for i, row in enumerate(self.fuse_layers):
            y = 0
            for j in range(self.nb):
                y = y + (xs[j] if i == j else row[j](xs[j]))
            out.append(F.relu(y))
        return out


class HRNetBackbone(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1, self.bn1 = _conv(3, 64, 3, 2), _bn(64)
        self.conv2, self.bn2 = _conv(64, 64, 3, 2), _bn(64)
        self.layer1 = nn.Sequential(Bottleneck(64, 64, True), Bottleneck(256, 64, False),
                                    Bottleneck(256, 64, False), Bottleneck(256, 64, False))
        pre = [256]
        for s, (n_mod, chans) in enumerate(STAGES):
            trans = nn.ModuleList()
            for i, c in enumerate(chans):
                if i < len(pre):
                    trans.append(nn.Sequential(_conv(pre[i], c, 3, 1), _bn(c), nn.ReLU()) if c != pre[i] else None)
                else:
                    trans.append(nn.Sequential(nn.Sequential(_conv(pre[-1], c, 3, 2), _bn(c), nn.ReLU())))
            setattr(self, f"transition{s + 1}", trans)
            last = s == len(STAGES) - 1
            setattr(self, f"stage{s + 2}", nn.ModuleList(
                [HRModule(list(chans), multiscale_output=not (last and m == n_mod - 1)) for m in range(n_mod)]))
            pre = list(chans)

    def forward(self, x):
        x = F.relu(self.bn1(self.conv1(x)))
        x = F.relu(self.bn2(self.conv2(x)))
        x = self.layer1(x)
        ys = [x]
        for s in range(len(STAGES)):
            trans = getattr(self, f"transition{s + 1}")
            # mmpose: a non-None transition always reads the previous stage's LAST output
            xs = [ys[i] if t is None else t(ys[-1]) for i, t in enumerate(trans)]
            for m in getattr(self, f"stage{s + 2}"):
                xs = m(xs)
            ys = xs
        return ys


class HeatmapHead(nn.Module):
    def __init__(self, cin=32, n_joints=17):
        super().__init__()
        self.final_layer = nn.Conv2d(cin, n_joints, 1, 1, 0, bias=True)

    def forward(self, x):
        return self.final_layer(x)


class TopdownHRNet(nn.Module):
    """backbone + head; (N,3,256,192) -> (N,17,64,48)."""

    def __init__(self):
        super().__init__()
        self.backbone = HRNetBackbone()
        self.head = HeatmapHead()

    def forward(self, x):
        return self.head(self.backbone(x)[0])


def build(state_dict) -> TopdownHRNet:
    m = TopdownHRNet()
    m.load_state_dict(state_dict)
    return m.eval()


def flip_test_forward(model, x):
    """mmpose flip test (flip_mode='heatmap', shift_heatmap=True): returns
    (averaged heatmaps (N,17,64,48), raw, raw of the flipped input)."""
    from .heatmap_ref import COCO_FLIP_INDICES
    with torch.no_grad():
        h = model(x)
        hf = model(x.flip(-1))
    hfb = hf.flip(-1)[:, COCO_FLIP_INDICES].clone()
    hfb[..., 1:] = hfb[..., :-1].clone()
    return (h + hfb) * 0.5, h, hf


def conv_macs(model: nn.Module, in_hw=(256, 192)):
    """Per-conv (name, cin, cout, k, stride, out_h, out_w, MACs per crop)."""
    rows, hooks = [], []
    for name, m in model.named_modules():
        if isinstance(m, nn.Conv2d):
            def hook(mod, inp, out, name=name):
                oh, ow = out.shape[-2:]
                rows.append((name, mod.in_channels, mod.out_channels, mod.kernel_size[0], mod.stride[0], oh, ow,
                             mod.in_channels * mod.out_channels * mod.kernel_size[0] ** 2 * oh * ow))
            hooks.append(m.register_forward_hook(hook))
    with torch.no_grad():
        model(torch.zeros(1, 3, *in_hw))
    for h in hooks:
        h.remove()
    return rows
