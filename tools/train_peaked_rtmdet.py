"""Seeded fine-tuning that gives the synthetic RTMDet-m a trained-model-like, PEAKED person score.

The detector's end-to-end parity test (tests/test_rtmdet_gpu.py) compares the bf16 GPU
detector with the fp32 restatement (oracle/rtmdet_ref.py) on identical frames.  With the
seeded random weights (mvpose.rtmdet.random_state_dict) the class logits are noise-like, so
the selected prior (the per-frame argmax the reference's first-box hand-off reduces to) is
decided by near-ties.  As tools/train_peaked_hrnet.py does for HRNet-W32, this script keeps
the seeded random backbone and neck (with their calibrated BN statistics) and fits only the
head's classification branch on rendered skeleton frames (mvpose.synthetic.make_skeleton_frames:
one person of coloured discs per frame):

* every BatchNorm's running statistics are re-calibrated on skeleton frames (one train-mode
  pass with momentum 1, as tools/calibrate_rtmdet.py does on the bench's noise frames), so the
  activations are O(1) on these inputs;
* then each level's cls BatchNorm affine parameters and rtm_cls 1x1 conv are fitted (the
  shared random 3x3 cls convs stay as they are);
* target logits: -4 everywhere, and on the stride-8 level a Gaussian bump of height 8 (sigma
  0.8 grid cells) centred on the prior nearest to the person's head (the nose disc, the one
  red disc of the skeleton) — so the trained network has one clear best prior per frame, as a
  real detector has on a clearly visible person;
* loss: cross-entropy of the target prior over all 8,400 priors (a decisive top-1, as the
  selection needs) + 0.05 x MSE of the logits to the target map; Adam, fixed seeds; the backbone + neck features and the first cls conv's
  output are computed once (no gradient), so the fit runs on the CPU in a few minutes.

    python tools/train_peaked_rtmdet.py
writes multi-camera_3d_pose_estimation_amd/mvpose/data/rtmdet_m_peaked.npz (the fitted tensors
only, mmdet state-dict names), loaded by mvpose.rtmdet.peaked_state_dict() with numpy's
pickle-free loader.  The box-regression branch keeps its random weights (the parity test is
about the selected prior).
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd")]

from mvpose import rtmdet as D, synthetic as syn  # noqa: E402
from oracle import rtmdet_ref as R  # noqa: E402

OUT = os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd", "mvpose", "data", "rtmdet_m_peaked.npz")
BASE_SEED = 0
TRAIN_SEED, N_TRAIN = 41, 192
SIGMA, LOW, HIGH = 0.8, -4.0, 8.0
N_CALIB = 8
STRIDES = (8, 16, 32)


def nose_points(joints, h, w):
    """Image coordinates of each frame's nose disc (joint 0) as make_skeleton_frames draws it."""
    k, off = syn._whole_image_heatmap_to_image(h, w)
    return joints[:, 0] * k + off


def target_logits(pt_lb, shapes):
    """Per level (h, w) target logits for one letterboxed nose point (x, y)."""
    out = []
    for li, ((h, w), s) in enumerate(zip(shapes, STRIDES)):
        t = np.full((h, w), LOW, np.float32)
        if li == 0:
            gx, gy = int(np.clip(np.round(pt_lb[0] / s), 0, w - 1)), int(np.clip(np.round(pt_lb[1] / s), 0, h - 1))
            yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
            t += HIGH * np.exp(-((xx - gx) ** 2 + (yy - gy) ** 2) / (2 * SIGMA ** 2))
        out.append(t)
    return out


def calibrate_bn(sd, frames):
    """Every BN's running statistics = the activation statistics on these frames."""
    m = R.build_model(sd)
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.momentum = 1.0
    m.train()
    x = torch.cat([R.normalize(R.letterbox(f, D.SIZE)[0]) for f in frames])
    with torch.no_grad():
        m(x)
    return {k: v.clone() for k, v in m.state_dict().items()
            if k.endswith(".bn.running_mean") or k.endswith(".bn.running_var")}


def features(m, frames):
    """Backbone + neck features of the letterboxed, normalised frames (no gradient)."""
    feats = [[], [], []]
    with torch.no_grad():
        for f in frames:
            fs = m.neck(m.backbone(R.normalize(R.letterbox(f, D.SIZE)[0])))
            for i in range(3):
                feats[i].append(fs[i])
    return [torch.cat(f) for f in feats]


def conv1_out(m, feats):
    """The first (fixed) cls conv's pre-BN output per level."""
    with torch.no_grad():
        return [m.bbox_head.cls_convs[lvl][0].conv(x) for lvl, x in enumerate(feats)]


def head_cls(m, c1s):
    outs = []
    hd = m.bbox_head
    for lvl, c in enumerate(c1s):
        l0, l1 = hd.cls_convs[lvl]
        c = torch.nn.functional.silu(l0.bn(c))
        c = torch.nn.functional.silu(l1.bn(l1.conv(c)))
        outs.append(hd.rtm_cls[lvl](c)[:, 0])
    return outs


def trainable(m):
    ps = {}
    hd = m.bbox_head
    for lvl in range(3):
        for i, layer in enumerate(hd.cls_convs[lvl]):
            ps[f"bbox_head.cls_convs.{lvl}.{i}.bn.weight"] = layer.bn.weight
            ps[f"bbox_head.cls_convs.{lvl}.{i}.bn.bias"] = layer.bn.bias
        ps[f"bbox_head.rtm_cls.{lvl}.weight"] = hd.rtm_cls[lvl].weight
        ps[f"bbox_head.rtm_cls.{lvl}.bias"] = hd.rtm_cls[lvl].bias
    return ps


def lead_stats(outs):
    lg = torch.cat([o.reshape(o.shape[0], -1) for o in outs], 1)
    t2 = torch.topk(lg, 2, dim=1).values
    return (t2[:, 0] - t2[:, 1]).detach().numpy()


def main():
    torch.manual_seed(0)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    t0 = time.time()
    sd = D.random_state_dict(BASE_SEED)
    cal_frames, _ = syn.make_skeleton_frames(N_CALIB, seed=TRAIN_SEED - 1)
    stats = calibrate_bn(sd, cal_frames)
    sd.update(stats)
    m = R.build_model(sd)
    print(f"BN statistics of {len(stats)} tensors re-calibrated on {N_CALIB} skeleton frames ({time.time() - t0:.0f} s)")
    frames, joints = syn.make_skeleton_frames(N_TRAIN, seed=TRAIN_SEED)
    h, w = frames.shape[1:3]
    _, (sx, sy), _ = R.letterbox(frames[0], D.SIZE)
    pts = nose_points(joints, h, w) * np.array([sx, sy])
    c1 = conv1_out(m, features(m, frames))
    shapes = [tuple(f.shape[-2:]) for f in c1]
    tg = [torch.tensor(np.stack([target_logits(p, shapes)[i] for p in pts])) for i in range(3)]
    print(f"features of {N_TRAIN} frames in {time.time() - t0:.0f} s, levels {shapes}")
    ps = trainable(m)
    for p in m.parameters():
        p.requires_grad_(False)
    for p in ps.values():
        p.requires_grad_(True)
    opt = torch.optim.Adam(list(ps.values()), lr=1e-2)
    g = torch.Generator().manual_seed(1)
    n_steps = 500
    for it in range(n_steps):
        idx = torch.randperm(N_TRAIN, generator=g)[:16]
        outs = head_cls(m, [f[idx] for f in c1])
        lg = torch.cat([o.reshape(o.shape[0], -1) for o in outs], 1)
        tt = torch.cat([t[idx].reshape(len(idx), -1) for t in tg], 1)
        loss = torch.nn.functional.cross_entropy(lg, tt.argmax(1)) + 0.05 * ((lg - tt) ** 2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        if it % 50 == 0 or it == n_steps - 1:
            lead = lead_stats(outs)
            print(f"it {it:4d} loss {loss.item():.4f} top-1 lead median {np.median(lead):.2f} min {lead.min():.2f}",
                  flush=True)
    # held-out frames: the selected prior should be the target's
    tf, tj = syn.make_skeleton_frames(16, seed=TRAIN_SEED + 1000)
    with torch.no_grad():
        outs = head_cls(m, conv1_out(m, features(m, tf)))
    lead = lead_stats(outs)
    tp = nose_points(tj, h, w) * np.array([sx, sy])
    hit = 0
    for i in range(len(tf)):
        tt = torch.cat([torch.tensor(t).reshape(-1) for t in target_logits(tp[i], shapes)])
        lg = torch.cat([o[i].reshape(-1) for o in outs])
        hit += int(int(lg.argmax()) == int(tt.argmax()))
    print(f"held-out: selected prior = target's in {hit}/{len(tf)}; top-1 lead median {np.median(lead):.2f}, "
          f"min {lead.min():.2f}; total {time.time() - t0:.0f} s")
    out = {k: v.detach().numpy().astype(np.float32) for k, v in ps.items()}
    out.update({k: v.numpy().astype(np.float32) for k, v in stats.items()})
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT} ({os.path.getsize(OUT)} B, {len(out)} tensors)")


if __name__ == "__main__":
    main()
