"""Seeded CPU fine-tuning that gives the synthetic HRNet-W32 trained-model-like, PEAKED heatmaps.

The end-to-end parity test (tests/test_e2e_parity_gpu.py) compares the bf16 GPU pipeline with
the fp32 oracle on identical frames.  With purely random weights most heatmaps have no peak,
so argmax parity would be measured on near-ties.  This script keeps mvpose.hrnet's seeded
random weights (random_state_dict(BASE_SEED)) for the whole network except the last stage-4
HRModule's high-resolution branch (4 BasicBlocks), its three fuse projections into that branch
and the HeatmapHead, and fits those (~88 k parameters) on rendered skeleton frames
(mvpose.synthetic.make_skeleton_frames) with the standard top-down target: a Gaussian
(sigma 2 heatmap cells) per joint, MSE loss (mmpose MSRAHeatmap + KeypointMSELoss).
Training includes the flipped crops with the flip test's left/right-swapped targets, so the
flip-averaged maps the pipeline decodes have one clear maximum per joint.

Run once in the build container (CPU, ~10-20 min):
    python tools/train_peaked_hrnet.py
It writes multi-camera_3d_pose_estimation_amd/mvpose/data/hrnet_w32_peaked.npz (the trained
tensors only, mmpose state-dict names; loaded by mvpose.hrnet.peaked_state_dict with
numpy's pickle-free loader).  Everything is seeded; the fit is deterministic on one thread
count.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd")]

from mvpose import hrnet, synthetic as syn  # noqa: E402
from oracle import heatmap_ref, hrnet_ref  # noqa: E402

BASE_SEED = hrnet.PEAKED_BASE_SEED
OUT = os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd", "mvpose", "data", "hrnet_w32_peaked.npz")
SIGMA = 2.0
FLIP = heatmap_ref.COCO_FLIP_INDICES


def frozen_features(bb, x):
    """Inputs of the last stage-4 module: branch 0's input, branches 1-3 after their blocks."""
    x = F.relu(bb.bn1(bb.conv1(x)))
    x = F.relu(bb.bn2(bb.conv2(x)))
    x = bb.layer1(x)
    ys = [x]
    for s in range(3):
        trans = getattr(bb, f"transition{s + 1}")
        xs = [ys[i] if t is None else t(ys[-1]) for i, t in enumerate(trans)]
        mods = getattr(bb, f"stage{s + 2}")
        for m in (mods if s < 2 else mods[:-1]):
            xs = m(xs)
        ys = xs
    last = bb.stage4[-1]
    return [xs[0]] + [last.branches[j](xs[j]) for j in (1, 2, 3)]


def trainable_forward(model, feats):
    last = model.backbone.stage4[-1]
    y = last.branches[0](feats[0])
    for j in (1, 2, 3):
        y = y + last.fuse_layers[0][j](feats[j])
    return model.head(F.relu(y))


def calibrate_bn(model, feats, n=128):
    """Running statistics of the trainable part's BatchNorms from these inputs (the random
    ones were drawn for unit-variance noise): each BN in forward order sees its input's batch
    mean / variance, so the fit starts from O(1) activations.  (The GPU graph folds whatever
    statistics the state dict holds.)"""
    last = model.backbone.stage4[-1]
    bns = [mod for blk in last.branches[0] for mod in (blk.bn1, blk.bn2)]
    bns += [last.fuse_layers[0][j][1] for j in (1, 2, 3)]
    hooks = []

    def pre(mod, inp):
        x = inp[0]
        mod.running_mean.copy_(x.mean((0, 2, 3)))
        mod.running_var.copy_(x.var((0, 2, 3)))
    for b in bns:
        hooks.append(b.register_forward_pre_hook(pre))
    with torch.no_grad():
        trainable_forward(model, [f[:n] for f in feats])
    for h in hooks:
        h.remove()


def targets(joints, flipped):
    """(n, 17, 64, 48) Gaussian maps; flipped crops: joint k's disc sits at 47.75 - x and is
    the flip test's channel FLIP[k]."""
    yy, xx = np.mgrid[0:64, 0:48].astype(np.float32)
    n = joints.shape[0]
    t = np.zeros((n, 17, 64, 48), np.float32)
    for i in range(n):
        for k in range(17):
            x, y = joints[i, k]
            ch = k
            if flipped:
                x, ch = 47.75 - x, FLIP[k]
            t[i, ch] = np.exp(-((xx - x) ** 2 + (yy - y) ** 2) / (2 * SIGMA ** 2))
    return t


def crops_of(frames):
    M, _, _ = heatmap_ref.topdown_crop_matrix(frames.shape[2], frames.shape[1])
    return np.stack([heatmap_ref.preprocess(f, M) for f in frames])


def evaluate(model, feats_o, feats_f, joints):
    with torch.no_grad():
        h = trainable_forward(model, feats_o)
        hf = trainable_forward(model, feats_f)
    hfb = hf.flip(-1)[:, FLIP].clone()
    hfb[..., 1:] = hfb[..., :-1].clone()
    avg = ((h + hfb) * 0.5).reshape(h.shape[0], 17, -1).numpy()
    top2 = -np.sort(-avg, axis=-1)[..., :2]
    lead = (top2[..., 0] - top2[..., 1]) / np.abs(avg).max(axis=-1)
    am = avg.argmax(-1)
    want = np.round(joints[..., 1] - 0.25).astype(int) * 48 + np.round(joints[..., 0]).astype(int)
    return (lead > 1e-2).mean(), (am == want).mean(), float(np.median(top2[..., 0]))


def main():
    torch.manual_seed(0)
    torch.set_num_threads(int(os.environ.get("TRAIN_THREADS", "6")))
    model = hrnet_ref.build(hrnet.random_state_dict(BASE_SEED))
    bb = model.backbone
    n_train, n_val = int(os.environ.get("N_TRAIN", "384")), 48
    t0 = time.time()
    fr, jt = syn.make_skeleton_frames(n_train, seed=1000)
    fv, jv = syn.make_skeleton_frames(n_val, seed=2000)
    print(f"rendered {n_train + n_val} frames in {time.time() - t0:.1f}s", flush=True)

    def cache(frames):
        outs_o, outs_f = [[] for _ in range(4)], [[] for _ in range(4)]
        for i in range(0, len(frames), 16):
            x = torch.from_numpy(crops_of(frames[i:i + 16]))
            with torch.no_grad():
                for outs, xin in ((outs_o, x), (outs_f, x.flip(-1))):
                    for k, f in enumerate(frozen_features(bb, xin)):
                        outs[k].append(f)
        return [torch.cat(o) for o in outs_o], [torch.cat(o) for o in outs_f]

    t0 = time.time()
    tr_o, tr_f = cache(fr)
    va_o, va_f = cache(fv)
    print(f"cached frozen features in {time.time() - t0:.1f}s", flush=True)
    feats = [torch.cat([a, b]) for a, b in zip(tr_o, tr_f)]
    tgt = torch.from_numpy(np.concatenate([targets(jt, False), targets(jt, True)]))
    last = bb.stage4[-1]
    params = list(last.branches[0].parameters()) + list(model.head.parameters())
    for j in (1, 2, 3):
        params += list(last.fuse_layers[0][j].parameters())
    for p in model.parameters():
        p.requires_grad_(False)
    for p in params:
        p.requires_grad_(True)
    calibrate_bn(model, feats)
    with torch.no_grad():   # a fresh head (the random one is biased to -0.15)
        model.head.final_layer.weight.normal_(0.0, 0.01)
        model.head.final_layer.bias.zero_()
    epochs, bs = int(os.environ.get("EPOCHS", "60")), int(os.environ.get("BATCH", "16"))
    opt = torch.optim.Adam(params, lr=float(os.environ.get("LR", "5e-4")))
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, epochs)
    n = tgt.shape[0]
    g = torch.Generator().manual_seed(1)
    model.eval()   # BN with its running statistics (affine parameters are trained)
    for ep in range(epochs):
        t0 = time.time()
        perm = torch.randperm(n, generator=g)
        tot = 0.0
        for i in range(0, n, bs):
            idx = perm[i:i + bs]
            out = trainable_forward(model, [f[idx] for f in feats])
            loss = F.mse_loss(out, tgt[idx]) * 1e3
            opt.zero_grad()
            loss.backward()
            opt.step()
            tot += float(loss.detach()) * len(idx)
        sched.step()
        if ep % 5 == 4 or ep == epochs - 1:
            dec, acc, peak = evaluate(model, va_o, va_f, jv)
            print(f"epoch {ep + 1}: loss {tot / n:.4f}  val decidable {dec:.3f} argmax-at-joint {acc:.3f} "
                  f"median peak {peak:.3f}  ({time.time() - t0:.1f}s/epoch)", flush=True)
        else:
            print(f"epoch {ep + 1}: loss {tot / n:.4f} ({time.time() - t0:.1f}s)", flush=True)
    sd = model.state_dict()
    keys = [k for k in sd if k.startswith("backbone.stage4.2.branches.0.") or k.startswith("head.")
            or any(k.startswith(f"backbone.stage4.2.fuse_layers.0.{j}.") for j in (1, 2, 3))]
    keys = [k for k in keys if not k.endswith("num_batches_tracked")]   # incl. the recalibrated BN statistics
    np.savez(OUT, **{k: sd[k].detach().numpy().astype(np.float32) for k in keys})
    print(f"wrote {len(keys)} tensors ({sum(sd[k].numel() for k in keys)} values) to {OUT}")


if __name__ == "__main__":
    main()
