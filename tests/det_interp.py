"""Test helper: executes a DetSpec (mvpose.rtmdet's op list for the HIP detector runtime)
with torch fp32 on the storage layouts the device uses (padded channels, channel views,
shared concat buffers, bf16-rounded weights from the blobs).

Run on the oracle's letterboxed input it must reproduce oracle/rtmdet_ref.py's RTMDet-m
candidates up to bf16 weight rounding: that pins the host builder's wiring (views,
padding maps, BN folding, fused sibling convs) independently of the GPU; on the GPU
the same interpreter is the per-layer reference with the device's exact weights.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from mvpose import rtmdet as D


def _act(x, a):
    return F.silu(x) if a == D.ACT_SILU else F.relu(x) if a == D.ACT_RELU else x


def apply_op(spec: D.DetSpec, T: list, op, cand: torch.Tensor, device_weights: bool = False) -> None:
    """Execute one op on the fp32 tensors T (list of (n, h, w, c)) in place.
    device_weights: the stem's f32 weights rounded to bf16 as the MFMA stem kernel uses them."""
    if not hasattr(spec, "_interp_blobs"):
        wbits, fblob = spec.blobs()
        spec._interp_blobs = (torch.from_numpy(wbits.astype(np.uint32) << 16).view(torch.float32), torch.from_numpy(fblob))
    wf, fb = spec._interp_blobs
    n = T[0].shape[0]

    def get(v):
        return T[v.t][..., v.coff:v.coff + v.c].permute(0, 3, 1, 2)

    def put(v, y):
        T[v.t][..., v.coff:v.coff + v.c] = y.permute(0, 2, 3, 1)

    if op.kind == D.DET_STEM:
        w = fb[op.w_off:op.w_off + 32 * 36].view(32, 3, 3, 4).permute(0, 3, 1, 2)
        if device_weights:
            w = w.to(torch.bfloat16).float()
        b = fb[op.b_off:op.b_off + 32]
        put(op.out, _act(F.conv2d(T[op.in_.t].permute(0, 3, 1, 2), w, b, stride=2, padding=1), op.act))
    elif op.kind == D.DET_CONV:
        cin, cout, ks = op.in_.c, op.out.c, op.ks
        cp = D.cout_pad(cout)
        if spec.f32_weights is not None and not device_weights:  # unrounded weights: a pure wiring check
            w = torch.from_numpy(spec.f32_weights[op.w_off])[:cout].permute(0, 3, 1, 2)
        else:
            w = wf[op.w_off:op.w_off + cp * ks * ks * cin].view(cp, ks, ks, cin)[:cout].permute(0, 3, 1, 2)
        b = fb[op.b_off:op.b_off + cout]
        y = F.conv2d(get(op.in_), w, b, stride=op.stride, padding=ks // 2)
        if op.act == D.ACT_SILU:  # SiLU before the residual (CSPNeXtBlock), ReLU after it
            y = _act(y, op.act)
        if op.res.t >= 0:
            y = y + get(op.res)
        put(op.out, y if op.act == D.ACT_SILU else _act(y, op.act))
    elif op.kind == D.DET_DW:
        c = op.in_.c
        w = fb[op.w_off:op.w_off + c * 25].view(c // 8, 25, 8).permute(0, 2, 1).reshape(c, 1, 5, 5)
        b = fb[op.b_off:op.b_off + c]
        put(op.out, _act(F.conv2d(get(op.in_), w, b, padding=2, groups=c), op.act))
    elif op.kind == D.DET_DWPW:   # depthwise 5x5 + SiLU, then pointwise 1x1 + SiLU (+ identity)
        c = op.in_.c
        w = fb[op.w_off:op.w_off + c * 25].view(c // 8, 25, 8).permute(0, 2, 1).reshape(c, 1, 5, 5)
        b = fb[op.b_off:op.b_off + c]
        t = _act(F.conv2d(get(op.in_), w, b, padding=2, groups=c), op.act)
        if device_weights:        # the kernel rounds the intermediate to bf16, as the unfused pair stores it
            t = t.to(torch.bfloat16).float()
        cout = op.out.c
        cp = D.cout_pad(cout)
        if spec.f32_weights is not None and not device_weights:
            wp = torch.from_numpy(spec.f32_weights[op.aux])[:cout].permute(0, 3, 1, 2)
        else:
            wp = wf[op.aux:op.aux + cp * c].view(cp, 1, 1, c)[:cout].permute(0, 3, 1, 2)
        y = _act(F.conv2d(t, wp, fb[op.b_off + c:op.b_off + c + cout]), op.act)
        if op.res.t >= 0:
            y = y + get(op.res)
        put(op.out, y)
    elif op.kind == D.DET_CA:
        c = op.in_.c
        x = get(op.in_)
        wt = fb[op.w_off:op.w_off + c * c].view(c, c)
        b = fb[op.b_off:op.b_off + c]
        s = F.hardsigmoid(x.mean(dim=(2, 3)) @ wt + b)
        put(op.in_, x * s[:, :, None, None])
    elif op.kind == D.DET_SPP:
        x = get(op.in_)
        c = op.in_.c
        for j in range(1, 4):
            x = F.max_pool2d(x, 5, 1, 2)
            T[op.in_.t][..., j * c:(j + 1) * c] = x.permute(0, 2, 3, 1)
    elif op.kind == D.DET_UP2:
        put(op.out, F.interpolate(get(op.in_), scale_factor=2, mode="nearest"))
    elif op.kind == D.DET_HEAD:
        x = get(op.in_)  # (n, 2F, h, w)
        fdim = op.in_.c // 2
        w = fb[op.w_off:op.w_off + 5 * fdim].view(5, fdim)
        b = fb[op.b_off:op.b_off + 5]
        cls = torch.einsum("nchw,c->nhw", x[:, :fdim], w[0]) + b[0]
        reg = torch.einsum("nchw,oc->nhwo", x[:, fdim:], w[1:]) + b[1:]
        h, ww = x.shape[2:]
        s = float(op.stride)
        ys, xs = torch.meshgrid(torch.arange(h, dtype=torch.float32) * s, torch.arange(ww, dtype=torch.float32) * s,
                                indexing="ij")
        d = torch.exp(reg) * s
        lim = float(spec.size)
        box = torch.stack([(xs - d[..., 0]).clamp(0, lim), (ys - d[..., 1]).clamp(0, lim),
                           (xs + d[..., 2]).clamp(0, lim), (ys + d[..., 3]).clamp(0, lim)], -1)
        rows = slice(op.aux, op.aux + h * ww)
        cand[:, rows, 0] = torch.sigmoid(cls).reshape(n, -1)
        cand[:, rows, 1:5] = box.reshape(n, -1, 4)
        cand[:, rows, 5] = cls.reshape(n, -1)


def run_spec(spec: D.DetSpec, x_nhwc4: torch.Tensor, trace: dict | None = None, n_ops: int | None = None):
    """x_nhwc4: (N, S, S, 4) f32 letterboxed + normalised input -> cand (N, P, 6) f32."""
    n = x_nhwc4.shape[0]
    T = [torch.zeros((n, h, w, c), dtype=torch.float32) for h, w, c, _ in spec.tensors]
    T[0] = x_nhwc4.float().clone()
    cand = torch.zeros((n, spec.n_priors, 6), dtype=torch.float32)
    for k, op in enumerate(spec.ops[:n_ops]):
        apply_op(spec, T, op, cand)
        if trace is not None:
            trace[k] = T
    return cand
