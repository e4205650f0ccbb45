"""ORACLE (test infrastructure only) — outlier-filtered local linear smoothing.

numpy restatement of the reference's ``linear_interpolation``
(pose_refinement.py:15-84), pinned by tests/golden/interp.npz (generated from
the reference itself).  Per (point, dim, t): window [t - k//2, t + k//2] clipped
to the sequence; keep samples within k_std·std of the window mean AND
median_std·MAD of its median (float32 statistics, numpy's sequential small-n
sums); fewer than 2 kept -> the output stays 0 (the reference ``continue``s
past the assignment, :60-62); otherwise the rolling mean of the kept samples
or the value at t of their least-squares line (np.polyfit degree 1, float64).
"""
from __future__ import annotations

import numpy as np


def _f32_sum(v):
    s = np.float32(0)
    for x in v:
        s = np.float32(s + x)
    return s


def _median(v):
    s = np.sort(v)
    n = len(s)
    if n % 2:
        return s[n // 2]
    return np.float32(np.float32(s[n // 2 - 1] + s[n // 2]) / np.float32(2))


def _window_value(w, start, t, k_std, median_std, rolling, use_median):
    n = len(w)
    mean = np.float32(_f32_sum(w) / np.float32(n))
    dev = (w - mean).astype(np.float32)
    std = np.float32(np.sqrt(np.float32(_f32_sum(dev * dev) / np.float32(n))))
    med = _median(w)
    mad = _median(np.abs(w - med).astype(np.float32))
    keep = np.abs(w - mean) <= np.float32(k_std) * std
    if use_median:
        keep &= np.abs(w - med) <= np.float32(median_std) * mad
    v = w[keep]
    if len(v) < 2:
        return np.float32(0)
    if rolling:
        return np.float32(_f32_sum(v) / np.float32(len(v)))
    tt = np.arange(start, start + n, dtype=np.float64)[keep]
    coef = np.polyfit(tt, v, 1)
    return np.float32(np.polyval(coef, t))


def linear_interpolation(points, k=5, k_std=2, median_std=2, use_rolling_average=False,
                         filter_distance_from_median=True):
    pts = np.array(points)
    squeeze = pts.ndim == 2
    if squeeze:
        pts = pts[:, :, None]
    T, P, D = pts.shape
    out = np.zeros_like(pts)
    for p in range(P):
        for d in range(D):
            for t in range(T):
                a, b = max(0, t - k // 2), min(T, t + k // 2 + 1)
                out[t, p, d] = _window_value(pts[a:b, p, d], a, t, k_std, median_std, use_rolling_average,
                                             filter_distance_from_median)
    return out[:, :, 0] if squeeze else out
