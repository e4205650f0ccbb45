"""Seeded refinement problems shared by the golden generator (tests/golden/make_golden.py)
and the parity tests.  Large problems (BASELINE config 5: V=8, T=400) are not stored in the
fixtures: the tests rebuild them from the seed and check a SHA-256 of the inputs against the
digest the generator recorded, so the fixture only holds seeds, digest and reference outputs.
"""
from __future__ import annotations

import hashlib

import numpy as np

from mvpose import synthetic as syn


def sgd_inputs(V, T, seed):
    """Synthetic heatmaps_2d (T,V,17,6) f64 Gaussians + kpts_3d (T,17,3) f32 init."""
    rng = np.random.default_rng(seed)
    cams = syn.make_rig(V, seed=seed)
    poses = syn.make_poses(T, seed=seed + 1)
    gauss = np.zeros((T, V, 17, 6))
    for v, c in enumerate(cams):
        uv = syn.project(poses, c) + rng.normal(0, 2.0, (T, 17, 2))
        sx = rng.uniform(2.0, 6.0, (T, 17))
        sy = rng.uniform(2.0, 6.0, (T, 17))
        rho = rng.uniform(-0.4, 0.4, (T, 17))
        gauss[:, v, :, 0:2] = uv
        gauss[:, v, :, 2] = sx * sx
        gauss[:, v, :, 3] = rho * sx * sy
        gauss[:, v, :, 4] = rho * sx * sy
        gauss[:, v, :, 5] = sy * sy
    init = (poses + rng.normal(0, 3.0, poses.shape)).astype(np.float32)
    return cams, gauss, init


def inputs_digest(cams, gauss, init):
    h = hashlib.sha256()
    for c in cams:
        for k in ("K", "R", "T", "dist"):
            h.update(np.ascontiguousarray(c[k], np.float64).tobytes())
    h.update(np.ascontiguousarray(gauss, np.float64).tobytes())
    h.update(np.ascontiguousarray(init, np.float32).tobytes())
    return h.hexdigest()


def bench_c5_inputs(V=8, T=400):
    """The bench's config-5 problem (bench.py::sgd_line): isotropic 3-px Gaussians around noisy
    projections of a seeded walk, init = poses + 3 cm noise."""
    rng = np.random.default_rng(5)
    cams = syn.make_rig(V, seed=5)
    poses = syn.make_poses(T, seed=6)
    g = np.zeros((T, V, 17, 6))
    for v, c in enumerate(cams):
        g[:, v, :, 0:2] = syn.project(poses, c) + rng.normal(0, 2.0, (T, 17, 2))
        g[:, v, :, 2] = g[:, v, :, 5] = 9.0
    x0 = (poses + rng.normal(0, 3.0, poses.shape)).astype(np.float32)
    return cams, g, x0


# bench.py::sgd_line's optimisation (early stop off: patience never reached)
BENCH_C5_ITERS = 40
BENCH_C5_KW = dict(lr=0.01, lambda_smooth=1e-6, lambda_body_length=1.0, patience=10 ** 9, tolerance=1e-5,
                   max_iter=BENCH_C5_ITERS - 1)
