"""Triangulation kernel roofline at BASELINE config-4 scale and beyond: T synchronised frames
(T x 17 (frame, joint) problems) per launch, synthetic rig and poses (1 px noise); solvers:
default (OpenCV rounding, QR + inverse iteration), exact (Jacobi restatement) and, for the
reference mode, tolerance (MVP_TRI_TOLERANCE).

    python tools/tri_roofline.py [T ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mvpose import ops, synthetic as syn  # noqa: E402

Ts = [int(a) for a in sys.argv[1:]] or [100_000, 1_000_000]
for T in Ts:
    for V, mode, ci in ((2, ops.TRI_REFERENCE, [0, 1]), (4, ops.TRI_ALL_VIEWS, [0, 1, 2, 3])):
        cams = syn.make_rig(V, seed=1)
        k = syn.make_kpts_2d(syn.make_poses(min(T, 2000), seed=2), cams, seed=3)
        k = np.ascontiguousarray(np.tile(k, (T // k.shape[0] + 1, 1, 1, 1))[:T])
        kd = torch.tensor(k, device="cuda")
        cd = torch.tensor(ops.pack_cameras(syn.reference_camera_params(cams)), device="cuda")
        outs = {}
        solvers = ("default", "exact", "tolerance") if mode == ops.TRI_REFERENCE else ("default", "exact")
        for sv in solvers:
            kw = {"exact": sv == "exact", "tolerance": sv == "tolerance"}
            out = torch.empty((T, 17, 3), device="cuda")
            for _ in range(3):
                ops.triangulate(kd, cd, ci, mode=mode, out=out, **kw)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 300 if T <= 100_000 else 40
            e0.record()
            for _ in range(n):
                ops.triangulate(kd, cd, ci, mode=mode, out=out, **kw)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / n
            v_used = V if mode == ops.TRI_ALL_VIEWS else 2
            gbs = T * 12 * 17 * (v_used + 1) / ms / 1e6
            outs[sv] = out.cpu().numpy()
            print(f"V={V} mode={mode} {sv:9s} T={T}: {ms:.4f} ms/launch, {T / ms * 1e3 / 1e6:.2f} M frames/s, "
                  f"{gbs:.1f} GB/s algorithmic ({100 * gbs / 8000:.2f}% of 8 TB/s)", flush=True)
        for sv in solvers[1:]:
            d = np.abs(outs["default"] - outs[sv]) if sv == "exact" else np.abs(outs[sv] - outs["exact"])
            ref = "default" if sv == "exact" else "exact"
            print(f"  {sv} vs {ref}: max |diff| {np.nanmax(d):.3e}, bit-identical {np.mean(d == 0):.5f}", flush=True)
        del kd
        torch.cuda.empty_cache()
