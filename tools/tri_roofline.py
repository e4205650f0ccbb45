"""Triangulation kernel roofline at BASELINE config-4 scale: 100k synchronised
frames (1.7 M (frame, joint) problems) per launch, synthetic rig and poses
(1 px noise), default solver (QR + inverse iteration) vs exact (Jacobi).

    python tools/tri_roofline.py [T]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mvpose import ops, synthetic as syn  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
for V, mode, ci in ((2, ops.TRI_REFERENCE, [0, 1]), (4, ops.TRI_ALL_VIEWS, [0, 1, 2, 3])):
    cams = syn.make_rig(V, seed=1)
    k = syn.make_kpts_2d(syn.make_poses(min(T, 2000), seed=2), cams, seed=3)
    k = np.ascontiguousarray(np.tile(k, (T // k.shape[0] + 1, 1, 1, 1))[:T])
    kd = torch.tensor(k, device="cuda")
    cd = torch.tensor(ops.pack_cameras(syn.reference_camera_params(cams)), device="cuda")
    outs = {}
    for exact in (False, True):
        out = torch.empty((T, 17, 3), device="cuda")
        for _ in range(3):
            ops.triangulate(kd, cd, ci, mode=mode, out=out, exact=exact)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 300
        e0.record()
        for _ in range(n):
            ops.triangulate(kd, cd, ci, mode=mode, out=out, exact=exact)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        gbs = T * 12 * 17 * (V + 1) / ms / 1e6
        outs[exact] = out.cpu().numpy()
        print(f"V={V} mode={mode} exact={int(exact)} T={T}: {ms:.4f} ms/launch, {T / ms * 1e3 / 1e6:.2f} M frames/s, "
              f"{gbs:.1f} GB/s algorithmic ({100 * gbs / 8000:.2f}% of 8 TB/s)", flush=True)
    d = np.abs(outs[False] - outs[True])
    print(f"  fast vs exact: max |diff| {np.nanmax(d):.3e}, bit-identical {np.mean(outs[False] == outs[True]):.5f}",
          flush=True)
