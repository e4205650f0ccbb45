"""Micro-benchmark of mvp_triangulate (HIP events on the launch stream)."""
import sys, os, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import numpy as np, torch
from mvpose import ops, synthetic as syn

T = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
for V, mode, ci in ((2, 0, [0, 1]), (4, 1, [0, 1, 2, 3])):
    cams = syn.make_rig(V, seed=1)
    poses = syn.make_poses(min(T, 2000), seed=2)
    k = syn.make_kpts_2d(poses, cams, seed=3)
    k = np.tile(k, (T // k.shape[0] + 1, 1, 1, 1))[:T]
    kd = torch.tensor(k, device="cuda")
    cd = torch.tensor(ops.pack_cameras(syn.reference_camera_params(cams)), device="cuda")
    out = torch.empty((T, 17, 3), device="cuda")
    for _ in range(3):
        ops.triangulate(kd, cd, ci, mode=mode, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    e0.record()
    for _ in range(n):
        ops.triangulate(kd, cd, ci, mode=mode, out=out)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    bytes_per_frame = 12 * 17 * (V + 1)
    print(f"V={V} mode={mode} T={T}: {ms:.3f} ms/launch, {T/ms*1e3/1e6:.2f} M frames/s, "
          f"{T*bytes_per_frame/ms/1e6:.1f} GB/s algorithmic ({100*T*bytes_per_frame/ms/1e6/8000:.2f}% of 8 TB/s)")
