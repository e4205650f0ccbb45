"""Same-box A/B of the tolerance triangulation kernel (MVP_TRI_TOLERANCE, the pipeline's
solver) across library builds, 1 M resident 2-cam frames (612 MB per launch):
    python tools/tri_tol_ab.py libA.so libB.so ...
Prints ms per launch per build (alternating, 3 rounds) and each build's max |d| and
bit-identity against the first build's output."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mvpose import ops, synthetic as syn  # noqa: E402

T = 1_000_000
cams = syn.make_rig(2, seed=1)
k = syn.make_kpts_2d(syn.make_poses(2000, seed=2), cams, seed=3)
kd = torch.tensor(k, device="cuda").repeat(T // 2000, 1, 1, 1).contiguous()
cd = torch.tensor(ops.pack_cameras(syn.reference_camera_params(cams)), device="cuda")
ci = (ctypes.c_int * 2)(0, 1)
libs = []
for path in sys.argv[1:]:
    lib = ctypes.CDLL(os.path.abspath(path))
    f = lib.mvp_triangulate
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                  ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_void_p]
    libs.append((os.path.basename(path), f))
outs = {}
times = {n: [] for n, _ in libs}
st = torch.cuda.current_stream().cuda_stream
for rnd in range(3):
    for name, f in libs:
        out = torch.empty((T, 17, 3), device="cuda")
        call = lambda: f(kd.data_ptr(), T * 17, 2, cd.data_ptr(), 2, ci, 2, ops.TRI_TOLERANCE, out.data_ptr(), None, st)
        for _ in range(2):
            assert call() == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            call()
        e1.record()
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) / 10)
        outs[name] = out.cpu().numpy()
ref = outs[libs[0][0]]
for name, _ in libs:
    d = np.abs(outs[name] - ref)
    print(f"{name}: ms per 1M-frame launch {' '.join(f'{t:.4f}' for t in times[name])}; "
          f"max |d| vs {libs[0][0]} {np.nanmax(d):.3g}, bit-identical {np.mean((d == 0) | np.isnan(d)):.6f}")
