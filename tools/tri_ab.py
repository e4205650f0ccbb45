"""A/B timing of triangulation builds: python tools/tri_ab.py lib1.so lib2.so ..."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mvpose import ops, synthetic as syn  # noqa: E402

T = 100_000
cams = syn.make_rig(2, seed=1)
k = syn.make_kpts_2d(syn.make_poses(2000, seed=2), cams, seed=3)
k = np.ascontiguousarray(np.tile(k, (T // k.shape[0] + 1, 1, 1, 1))[:T])
kd = torch.tensor(k, device="cuda")
cd = torch.tensor(ops.pack_cameras(syn.reference_camera_params(cams)), device="cuda")
ci = (ctypes.c_int * 2)(0, 1)
ref = None
for rnd in range(3):
    for path in sys.argv[1:]:
        lib = ctypes.CDLL(os.path.abspath(path))
        f = lib.mvp_triangulate
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                      ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                      ctypes.c_void_p]
        out = torch.empty((T, 17, 3), device="cuda")
        st = torch.cuda.current_stream().cuda_stream

        def run():
            assert f(kd.data_ptr(), T * 17, 2, cd.data_ptr(), 2, ci, 2, 0, out.data_ptr(), None, st) == 0

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(300):
            run()
        e1.record()
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        ref = o if ref is None else ref
        print(f"round {rnd} {os.path.basename(path)}: {e0.elapsed_time(e1) / 300:.4f} ms, identical {np.array_equal(o, ref)}",
              flush=True)
