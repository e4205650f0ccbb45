"""Run the heatmap-moments kernel on N flip-averaged synthetic heatmaps (for
rocprofv3 counter passes and timing).  python tools/moments_one.py [N] [reps]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import torch  # noqa: E402

from mvpose import estimator  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
est = estimator.BatchPoseEstimator(max_frames=n)
g = torch.Generator(device="cuda").manual_seed(0)
hm = torch.rand((n, 17, 64, 48), device="cuda", generator=g) * 0.05  # ~80 % of cells above the 0.01 threshold
out = torch.empty((n, 17, 6), dtype=torch.float64, device="cuda")
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(reps + 1):
    if r == 1:
        e0.record()
    estimator.call("mvp_heatmap_moments", ctypes.c_void_p(hm.data_ptr()), n, 17, 64, 48,
                   ctypes.c_void_p(est.revert_minv.data_ptr()), 720, 1280, ctypes.c_float(0.01),
                   int(est.separable), None, ctypes.c_void_p(out.data_ptr()), s)
e1.record()
torch.cuda.synchronize()
print(f"moments: {e0.elapsed_time(e1) / reps:.3f} ms per launch of {n} camera-frames", flush=True)
