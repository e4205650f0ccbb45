"""Moments kernel timing on the pipeline's own flip-averaged heatmaps (random-init
HRNet-W32 on synthetic frames, 512 camera-frames): closed-form path (separable=1) vs
walking every mixed row (separable=2), and the share of cells near the threshold.
    python tools/moments_real.py [reps]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import torch  # noqa: E402

from mvpose import estimator, hrnet, synthetic as syn  # noqa: E402
from mvpose.pipeline import MultiViewPipeline  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
B, V = 256, 2
est = estimator.BatchPoseEstimator(hrnet.random_state_dict(0), max_frames=B * V)
pipe = MultiViewPipeline(syn.reference_camera_params(syn.make_rig(V, seed=1)), estimator=est)
g = torch.Generator(device="cuda").manual_seed(1234)
frames = torch.randint(0, 256, (B, V, 720, 1280, 3), dtype=torch.uint8, device="cuda", generator=g)
pipe.process(frames)
torch.cuda.synchronize()
avg = est.avg[: B * V].contiguous()
print(f"heatmaps: min {avg.min().item():.4g} max {avg.max().item():.4g} mean {avg.mean().item():.4g}; "
      f"cells >= 0.01: {(avg >= 0.01).float().mean().item():.3f}", flush=True)
out = torch.empty((B * V, 17, 6), dtype=torch.float64, device="cuda")
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for sep in (1, 2):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(reps + 1):
        if r == 1:
            e0.record()
        estimator.call("mvp_heatmap_moments", ctypes.c_void_p(avg.data_ptr()), B * V, 17, 64, 48,
                       ctypes.c_void_p(est.revert_minv.data_ptr()), 720, 1280, ctypes.c_float(0.01), sep,
                       None, ctypes.c_void_p(out.data_ptr()), s)
    e1.record()
    torch.cuda.synchronize()
    print(f"separable={sep}: {e0.elapsed_time(e1) / reps:.3f} ms", flush=True)
