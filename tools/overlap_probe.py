"""Does the moments kernel overlap the backbone when issued on a second stream?
Times backbone(1024 crops) alone, moments(512 camera-frames) alone, and both issued
concurrently on two streams.  python tools/overlap_probe.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import torch  # noqa: E402

from mvpose import estimator, hrnet  # noqa: E402

est = estimator.BatchPoseEstimator(max_frames=512)
bb = est.backbone
x = torch.randn((1024, 256, 192, 4), device="cuda").bfloat16()
hm = torch.rand((512, 17, 64, 48), device="cuda") * 0.05
out = torch.empty((512, 17, 6), dtype=torch.float64, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def moments(stream):
    estimator.call("mvp_heatmap_moments", ctypes.c_void_p(hm.data_ptr()), 512, 17, 64, 48,
                   ctypes.c_void_p(est.revert_minv.data_ptr()), 720, 1280, ctypes.c_float(0.01),
                   int(est.separable), None, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(stream.cuda_stream))


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def run_bb():
    with torch.cuda.stream(s1):
        bb.forward(x, out=est.heatmaps)


def run_mom():
    moments(s2)


def run_both():
    run_bb()
    run_mom()


tb = timed(run_bb)
tm = timed(run_mom)
tt = timed(run_both)
print(f"backbone {tb:.2f} ms, moments {tm:.2f} ms, sum {tb + tm:.2f} ms, concurrent {tt:.2f} ms", flush=True)
