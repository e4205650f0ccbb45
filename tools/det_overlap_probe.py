"""Probe (round 6): does the detector of one batch overlap the 2D->3D pipeline of another on two
streams?  Times, per step, detect(512 camera-frames) and process(256 2-cam frames) in series on one
stream and side by side on two streams (independent inputs, as a pipelined stream of batches)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd")]
from mvpose import hrnet, synthetic as syn  # noqa: E402
from mvpose.estimator import BatchPoseEstimator  # noqa: E402
from mvpose.pipeline import MultiViewPipeline  # noqa: E402
from mvpose.rtmdet import RTMDetector  # noqa: E402

dev = torch.device("cuda:0")
B, V, reps = 256, 2, 5
est = BatchPoseEstimator(hrnet.random_state_dict(0), max_frames=B * V, device=dev)
pipe = MultiViewPipeline(syn.reference_camera_params(syn.make_rig(V, seed=1)), estimator=est, device=dev)
det = RTMDetector(seed=0, max_batch=B * V, device=dev)
g = torch.Generator(device=dev).manual_seed(5)
fr = torch.randint(0, 256, (B * V, 720, 1280, 3), dtype=torch.uint8, device=dev, generator=g)
fr2 = torch.randint(0, 256, (B, V, 720, 1280, 3), dtype=torch.uint8, device=dev, generator=g)
out = {}
sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def timed(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def det_only():
    det.detect(fr)


def pose_only():
    pipe.process(fr2, out)


def serial():
    det.detect(fr)
    pipe.process(fr2, out)


def side_by_side():
    cur = torch.cuda.current_stream(dev)
    sa.wait_stream(cur)
    sb.wait_stream(cur)
    with torch.cuda.stream(sa):
        det.detect(fr)
    with torch.cuda.stream(sb):
        pipe.process(fr2, out)
    cur.wait_stream(sa)
    cur.wait_stream(sb)


for name, fn in (("detect", det_only), ("pose", pose_only), ("serial", serial), ("two streams", side_by_side),
                 ("serial", serial), ("two streams", side_by_side)):
    print(f"{name:12s} {timed(fn):8.2f} ms per step", flush=True)
