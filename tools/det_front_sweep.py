"""Detector micro-batched front sweep (mvp_det_set_front), one process, same frames:
    python tools/det_front_sweep.py [batch=512] [iters=5]
For each (front end stage, micro-batch): ms per forward (HIP events), and whether best / cand equal
the un-micro-batched forward bit for bit."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd")]
from mvpose import rtmdet as D  # noqa: E402

batch = int(sys.argv[1]) if len(sys.argv) > 1 else 512
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
os.environ["MVPOSE_DET_MB"] = "0"
det = D.RTMDetector(seed=0, max_batch=batch)
g = torch.Generator(device="cuda").manual_seed(0)
frames = torch.randint(0, 256, (batch, 720, 1280, 3), dtype=torch.uint8, device="cuda", generator=g)


def run():
    for _ in range(2):
        r = det.detect(frames)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        r = det.detect(frames)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters, r["best"].clone(), r["cand"].clone()


configs = [("", 0)] + [(st, mb) for st in ("backbone.stage2", "backbone.stage3") for mb in (8, 16, 32, 64)] + [("", 0)]
base = None
for st, mb in configs:
    det.set_front(st, mb)
    ms, best, cand = run()
    if base is None:
        base = (best, cand)
    same = torch.equal(best, base[0]) and torch.equal(cand, base[1])
    print(f"front {st or '-':16s} mb {mb:3d}: {ms:7.2f} ms/forward {batch / ms * 1e3:7.0f} frames/s  "
          f"arena {det.arena_bytes / 2**30:5.2f} GiB  bit-identical {same}", flush=True)
