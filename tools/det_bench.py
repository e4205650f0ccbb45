"""Detector throughput on one GPU: RTMDet-m forward (letterbox -> graph -> per-frame
selection) over resident 720x1280 synthetic frames.

    python tools/det_bench.py [batch] [iters]
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd")]

from mvpose import rtmdet as D  # noqa: E402


def main(batch=128, iters=10):
    det = D.RTMDetector(seed=0, max_batch=batch)
    g = torch.Generator(device="cuda").manual_seed(0)
    frames = torch.randint(0, 256, (batch, 720, 1280, 3), dtype=torch.uint8, device="cuda", generator=g)
    for _ in range(2):
        det.detect(frames)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for _ in range(iters):
        det.detect(frames)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    flops = 2 * det.macs_per_frame * batch
    print(f"batch {batch}: {ms:.2f} ms/forward, {batch / ms * 1e3:.0f} frames/s, "
          f"{flops / ms / 1e9:.1f} TFLOP/s ({flops / ms / 1e9 / 2500 * 100:.1f}% of bf16 peak), "
          f"arena {det.arena_bytes / 2**30:.2f} GiB, wall {(time.perf_counter() - t0) / iters * 1e3:.2f} ms")


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
