"""Per-plane BasicBlock timing (two 3x3 convs + residual) at the bench batch, per
conv kernel family (generic conv_mfma_kernel, tconv / tconv16).  HIP events on
torch's stream.
  python tools/conv_bench.py [batch] [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import torch  # noqa: E402

from mvpose import hrnet  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
_OFF = {"MVPOSE_NO_TCONV": "1", "MVPOSE_NO_TBLOCK": "1"}
MODES = {"generic": dict(_OFF), "tconv": dict(_OFF, MVPOSE_NO_TCONV="0", MVPOSE_NO_TBLOCK="0")}
for c, h, w in [(32, 64, 48), (64, 32, 24), (128, 16, 12), (256, 8, 6), (64, 64, 48)]:
    for mode, env in MODES.items():
        os.environ.update(env)
        spec, xi, yo, _ = hrnet.basic_block_spec(c, h, w, seed=1)
        g = hrnet.ConvGraph(spec, xi, yo, max_batch=n)
        x = torch.randn((n, h, w, c), device="cuda").bfloat16()
        y = torch.empty_like(x)
        for _ in range(3):
            g.run(x, y)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            g.run(x, y)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps / 2  # per conv
        flop = 2.0 * n * h * w * c * c * 9
        print(f"C={c:3d} {h}x{w} {mode:8s}: {us:7.1f} us/conv  "
              f"{flop / us / 1e6:6.1f} TFLOP/s ({flop / us / 1e6 / 2500 * 100:4.1f}% of 2.5 PF)", flush=True)
        g.close()
