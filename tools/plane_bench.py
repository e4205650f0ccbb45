"""BasicBlock planes with the graph's default kernels at the bench batch (1024 crops):
us per conv (HIP events on torch's stream).  Diagnostics through the kernels' env
switches (e.g. MVPOSE_TCONV_DIAG).
    python tools/plane_bench.py [reps] [C,H,W ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import torch  # noqa: E402

from mvpose import hrnet  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
planes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[2:]] or \
    [(32, 64, 48), (64, 32, 24), (128, 16, 12), (256, 8, 6), (64, 64, 48)]
n = 1024
for c, h, w in planes:
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
    us = e0.elapsed_time(e1) * 1e3 / reps / 2
    print(f"C={c:3d} {h}x{w}: {us:7.1f} us/conv", flush=True)
    g.close()
