"""tconv look-ahead experiment: per-conv time of the 64-ch 32x24 BasicBlock plane and
the 256-ch 8x6 plane at 1024 crops, MVPOSE_TCONV_LD=1 vs 2 (set in the env)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import torch
from mvpose import hrnet
n, reps = 1024, 30
for c, h, w in [(64, 32, 24), (256, 8, 6), (64, 64, 48)]:
    spec, xi, yo, _ = hrnet.basic_block_spec(c, h, w, seed=1)
    if c == 64 and h == 64:
        spec, xi, yo, _ = hrnet.conv_spec(64, 64, 64, 48)
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
    nconv = 1 if h == 64 else 2
    print(f"LD={os.environ.get('MVPOSE_TCONV_LD', '1')} C={c} {h}x{w}: {e0.elapsed_time(e1) * 1e3 / reps / nconv:.1f} us/conv", flush=True)
    g.close()
