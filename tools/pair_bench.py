"""Layer1 Bottleneck-join planes at 1024 crops, for rocprofv3 kernel timing:
cat-fused join (conv1x1_pair_kernel<4, no residual>), residual join (<2, residual>,
after the 64->256 conv1x1 that makes its residual) and the standalone conv3 + residual
(projection_spec: conv1x1 64->256 twice).
    python tools/pair_bench.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import torch  # noqa: E402

from mvpose import hrnet  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
n, h, w = 1024, 64, 48
x = torch.randn((n, h, w, 64), device="cuda").bfloat16()
for name, (spec, xi, yo, _) in (("join_cat", hrnet.join_spec(h, w, seed=1, cat=True)),
                                ("join_res", hrnet.join_spec(h, w, seed=2, cat=False)),
                                ("proj", hrnet.projection_spec(64, 256, h, w, seed=3))):
    g = hrnet.ConvGraph(spec, xi, yo, max_batch=n)
    y = torch.empty((n, h, w, 256 if name == "proj" else 64), device="cuda").bfloat16()
    g.run(x, y)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.run(x, y)
    e1.record()
    torch.cuda.synchronize()
    print(f"{name}: {e0.elapsed_time(e1) / reps * 1e3:.1f} us per graph run", flush=True)
