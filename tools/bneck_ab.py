"""Same-box A/B of HRNet layer1 (bottleneck_spec, 4 blocks, 1024 crops): the fused Bottleneck
(bneck.hip) against the unfused graph (MVPOSE_NO_BNECK=1).  Prints ms per forward."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "multi-camera_3d_pose_estimation_amd"))
from mvpose import hrnet  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
spec, xi, yo, _ = hrnet.bottleneck_spec(seed=1, n_blocks=4, lead=True)
x = torch.relu(torch.randn((n, 64, 48, 64), device="cuda")).bfloat16()
out = torch.empty((n, 64, 48, 256), dtype=torch.bfloat16, device="cuda")
graphs = {}
for mode in (("0",) if os.environ.get("BNECK_AB_ONLY") == "fused" else ("1", "0")):
    os.environ["MVPOSE_NO_BNECK"] = mode
    graphs[mode] = hrnet.ConvGraph(spec, xi, yo, max_batch=n)
for rnd in range(3):
    for mode, g in graphs.items():
        for _ in range(3):
            g.run(x, out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(10):
            g.run(x, out)
        e1.record()
        torch.cuda.synchronize()
        print(f"round {rnd} {'unfused' if mode == '1' else 'fused  '}: {e0.elapsed_time(e1) / 10:.3f} ms per layer1 forward "
              f"({n} crops), arena {g.arena_bytes / 2**30:.2f} GiB", flush=True)
