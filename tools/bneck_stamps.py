"""Phase timeline of the fused Bottleneck (workgroup 0 of the last layer1 launch), from a
-DBNECK_STAMPS build loaded through MVPOSE_LIB: per wave role, median cycles of each phase."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "multi-camera_3d_pose_estimation_amd"))
from mvpose import hrnet  # noqa: E402

n = 1024
spec, xi, yo, _ = hrnet.bottleneck_spec(seed=1, n_blocks=4, lead=True)
x = torch.relu(torch.randn((n, 64, 48, 64), device="cuda")).bfloat16()
out = torch.zeros((n, 64, 48, 256), dtype=torch.bfloat16, device="cuda")
g = hrnet.ConvGraph(spec, xi, yo, max_batch=n)
for _ in range(3):
    g.run(x, out)
torch.cuda.synchronize()
st = out.view(-1)[: 8 * 128 * 8 * 4].view(torch.int64).cpu().numpy().reshape(8, 128, 8).astype(np.int64)
names = ["P1 work", "B1 wait", "P2 work", "B2 wait", "P3 work", "B3 wait"]
for role, waves in (("C13", range(0, 4)), ("C2", range(4, 8))):
    for w in waves:
        d = []
        for s in range(4, 120):
            t = st[w, s]
            nxt = st[w, s + 1, 0]
            seq = [t[0], t[1] if role == "C13" else t[0], t[2], t[3] if role == "C2" else t[2], t[4], t[5], nxt]
            d.append(np.diff(seq))
        d = np.median(np.array(d), axis=0)
        step = np.median([st[w, s + 1, 0] - st[w, s, 0] for s in range(4, 120)])
        print(f"{role} wave {w}: step {step:7.0f} cyc | " + " ".join(f"{nm} {v:6.0f}" for nm, v in zip(names, d)))
