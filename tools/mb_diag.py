"""Micro-batching bit-equality diagnostic: plain vs split segments, with and without tblock64."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import torch  # noqa: E402

from mvpose import hrnet  # noqa: E402

sd = hrnet.random_state_dict(7)
g = torch.Generator().manual_seed(2)
x = torch.zeros((7, 256, 192, 4))
x[..., :3] = torch.randn((7, 256, 192, 3), generator=g)
xb = x.bfloat16().cuda()
for off in ("1", "0"):
    os.environ["MVPOSE_NO_TBLOCK64"] = off
    outs = {}
    for name, mb in (("plain", {"stem": 0, "branch0": 0, "branch1": 0}),
                     ("split", {"stem": 3, "branch0": 2, "branch1": 5, "branch2": 3}),
                     ("b1only", {"branch1": 5}), ("dflt", None)):
        m = hrnet.HRNetBackbone(sd, max_batch=8, micro_batch=mb) if mb is not None else hrnet.HRNetBackbone(sd, max_batch=8)
        outs[name] = [m.forward(xb).clone() for _ in range(2)]
        torch.cuda.synchronize()
    ref = outs["plain"][0]
    for k, v in outs.items():
        print(f"NO_TBLOCK64={off} {k}: repeat-equal {torch.equal(v[0], v[1])}, vs plain max "
              f"{(v[0] - ref).abs().max().item():.3g} per-crop {[(v[0][i] - ref[i]).abs().max().item() for i in range(7)]}",
              flush=True)
