"""Run the HRNet backbone forward a few times (for rocprofv3 counter passes)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import torch
from mvpose import hrnet
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
bb = hrnet.HRNetBackbone(hrnet.random_state_dict(0), max_batch=n)
x = torch.randn((n, 256, 192, 4), device="cuda").bfloat16()
for _ in range(reps):
    bb.forward(x)
torch.cuda.synchronize()
print("done")
