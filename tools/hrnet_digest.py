"""SHA-256 of an HRNet-W32 backbone forward (random-init weights, seeded crops) for the library
MVPOSE_LIB names: bit-identity checks between two builds.
    MVPOSE_LIB=.../libX.so python tools/hrnet_digest.py [crops]"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import torch  # noqa: E402
from mvpose import hrnet  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
g = torch.Generator().manual_seed(21)
x = torch.randn((n, 256, 192, 4), generator=g).bfloat16().cuda()
bb = hrnet.HRNetBackbone(hrnet.random_state_dict(0), max_batch=n)
y = bb.forward(x)
torch.cuda.synchronize()
h = hashlib.sha256(y.float().cpu().numpy().tobytes()).hexdigest()
print(f"{os.path.basename(os.environ.get('MVPOSE_LIB', 'libmvpose.so'))} backbone n={n} sha256 {h}")
