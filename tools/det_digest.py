"""SHA-256 of one RTMDet-m forward's candidates and selected boxes (random-init weights, seeded
frames) for the library MVPOSE_LIB names: bit-identity checks between two builds.
    MVPOSE_LIB=.../libX.so python tools/det_digest.py [frames] [size]"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mvpose import rtmdet as D  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
size = int(sys.argv[2]) if len(sys.argv) > 2 else 640
frames = torch.from_numpy(np.random.default_rng(3).integers(0, 256, (n, 720, 1280, 3), dtype=np.uint8)).cuda()
det = D.RTMDetector(D.random_state_dict(0), max_batch=n, size=size)
det.run_ops(frames, 0, len(det.spec.ops))
torch.cuda.synchronize()
h = hashlib.sha256(det.cand[:n].cpu().numpy().tobytes()).hexdigest()
det.close()
print(f"{os.path.basename(os.environ.get('MVPOSE_LIB', 'libmvpose.so'))} cand sha256 {h}")
