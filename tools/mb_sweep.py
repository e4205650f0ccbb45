"""Backbone forward time (HIP events) for several micro-batch segment configs."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import torch  # noqa: E402

from mvpose import hrnet  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
configs = [json.loads(a) for a in sys.argv[2:]] or [{}]
sd = hrnet.random_state_dict(0)
x = torch.randn((n, 256, 192, 4), device="cuda").bfloat16()
for cfg in configs:
    mb = {"stem": 0, "branch0": 0, "branch1": 0}
    mb.update(cfg)
    bb = hrnet.HRNetBackbone(sd, max_batch=n, micro_batch=mb)
    out = bb.forward(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        bb.forward(x, out=out)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"micro_batch": mb, "ms_per_forward": e0.elapsed_time(e1) / 5,
                      "arena_GB": bb.arena_bytes / 1e9}), flush=True)
    del bb
    torch.cuda.empty_cache()
