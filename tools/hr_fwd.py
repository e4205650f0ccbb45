"""HRNet-W32 backbone forwards only (for kernel traces and the per-forward breakdown):
    python tools/hr_fwd.py [CROPS=1024] [PLAN_OUT.npz]
3 warm-up forwards, then 10 forwards timed with HIP events on the launch stream (torch's
current stream, which mvp_graph_forward runs on).  With PLAN_OUT, saves the graph's launch
plan (mvp_graph_plan: launching op, route, crops, MACs per kernel launch) and the timing, for
tools/fwd_breakdown.py to pair with the trace's last forward."""
import os, sys, torch
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multi-camera_3d_pose_estimation_amd"))
from mvpose import hrnet
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
m = hrnet.HRNetBackbone(seed=0, max_batch=n)
x = torch.randn((n, 256, 192, 4), device="cuda").bfloat16()
for _ in range(3):
    m.forward(x)
torch.cuda.synchronize()
reps = 10
ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
ev[0].record()
for i in range(reps):
    m.forward(x)
    ev[i + 1].record()
torch.cuda.synchronize()
ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(reps)]
print(f"forward {n} crops: HIP events mean {np.mean(ms):.3f} ms, min {np.min(ms):.3f}, max {np.max(ms):.3f}")
if len(sys.argv) > 2:
    np.savez(sys.argv[2], plan=m.launch_plan(n), event_ms=np.array(ms), crops=n,
             macs_per_crop=m.macs_per_crop())
print("ok")
