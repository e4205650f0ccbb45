"""Backbone throughput: one 1,024-crop forward vs two 512-crop forwards on two streams (two
graphs, two arenas) — whether overlapping the launches' ramps and tails pays.
    python tools/two_stream_probe.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"))
import torch  # noqa: E402

from mvpose import hrnet  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
sd = hrnet.random_state_dict(0)
n = 1024
x = torch.randn((n, 256, 192, 4), device="cuda").bfloat16()
one = hrnet.HRNetBackbone(sd, max_batch=n)
halves = [hrnet.HRNetBackbone(sd, max_batch=n // 2) for _ in range(2)]
streams = [torch.cuda.Stream() for _ in range(2)]
outs = [None, None]


def run_one():
    one.forward(x)


def run_two():
    cur = torch.cuda.current_stream()
    for i in range(2):
        streams[i].wait_stream(cur)
        with torch.cuda.stream(streams[i]):
            outs[i] = halves[i].forward(x[i * n // 2:(i + 1) * n // 2])
    for i in range(2):
        cur.wait_stream(streams[i])


for name, f in (("one 1024", run_one), ("two 512 x 2 streams", run_two)) * 2:
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name}: {e0.elapsed_time(e1) / reps:.3f} ms per 1,024 crops", flush=True)
