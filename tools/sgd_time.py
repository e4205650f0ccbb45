"""Config-5 SGD timing without the parity assertion (for ablation variants): bench.py's problem,
M trajectories per launch, HIP events around the refine call and around the kernel launch alone.
    MVPOSE_LIB=.../libX.so python tools/sgd_time.py [M]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from mvpose import refine  # noqa: E402
from sgd_problem import BENCH_C5_KW, bench_c5_inputs  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else bench.SGD_M
dev = "cuda:0"
cams, g, x0 = bench_c5_inputs(bench.SGD_V, bench.SGD_T)
with open(os.path.join(ROOT, "tests", "golden", "body_part_lengths.json")) as f:
    lengths = json.load(f)["my_lengths"]
camlist = [[c["K"], c["R"], c["T"], c["dist"]] for c in cams]
kw = dict(BENCH_C5_KW, body_lengths=dict(lengths), device=dev)
G = torch.tensor(np.broadcast_to(g, (M,) + g.shape).copy(), device=dev)
X = torch.tensor(np.broadcast_to(x0, (M,) + x0.shape).copy(), device=dev)
s = torch.cuda.current_stream()
k0, k1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
orig = refine.call


def timed_call(name, *a):
    if name.startswith("mvp_sgd_refine"):
        k0.record(s)
        r = orig(name, *a)
        k1.record(s)
        return r
    return orig(name, *a)


refine.call = timed_call
res = []
for rep in range(4):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    r = refine.refine_trajectories(G, X, camlist, **kw)
    e1.record(s)
    torch.cuda.synchronize()
    if rep:
        res.append((e0.elapsed_time(e1) / bench.SGD_ITERS, k0.elapsed_time(k1) / bench.SGD_ITERS))
dev_max = float(np.abs(r["final"].cpu().numpy() - np.load(os.path.join(ROOT, "tests", "golden", "bench_sgd_c5.npz"))["final"]).max())
print(json.dumps({"lib": os.path.basename(os.environ.get("MVPOSE_LIB", "libmvpose.so")), "M": M,
                  "ms_call": float(np.median([a for a, _ in res])), "ms_kernel": float(np.median([b for _, b in res])),
                  "dev": dev_max}))
