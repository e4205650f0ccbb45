"""cProfile of refine_trajectories' host side (config-5 problem, 20 calls, max_iter 0)."""
import cProfile
import json
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mvpose import refine  # noqa: E402
from sgd_problem import BENCH_C5_KW, bench_c5_inputs  # noqa: E402

cams, g, x0 = bench_c5_inputs(8, 400)
with open(os.path.join(ROOT, "tests", "golden", "body_part_lengths.json")) as f:
    lengths = json.load(f)["my_lengths"]
camlist = [[c["K"], c["R"], c["T"], c["dist"]] for c in cams]
kw = dict(BENCH_C5_KW, body_lengths=dict(lengths), device="cuda:0")
kw["max_iter"] = 0
G = torch.tensor(np.broadcast_to(g, (256,) + g.shape).copy(), device="cuda:0")
X = torch.tensor(np.broadcast_to(x0, (256,) + x0.shape).copy(), device="cuda:0")
for _ in range(3):
    refine.refine_trajectories(G, X, camlist, **kw)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    refine.refine_trajectories(G, X, camlist, **kw)
    torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("cumtime").print_stats(25)
