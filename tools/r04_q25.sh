#!/bin/bash
# SGD phase costs (timing only, wrong trajectories): no pass-A camera loop (dA), no pass-B
# point loop (dB), no Adam trajectory loop (dC) vs shipped (libJ); bench config-5 timing
set -o pipefail
for L in libJ lib_dA lib_dB lib_dC libJ; do
  MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/$L.so timeout -k 10 240 python3 - <<'PY' 2>/dev/null | tail -1
import os, sys, json, time
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "multi-camera_3d_pose_estimation_amd"), os.path.join(os.getcwd(), "tests")]
import numpy as np, torch
import bench
from mvpose import refine
from sgd_problem import BENCH_C5_KW, bench_c5_inputs
cams, g, x0 = bench_c5_inputs(8, 400)
import json as _j
lengths = _j.load(open("tests/golden/body_part_lengths.json"))["my_lengths"]
camlist = [[c["K"], c["R"], c["T"], c["dist"]] for c in cams]
kw = dict(BENCH_C5_KW, body_lengths=dict(lengths), device="cuda:0")
M = 256
G = torch.tensor(np.broadcast_to(g, (M,) + g.shape).copy(), device="cuda:0")
X = torch.tensor(np.broadcast_to(x0, (M,) + x0.shape).copy(), device="cuda:0")
refine.refine_trajectories(G, X, camlist, **kw)
s = torch.cuda.current_stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
r = refine.refine_trajectories(G, X, camlist, **kw)
e1.record(s)
torch.cuda.synchronize()
print(json.dumps({"lib": os.environ["MVPOSE_LIB"].split("/")[-1], "ms_per_iter_M256": e0.elapsed_time(e1) / 40}))
PY
done
