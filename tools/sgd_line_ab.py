"""bench.py's config-5 SGD line (device-resident inputs, HIP-event timing, parity asserted against
tests/golden/bench_sgd_c5.npz) for the library MVPOSE_LIB names: one JSON line.
    MVPOSE_LIB=.../libX.so python tools/sgd_line_ab.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multi-camera_3d_pose_estimation_amd")]
import bench  # noqa: E402

r = bench.sgd_line("cuda:0")
print(json.dumps({"lib": os.environ.get("MVPOSE_LIB", "libmvpose.so"), "ms_1": r["ms_per_iter_1traj"],
                  "ms_M": r["ms_per_iter_M"], "frac": r["roofline"]["frac"], "dev": r["parity"]["max_abs_cm_vs_reference"]}))
