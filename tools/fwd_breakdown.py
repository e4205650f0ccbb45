"""Per-kernel-family breakdown of ONE HRNet-W32 forward from a rocprofv3 kernel trace of
tools/hr_fwd.py (backbone forwards only: no detector, no small-batch forwards in the trace):
    python tools/fwd_breakdown.py run_kernel_trace.csv plan.npz [OUT.json]
The last len(plan) kernels of the trace are the last forward; the plan (mvp_graph_plan) gives
each launch's MACs, so each family gets launches per forward, µs, GFLOP and its fraction of
dense bf16 MFMA peak.  The forward's 13 timed repeats (warm-up aside) are checked to launch the
same kernel sequence, and the per-family times are averaged over the traced forwards."""
import collections
import csv
import json
import re
import sys

import numpy as np

PEAK = 2500.0  # dense bf16 TFLOP/s (MI355X_MICROARCH.md)
ROUTES = {1: "BasicBlock", 2: "transition twin", 3: "s2 siblings", 4: "head + fuse", 5: "Bottleneck",
          6: "stem pair", 7: "stem", 8: "conv", 9: "1x1 pair", 10: "fuse sum"}

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
z = np.load(sys.argv[2])
plan, ev_ms, crops = z["plan"], z["event_ms"], int(z["crops"])
L = len(plan)


def fam(r):
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", n).replace("mvp::", "")[:64]


# the traced forwards: walk back from the end in blocks of L while the name sequence repeats
last = rows[-L:]
names = [fam(r) for r in last]
fwds = [last]
while len(rows) >= (len(fwds) + 1) * L:
    blk = rows[-(len(fwds) + 1) * L:-len(fwds) * L]
    if [fam(r) for r in blk] != names:
        break
    fwds.append(blk)
agg = collections.OrderedDict()
for i, nm in enumerate(names):
    key = (nm, int(last[i]["Grid_Size_X"]) if "Grid_Size_X" in last[i] else 0)
    a = agg.setdefault(key, dict(n=0, us=0.0, macs=0, routes=set()))
    a["n"] += 1
    a["macs"] += int(plan[i, 3])
    a["routes"].add(ROUTES[int(plan[i, 1])])
    a["us"] += np.mean([(int(f[i]["End_Timestamp"]) - int(f[i]["Start_Timestamp"])) / 1e3 for f in fwds])
walls = [(int(f[-1]["End_Timestamp"]) - int(f[0]["Start_Timestamp"])) / 1e3 for f in fwds]
tot_us = sum(a["us"] for a in agg.values())
tot_flop = 2.0 * plan[:, 3].sum()
lines = [f"HRNet-W32 forward, {crops} crops: {L} launches, {len(fwds)} traced forwards averaged; "
         f"{tot_flop / 1e12:.3f} TFLOP per forward ({2.0 * z['macs_per_crop'] / 1e9:.2f} GFLOP per crop)",
         f"{'us':>9} {'share':>6} {'n':>3} {'us/launch':>9} {'GFLOP':>8} {'TFLOP/s':>8} {'MFMA%':>6}  grid      kernel [graph route]"]
out = []
for (nm, gx), a in sorted(agg.items(), key=lambda kv: -kv[1]["us"]):
    gf = 2.0 * a["macs"] / 1e9
    tf = gf / 1e3 / (a["us"] * 1e-6) if a["us"] else 0.0
    lines.append(f"{a['us']:9.1f} {100 * a['us'] / tot_us:5.1f}% {a['n']:3d} {a['us'] / a['n']:9.1f} {gf:8.1f} "
                 f"{tf:8.1f} {100 * tf / PEAK:5.1f}%  {gx:<9} {nm} [{', '.join(sorted(a['routes']))}]")
    out.append(dict(kernel=nm, grid=gx, launches=a["n"], us=a["us"], gflop=gf, tflops=tf, mfma_frac=tf / PEAK,
                    routes=sorted(a["routes"])))
ev = float(np.mean(ev_ms))
wall = float(np.mean(walls))
lines.append(f"sum of kernel times {tot_us / 1e3:.3f} ms; trace wall {wall / 1e3:.3f} ms per forward; "
             f"HIP-event forward (untraced, 10 repeats) {ev:.3f} ms: kernels sum to {100 * tot_us / 1e3 / ev:.1f} % of it")
lines.append(f"forward: {tot_flop / 1e12 / (ev * 1e-3):.1f} TFLOP/s = {100 * tot_flop / 1e12 / (ev * 1e-3) / PEAK:.1f} % "
             f"of dense bf16 peak ({PEAK:.0f})")
print("\n".join(lines))
if len(sys.argv) > 3:
    json.dump(dict(crops=crops, launches=L, traced_forwards=len(fwds), tflop_per_forward=tot_flop / 1e12,
                   kernel_sum_ms=tot_us / 1e3, trace_wall_ms=wall / 1e3, event_ms=ev, families=out),
              open(sys.argv[3], "w"), indent=1)
