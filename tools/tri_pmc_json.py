"""Summarise rocprofv3 --pmc passes of one kernel into a profiles/*_pmc.json record.

    python tools/tri_pmc_json.py KERNEL_SUBSTR OUT.json [--points N] pass1/run_counter_collection.csv [pass2 ...]

Per pass: the kernel's dispatches, their counters summed, and each dispatch's duration from the
CSV's own Start/End timestamps.  Derived (MI355X_MICROARCH.md, "DVFS give-back"):
  clock_GHz      = GRBM_GUI_ACTIVE / 8 XCDs / duration (per dispatch, then the median);
  valu_busy      = SQ_ACTIVE_INST_VALU x 4 cycles / 1,024 SIMDs / (GRBM_GUI_ACTIVE / 8): the
                   fraction of each SIMD's cycles the kernel spent issuing VALU instructions;
  per_wave       = every counter / SQ_WAVES;
  per_64_points  = every counter per 64 points (--points N = points per dispatch; a grid-stride
                   kernel's waves each handle many points, so per_wave is not per point).
The bench's `valu_issue` and DESIGN.md quote these numbers from the same file."""
import csv
import json
import statistics
import sys
from collections import defaultdict

sub, out_path, passes = sys.argv[1], sys.argv[2], sys.argv[3:]
points = None
if passes and passes[0] == "--points":
    points, passes = int(passes[1]), passes[2:]
counters = defaultdict(float)
durations, clocks = [], []
dispatches = set()
for path in passes:
    per = defaultdict(dict)
    span = {}
    for r in csv.DictReader(open(path)):
        if sub not in r["Kernel_Name"]:
            continue
        d = (path, r["Dispatch_Id"])
        per[d][r["Counter_Name"]] = float(r["Counter_Value"])
        span[d] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    for d, cs in per.items():
        for k, v in cs.items():
            if k == "GRBM_GUI_ACTIVE" and k in counters and path != passes[0]:
                continue  # GRBM is collected in every pass; keep the first pass's
            counters[k] += v
        dur = (span[d][1] - span[d][0]) * 1e-9
        durations.append(dur)
        if "GRBM_GUI_ACTIVE" in cs and dur > 0:
            clocks.append(cs["GRBM_GUI_ACTIVE"] / 8 / dur / 1e9)
        dispatches.add(d)
n_first = sum(1 for d in dispatches if d[0] == passes[0])
waves = counters.get("SQ_WAVES", 0)
res = {"source": f"rocprofv3 --kernel-trace --pmc, {len(passes)} pass(es): " + ", ".join(passes),
       "kernel": sub, "dispatches_per_pass": n_first, "counters": dict(counters)}
if waves:
    res["per_wave"] = {k: v / waves for k, v in counters.items() if k.startswith("SQ_") and k != "SQ_WAVES"}
if points:
    groups = n_first * points / 64.0
    res["points_per_dispatch"] = points
    res["per_64_points"] = {k: v / groups for k, v in counters.items() if k.startswith("SQ_") and k != "SQ_WAVES"}
if clocks:
    res["clock_GHz_median"] = statistics.median(clocks)
    res["duration_ms_median"] = statistics.median(durations) * 1e3
if "SQ_ACTIVE_INST_VALU" in counters and "GRBM_GUI_ACTIVE" in counters:
    res["valu_busy"] = counters["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (counters["GRBM_GUI_ACTIVE"] / 8)
res["note"] = ("SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES / SQ_WAIT_* count quad-cycles; GRBM_GUI_ACTIVE is summed over the "
               "8 XCDs (MI355X_MICROARCH.md)")
json.dump(res, open(out_path, "w"), indent=1)
print(json.dumps({k: res[k] for k in ("dispatches_per_pass", "clock_GHz_median", "duration_ms_median", "valu_busy")
                  if k in res}))
