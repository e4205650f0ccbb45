"""Per-kernel-family breakdown of the LAST backbone forward in a rocprofv3 kernel trace
(tools/prof_backbone.py under --kernel-trace):
    python tools/fwd_breakdown.py run_kernel_trace.csv"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "stem2_kernel" in r["Kernel_Name"]]
a = starts[-1]
b = next((i for i in range(a, len(rows)) if "head1x1" in rows[i]["Kernel_Name"] or "head_fuse" in rows[i]["Kernel_Name"]), len(rows) - 1)
seg = rows[a:b + 1]
fam = collections.defaultdict(lambda: [0, 0.0])
for r in seg:
    n = re.sub(r"\(mvp::.*|\(unsigned.*", "", r["Kernel_Name"]).replace("void ", "")
    n = n.replace("mvp::(anonymous namespace)::", "")[:60]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    fam[(n, r["Grid_Size_X"])][0] += 1
    fam[(n, r["Grid_Size_X"])][1] += d
wall = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in fam.values())
for (n, gx), (c, d) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
    print(f"{d:9.1f} us {c:3d} x {d / c:7.1f}  grid {gx:>9}  {n}")
print(f"sum {tot / 1e3:.3f} ms over {len(seg)} launches; wall {wall / 1e3:.3f} ms")
