"""Dispatch-ordered kernel durations of the LAST backbone forward in a rocprofv3
kernel trace (tools/prof_backbone.py under --kernel-trace):

    python tools/op_times.py run_kernel_trace.csv [n_ops_per_forward]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "rocclr" not in r["Kernel_Name"] and "at::" not in r["Kernel_Name"]]
n = int(sys.argv[2]) if len(sys.argv) > 2 else len(rows) // 2
last = rows[-n:]
t0 = int(last[0]["Start_Timestamp"])
tot = 0.0
for i, r in enumerate(last):
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    name = r["Kernel_Name"].replace("void mvp::(anonymous namespace)::", "").replace("mvp::", "")[:70]
    print(f"{i:4d} {(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {d:8.1f} us  {name}")
print(f"sum {tot / 1e3:.3f} ms over {len(last)} dispatches; wall {(int(last[-1]['End_Timestamp']) - t0) / 1e6:.3f} ms")
