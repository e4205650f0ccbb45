"""Summarise a rocprofv3 --stats kernel_stats.csv (top kernels by total time)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:n]:
    name = r['Name'].replace('void mvp::(anonymous namespace)::', '').replace('(mvp::(anonymous namespace)::ConvParams)', '')
    name = name.replace('(anonymous namespace)::', '')[:72]
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {100*float(r['TotalDurationNs'])/tot:5.1f}% "
          f"calls={r['Calls']:>5} avg={float(r['AverageNs'])/1e3:9.1f}us  {name}")
print(f"total {tot/1e6:.2f} ms")
