"""Print a rocprofv3 kernel_stats.csv as per-step milliseconds (top kernels)."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.2f} ms/step n={int(r['Calls'])/steps:6.1f} "
          f"avg={float(r['AverageNs'])/1e3:8.1f}us {r['Name'][:90]}")
print(f"total GPU ms/step {tot/1e6/steps:.2f}")
