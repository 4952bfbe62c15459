"""Summarise a rocprofv3 --kernel-trace --stats CSV directory: top kernels by total time."""
import csv
import glob
import sys

d = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
f = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total kernel time {tot/1e6:.2f} ms ({tot/1e6/steps:.2f} ms per step over {steps:g} steps)")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    name = r['Name'].replace('(anonymous namespace)::', '')
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} ms/step {int(r['Calls'])/steps:7.1f} calls/step "
          f"{float(r['AverageNs'])/1e3:8.1f} us avg {float(r['Percentage']):5.1f}%  {name[:90]}")
