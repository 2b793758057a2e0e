"""Summarise a rocprofv3 *_kernel_stats.csv per training step."""
import csv
import sys

path, steps = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:9.2f} ms/step {int(r['Calls'])/steps:7.0f} calls "
          f"avg {float(r['AverageNs'])/1e3:9.1f} us {float(r['Percentage']):5.1f}%  {r['Name'][:100]}")
print(f"total kernel time per step: {tot/1e6/steps:.2f} ms")
