#!/usr/bin/env python3
"""Top kernels of a rocprofv3 --stats kernel_stats.csv, per step (usage: kstats.py CSV STEPS [N])."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
n = int(sys.argv[3]) if len(sys.argv) > 3 else 30
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / steps / 1e6:.3f} ms/step")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{float(r['TotalDurationNs']) / steps / 1e6:8.3f} ms/step {int(r['Calls']) / steps:7.1f} calls/step "
          f"{float(r['AverageNs']) / 1e3:8.1f} us  {r['Name'][:110]}")
