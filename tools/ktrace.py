#!/usr/bin/env python3
"""Dispatches of a rocprofv3 kernel_trace.csv grouped by (kernel, grid, workgroup): count, mean
and total duration, so that one kernel's launches can be told apart by shape.
usage: ktrace.py TRACE_CSV [name-substring] [batches] [N]"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
per = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
n = int(sys.argv[4]) if len(sys.argv) > 4 else 40
groups = defaultdict(list)
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    if pat and pat not in name:
        continue
    key = (name[:70], int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), int(r.get("Grid_Size_Y", 1)),
           int(r.get("Grid_Size_Z", 1)), int(r["Workgroup_Size_X"]), int(r.get("LDS_Block_Size", 0) or 0))
    groups[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in groups.values())
print(f"total {tot / per / 1e6:.3f} ms per unit ({per:g} units)")
print(f"{'kernel':70s} {'wgs_x':>6s} {'gy':>5s} {'gz':>4s} {'wg':>4s} {'lds':>6s} {'n/unit':>7s} {'mean us':>8s} {'ms/unit':>8s}")
for k, v in sorted(groups.items(), key=lambda kv: -sum(kv[1]))[:n]:
    print(f"{k[0]:70s} {k[1]:6d} {k[2]:5d} {k[3]:4d} {k[4]:4d} {k[5]:6d} {len(v) / per:7.1f} {sum(v) / len(v) / 1e3:8.1f} {sum(v) / per / 1e6:8.3f}")
