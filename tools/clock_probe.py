#!/usr/bin/env python3
"""Effective clock per kernel from a rocprofv3 GRBM_GUI_ACTIVE pass (MI355X_MICROARCH.md
'DVFS give-back': clock = GRBM_GUI_ACTIVE / 8 XCDs / dispatch wall time; reads high on
dispatches shorter than ~0.3 ms).

usage: clock_probe.py DIR [--match SUBSTR] -> per kernel: dispatches, median duration (us),
median effective clock (GHz), and the same for the longest dispatches.
"""
import argparse
import csv
import glob
import os
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    per = defaultdict(list)  # kernel -> [(dur_ns, ghz)]
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
                    continue
                k = r["Kernel_Name"]
                if a.match and a.match not in k:
                    continue
                dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                if dur <= 0:
                    continue
                per[k].append((dur, float(r["Counter_Value"]) / 8.0 / dur))
    for k, v in sorted(per.items(), key=lambda kv: -sum(d for d, _ in kv[1])):
        durs = [d for d, _ in v]
        ghz = [g for _, g in v]
        print(f"{len(v):5d}  dur {statistics.median(durs) / 1e3:9.1f} us  clock {statistics.median(ghz):5.3f} GHz "
              f"(min {min(ghz):5.3f} max {max(ghz):5.3f})  {k[:110]}")


if __name__ == "__main__":
    main()
