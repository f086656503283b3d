#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 PMC passes (counter_collection.csv files under the
given directories), with the derived ratios used in DESIGN.md:

  mfma_util   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 4 SIMDs * 32 CUs) per-XCD-normalised
                (reported raw too; counters are summed over the chip)
  wait_any    = SQ_WAIT_ANY / SQ_WAVE_CYCLES   (waves parked: s_waitcnt / barrier)
  wait_inst   = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES, lds_issue = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES
  fetch_bytes = FETCH_SIZE KiB x 1024 x 2 (gfx950 half-counts 16-B/lane streaming reads,
                MI355X_MICROARCH.md HBM section); write_bytes = WRITE_SIZE KiB x 1024

usage: pmc_summary.py DIR [DIR ...] [--match SUBSTR[,SUBSTR]] [--json OUT]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(dirs, match):
    acc = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per-dispatch values]
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(float)
            names = {}
            with open(f, newline="") as fh:
                for r in csv.DictReader(fh):
                    k = r["Kernel_Name"]
                    if match and not any(m in k for m in match):
                        continue
                    key = (int(r["Dispatch_Id"]), r["Counter_Name"])
                    per[key] += float(r["Counter_Value"])
                    names[int(r["Dispatch_Id"])] = k
            for (disp, cn), v in per.items():
                acc[names[disp]][cn].append(v)
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="")
    ap.add_argument("--json")
    a = ap.parse_args()
    match = [m for m in a.match.split(",") if m]
    acc = load(a.dirs, match)
    out = {}
    for k, cs in acc.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        d = {"dispatches": max(len(v) for v in cs.values()), "avg": avg}
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for c, n in (("SQ_WAIT_ANY", "wait_any"), ("SQ_WAIT_INST_ANY", "wait_inst"),
                         ("SQ_ACTIVE_INST_ANY", "active_inst"), ("SQ_WAIT_INST_LDS", "lds_issue")):
                if c in avg:
                    d[n] = avg[c] / wc
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "SQ_BUSY_CYCLES" in avg:
            d["mfma_busy_per_busy_cycle"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / avg["SQ_BUSY_CYCLES"]
        if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_LDS_IDX_ACTIVE" in avg and avg["SQ_LDS_IDX_ACTIVE"]:
            d["lds_conflict_frac"] = avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"]
        if "FETCH_SIZE" in avg:
            d["fetch_bytes"] = avg["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in avg:
            d["write_bytes"] = avg["WRITE_SIZE"] * 1024
        if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
            d["l2_hit"] = avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
        out[k] = d
    for k, d in sorted(out.items(), key=lambda kv: kv[0]):
        print(k[:100])
        print("   ", json.dumps({x: (round(y, 4) if isinstance(y, float) else y) for x, y in d.items() if x != "avg"}))
        print("    avg:", json.dumps({x: round(y) for x, y in d["avg"].items()}))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
