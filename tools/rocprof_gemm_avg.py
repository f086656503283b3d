#!/usr/bin/env python3
"""Cross-check bench.py's live GEMM roofline against a rocprofv3 --kernel-trace --stats
summary of the same command: average GEMM launch duration = (total time of the GEMM
kernels, split-K reduce included) / (number of GEMM launches), over every step rocprof
saw (warm-up steps have the same launches as timed ones, so the average is comparable
with bench.py's roofline.avg_launch_ms).

usage: rocprof_gemm_avg.py KERNEL_STATS_CSV [BENCH_JSON] [--out FILE]
"""
import csv
import json
import sys

MAIN = ("gemm_bf16_kernel", "gemm256_kernel", "Cijk_")
AUX = ("splitk_reduce_kernel", "act_pass_kernel")  # both launched inside capk_gemm (gemm.hip)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    if out in args:
        args.remove(out)
    tot_ns, n_main, by = 0.0, 0, {}
    with open(args[0], newline="") as f:
        for r in csv.DictReader(f):
            name = r["Name"]
            if any(m in name for m in MAIN + AUX):
                tot_ns += float(r["TotalDurationNs"])
                key = ("hipblaslt" if "Cijk_" in name else "splitk_reduce" if "splitk" in name
                       else "act_pass" if "act_pass" in name else "gemm_bf16_kernel")
                e = by.setdefault(key, [0, 0.0])
                e[0] += int(r["Calls"])
                e[1] += float(r["TotalDurationNs"])
                if any(m in name for m in MAIN):
                    n_main += int(r["Calls"])
    res = {"rocprof_gemm_launches": n_main, "rocprof_gemm_total_ms": tot_ns / 1e6,
           "rocprof_avg_launch_ms": tot_ns / 1e6 / max(n_main, 1),
           "by_kind": {k: {"calls": v[0], "total_ms": v[1] / 1e6} for k, v in by.items()}}
    if len(args) > 1:
        with open(args[1]) as f:
            line = [ln for ln in f if ln.startswith("{")][-1]
        rf = json.loads(line)["roofline"]
        res["bench_avg_launch_ms"] = rf["avg_launch_ms"]
        res["ratio_rocprof_over_bench"] = res["rocprof_avg_launch_ms"] / rf["avg_launch_ms"]
    s = json.dumps(res, indent=1)
    if out:
        with open(out, "w") as f:
            f.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
