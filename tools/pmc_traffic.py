#!/usr/bin/env python3
"""HBM traffic per GEMM launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE)
over the same command (scripts/gpu_counters.sh with PMC_GROUPS=scripts/pmc_traffic.txt).

Corrections (MI355X_MICROARCH.md, HBM section): both counters are in KiB; on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced streaming read (16 B per lane,
global_load_lds / buffer_load ... lds alike -- how every GEMM operand tile is staged),
so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores (the GEMM epilogue).
Infinity-Cache hits are counted, so tile re-reads absorbed on-die still show up here.

usage: pmc_traffic.py FETCH_DIR WRITE_DIR [--match ...] [--out FILE] [--cmd TEXT]
The output records src_hash (bench.kernel_source_hash() of this tree): bench.py reports the
traffic only while the GEMM sources still hash to it.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def per_dispatch(d, counter, match):
    vals, names = defaultdict(float), {}
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    for f in files:
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != counter or not any(m in r["Kernel_Name"] for m in match):
                    continue
                key = (f, int(r["Dispatch_Id"]))
                vals[key] += float(r["Counter_Value"])
                names[key] = r["Kernel_Name"]
    return vals, names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--match", default="gemm_bf16_kernel,gemm_s64_kernel,gemm8p_kernel,gemm8q_kernel,act_pass_kernel,splitk_reduce_kernel,colsum_finish_kernel")
    ap.add_argument("--out")
    ap.add_argument("--cmd", default="")
    a = ap.parse_args()
    match = a.match.split(",")
    fv, fn = per_dispatch(a.fetch_dir, "FETCH_SIZE", match)
    wv, _ = per_dispatch(a.write_dir, "WRITE_SIZE", match)
    nf, nw = len(fv), len(wv)
    # per GEMM launch: all matched dispatches' bytes (the GEMM kernel and its companions -- the
    # split-K reduce, the column-sum finish, the activation pass) over the number of GEMM-kernel
    # dispatches, i.e. one capk_gemm call's HBM traffic
    primary = ("gemm_bf16_kernel", "gemm_s64_kernel", "gemm8p_kernel", "gemm8q_kernel")
    npf = sum(1 for k in fv if any(m in fn[k] for m in primary)) or nf
    _, wn = per_dispatch(a.write_dir, "WRITE_SIZE", match)
    npw = sum(1 for k in wv if any(m in wn[k] for m in primary)) or nw
    fetch = 2.0 * 1024.0 * sum(fv.values()) / max(npf, 1)
    write = 1024.0 * sum(wv.values()) / max(npw, 1)
    by_kernel = defaultdict(lambda: [0, 0.0])
    for k, v in fv.items():
        e = by_kernel[fn[k][:90]]
        e[0] += 1
        e[1] += 2.0 * 1024.0 * v
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    res = {"counters": ["FETCH_SIZE", "WRITE_SIZE"], "kernels_matched": match, "command": a.cmd,
           "src_hash": bench.kernel_source_hash(),
           "dispatches_fetch_pass": nf, "dispatches_write_pass": nw,
           "gemm_launches_fetch_pass": npf, "gemm_launches_write_pass": npw,
           "avg_fetch_bytes": fetch, "avg_write_bytes": write, "avg_hbm_bytes": fetch + write,
           "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 reports half of 16-B/lane streaming reads); WRITE_SIZE KiB x1024",
           "fetch_by_kernel": {k: {"dispatches": n, "avg_fetch_bytes": b / n} for k, (n, b) in sorted(by_kernel.items())}}
    s = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
