#!/usr/bin/env python3
"""Per-case table from scripts/gpu_r4_traffic.sh output: for each case and kernel, the median
over the case's timed launches of FETCH_SIZE (x2, the gfx950 streaming-read correction of
MI355X_MICROARCH.md's HBM section), WRITE_SIZE and the L2 hit rate, against the algorithmic
bytes of tools/traffic_calib.py.  Counters are KiB.  The 512 MiB uint8 fill that flushes the
Infinity Cache between launches is excluded; the L2-miss model column is l2_model().

usage: traffic_table.py OUT_DIR"""
import csv
import glob
import json
import os
import statistics
import subprocess
import sys
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))


def dispatches(d, counters):
    """{dispatch_id: (kernel, {counter: value})} of every counter_collection.csv under d."""
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] not in counters:
                    continue
                key = int(r["Dispatch_Id"])
                name, vals = out.setdefault(key, (r["Kernel_Name"], defaultdict(float)))
                vals[r["Counter_Name"]] += float(r["Counter_Value"])
    return out


KEEP = {"copy": ("copy",), "fill": ("FillFunctor",), "read": ("reduce_kernel",),
        "gemm": ("gemm8q_kernel", "gemm8p_kernel", "gemm_bf16_kernel", "splitk_reduce_kernel", "colsum_finish_kernel")}


def l2_model(kind, M, N, K, cap=4 << 20):
    """Predicted L2-miss bytes of one gemm8q launch: each XCD runs rounds of 32 consecutive
    row-major tiles (WG b: items (b & 7) * 32 + (b >> 3) + 256 j); a round touches its tiles'
    A row blocks and B column blocks (256 x K bf16 each), kept in an LRU of the XCD's 4 MiB
    L2 across rounds; side operands (residual / aux) are read once."""
    if kind in ("copy", "fill", "read", "dw"):
        return None
    ntm, ntn = -(-M // 256), -(-N // 256)
    items, blk = ntm * ntn, 256 * K * 2
    total = 0
    for x in range(8):
        lru = []
        for j in range(0, items, 256):
            touched = []
            for i in range(32):
                it = j + x * 32 + i
                if it < items:
                    touched += [("A", it // ntn), ("B", it % ntn)]
            for t in dict.fromkeys(touched):
                if t in lru:
                    lru.remove(t)
                else:
                    total += blk
                lru.append(t)
                while len(lru) * blk > cap:
                    lru.pop(0)
    side = 2 * M * N if ("res" in kind or kind == "dx_dsum") else 0
    return total + side


def short(name):
    n = name.split("(")[0]
    for k in ("gemm8q_kernel", "gemm8p_kernel", "gemm_bf16_kernel", "splitk_reduce_kernel", "colsum_finish_kernel",
              "copy", "fill", "reduce_kernel", "FillFunctor", "elementwise"):
        if k in name:
            return k + ("<" + n.split("<", 1)[1][:40] if "<" in n and k.startswith("gemm") else "")
    return n[:60]


def main():
    out = sys.argv[1]
    alg = json.loads(subprocess.check_output([sys.executable, os.path.join(HERE, "traffic_calib.py"), "--list"]))
    sys.path.insert(0, HERE)
    import traffic_calib
    rows = []
    for case, a in alg.items():
        per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values
        for pn, counters in (("FETCH_SIZE", ["FETCH_SIZE"]), ("WRITE_SIZE", ["WRITE_SIZE"]),
                             ("TCC_HIT_sum_TCC_MISS_sum", ["TCC_HIT_sum", "TCC_MISS_sum"])):
            d = os.path.join(out, case, pn)
            if not os.path.isdir(d):
                continue
            keep = KEEP.get(a["kind"], KEEP["gemm"])
            for _, (name, vals) in sorted(dispatches(d, counters).items()):
                if "FillFunctor<unsigned char>" in name or not any(m in name for m in keep):  # cache flush / input set-up
                    continue
                for c, v in vals.items():
                    per[short(name)][c].append(v)
        kind, M, N, K = traffic_calib.CASES[case]
        model = l2_model(kind, M, N, K)
        for k, cv in per.items():
            # the case's last 3 launches (after one warm-up launch)
            med = lambda c: statistics.median(cv[c][-3:]) if cv.get(c) else None
            f, w, h, m = med("FETCH_SIZE"), med("WRITE_SIZE"), med("TCC_HIT_sum"), med("TCC_MISS_sum")
            rows.append((case, k, a["read"] / 1e6, None if f is None else 2 * f * 1024 / 1e6,
                         None if model is None or not k.startswith("gemm8q") else model / 1e6, a["write"] / 1e6,
                         None if w is None else w * 1024 / 1e6, None if h is None or h + m == 0 else h / (h + m)))
    fmt = lambda x, p=1: "-" if x is None else f"{x:.{p}f}"
    print("| case | kernel | alg. read MB | FETCH_SIZE x2 MB | ratio | L2-miss model MB | measured / model "
          "| alg. write MB | WRITE_SIZE MB | ratio | L2 hit |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for case, k, ar, f, mo, aw, w, h in rows:
        rr = None if f is None or ar == 0 else f / ar
        rm = None if f is None or mo is None else f / mo
        rw = None if w is None or aw == 0 else w / aw
        print(f"| {case} | `{k}` | {fmt(ar)} | {fmt(f)} | {fmt(rr, 2)} | {fmt(mo)} | {fmt(rm, 2)} | {fmt(aw)} | {fmt(w)} "
              f"| {fmt(rw, 2)} | {fmt(h, 3)} |")


if __name__ == "__main__":
    main()
