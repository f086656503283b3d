"""Known-byte workloads for reconciling the rocprofv3 traffic counters (FETCH_SIZE /
WRITE_SIZE / TCC hit-miss) with algorithmic bytes: streaming copies / fills / reads of
1 GiB, and the config-3 GEMM launches with their epilogues, one case per process
(scripts/gpu_r4_traffic.sh runs every case under each counter pass; tools/traffic_table.py
turns the per-dispatch counters into profiles/round4/gemm_traffic_reconcile.md).

usage: python tools/traffic_calib.py --case NAME [--reps 3]   (--list: case names and bytes)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-captioning-ml-project_amd"))

T = 256 * 197
GiB = 1 << 30
# name: (kind, M, N, K) -- GEMM cases: C[M,N] = A[M,K] B^T (+ epilogue)
CASES = {
    "copy1g": ("copy", 0, 0, 0), "fill1g": ("fill", 0, 0, 0), "read1g": ("read", 0, 0, 0),
    "qkv_fwd": ("fwd", T, 2304, 768), "fc1_gelu_deriv": ("fwd_gelu_deriv", T, 3072, 768),
    "fc2_fwd_res": ("fwd_res", T, 768, 3072), "o_dx": ("dx", T, 768, 768),
    "fc2_dx_dsum": ("dx_dsum", T, 3072, 768), "lm_fwd": ("fwd", 5120, 50304, 768),
    "qkv_dw": ("dw", T, 2304, 768),
}


def algorithmic(kind, M, N, K):
    """(read bytes, write bytes) every launch must move at least once."""
    if kind == "copy":
        return GiB, GiB
    if kind == "fill":
        return 0, GiB
    if kind == "read":
        return GiB, 0
    a, b, c = 2 * M * K, 2 * N * K, 2 * M * N
    if kind == "dw":  # dW[N,K] fp32 = dY[M,N]^T X[M,K]
        return 2 * M * N + 2 * M * K, 4 * N * K
    if kind == "dx_dsum":  # dX[M,N] = dY[M,K] W[K,N] * aux[M,N]; + column-sum partials
        return a + b + c, c
    r = a + b + (c if "res" in kind else 0)
    w = c * (2 if "gelu" in kind else 1)
    return r, w


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--list", action="store_true")
    a = ap.parse_args()
    if a.list:
        print(json.dumps({n: dict(zip(("read", "write"), algorithmic(*v))) | {"kind": v[0]} for n, v in CASES.items()}))
        return
    import torch
    from capk import ops
    from capk._lib import ACT_DERIV, ACT_GELU_ERF
    kind, M, N, K = CASES[a.case]
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    if kind in ("copy", "fill", "read"):
        x = torch.randn(GiB // 2, device=dev, generator=g).bfloat16()
        y = torch.empty_like(x)
        fn = {"copy": lambda: y.copy_(x), "fill": lambda: y.fill_(1.0), "read": lambda: x.sum()}[kind]
    elif kind.startswith("fwd"):
        x = torch.randn(M, K, device=dev, generator=g).bfloat16()
        w = (torch.randn(N, K, device=dev, generator=g) * 0.02).bfloat16()
        b = torch.zeros(N, device=dev)
        pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16) if "gelu" in kind else None
        res = torch.randn(M, N, device=dev, generator=g).bfloat16() if "res" in kind else None
        act = (ACT_GELU_ERF | ACT_DERIV) if pre is not None else 0
        fn = lambda: ops.linear(x, w, b, act=act, preact=pre, residual=res)
    elif kind.startswith("dx"):
        dy = torch.randn(M, K, device=dev, generator=g).bfloat16()
        w = (torch.randn(K, N, device=dev, generator=g) * 0.02).bfloat16()
        if kind == "dx_dsum":
            aux = torch.randn(M, N, device=dev, generator=g).bfloat16()
            db = torch.empty(N, device=dev)
            fn = lambda: ops.linear_dx(dy, w, act_bwd=ACT_GELU_ERF | ACT_DERIV, aux=aux, dsum=db)
        else:
            fn = lambda: ops.linear_dx(dy, w)
    else:
        dy = torch.randn(M, N, device=dev, generator=g).bfloat16()
        x = torch.randn(M, K, device=dev, generator=g).bfloat16()
        dw = torch.empty(N, K, device=dev)
        fn = lambda: ops.linear_dw(dy, x, dw)
    # a 512 MiB write between launches pushes the operands out of the Infinity Cache (256 MiB)
    flush = torch.empty(GiB // 2, dtype=torch.uint8, device=dev)
    for _ in range(1 + a.reps):
        flush.fill_(1)
        torch.cuda.synchronize()
        fn()
        torch.cuda.synchronize()
    print(a.case, "done", flush=True)


if __name__ == "__main__":
    main()
