"""Which K-tiles does a forced GEMM configuration get wrong?  For each K (single 256 x 256
item, both operands K-major), fit C against per-K-tile partial products: C ~ sum_j w_j P_j,
P_j = A[:, 64j:64j+64] B[:, 64j:64j+64]^T, and print the tiles whose weight is not 1
(0 = missing, 2 = counted twice; a tile replaced by another shows as a 0 and a 2)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-captioning-ml-project_amd"))
import torch  # noqa: E402

from capk import _lib, ops  # noqa: E402

cfg = int(os.environ.get("CFG", "6"))
ak = os.environ.get("AK", "1") == "1"
bk = os.environ.get("BK", "1") == "1"
L = _lib.load()
L.capk_gemm_force_config(cfg)
g = torch.Generator(device="cuda").manual_seed(0)
M = N = 256
for nk in range(2, 37):
    K = 64 * nk
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    A = a if ak else a.t().contiguous()
    B = b if bk else b.t().contiguous()
    C = torch.empty(M, N, device="cuda", dtype=torch.float32)
    ops.gemm(A, ak, B, bk, M, N, K, C, lda=A.stride(0), ldb=B.stride(0), ldc=C.stride(0))
    P = torch.stack([a[:, 64 * j:64 * j + 64].float() @ b[:, 64 * j:64 * j + 64].float().t() for j in range(nk)])
    w = torch.linalg.lstsq(P.reshape(nk, -1).t(), C.reshape(-1, 1)).solution.flatten()
    off = [(j, round(float(x), 2)) for j, x in enumerate(w.tolist()) if abs(x - 1) > 0.05]
    res = float((C - (P * w[:, None, None]).sum(0)).norm() / C.norm())
    print(f"nk={nk:2d} K={K:5d} off={off} fit_residual={res:.1e}", flush=True)
