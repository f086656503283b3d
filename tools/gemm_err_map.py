"""Error map of one forced-configuration GEMM (debug aid): per 16-row block x 16-column block
relative error, as a character map ('.' < 1e-3, 'x' >= 1e-3)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-captioning-ml-project_amd"))
import torch  # noqa: E402

from capk import _lib, ops  # noqa: E402

L = _lib.load()
L.capk_gemm_force_config(int(os.environ.get("CFG", "6")))
g = torch.Generator(device="cuda").manual_seed(0)
M = N = 256
for K in [int(k) for k in os.environ.get("KS", "576").split(",")]:
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    C = torch.empty(M, N, device="cuda", dtype=torch.float32)
    ops.gemm(a, True, b, True, M, N, K, C, lda=K, ldb=K, ldc=N)
    ref = a.float() @ b.float().t()
    e = ((C - ref) ** 2).reshape(16, 16, 16, 16).sum((1, 3)).sqrt() / (ref ** 2).reshape(16, 16, 16, 16).sum((1, 3)).sqrt()
    print(f"K={K}: rel {float((C - ref).norm() / ref.norm()):.3e}")
    for r in range(16):
        print("  " + "".join("x" if float(e[r, c]) > 1e-3 else "." for c in range(16)))
    # is the wrong part a product over a shifted K window?  (A K-tile j against B K-tile j')
    nk = K // 64
    D = C - ref
    best = []
    for j in range(nk):
        for jj in range(nk):
            P = a[:, 64 * j:64 * j + 64].float() @ b[:, 64 * jj:64 * jj + 64].float().t()
            cc = float((D * P).sum() / (P.norm() ** 2 + 1e-30))
            if abs(cc) > 0.2:
                best.append((j, jj, round(cc, 2)))
    print("  tile pairs (A j, B j', weight):", best[:20])
