"""Which k does the kernel pair with which k? (debug aid)  B[n][k] = 1 iff k == n (one-hot),
A[m][k] = code(k): C[m][n] = code(k_used) decodes the A column read against B row n's one."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-captioning-ml-project_amd"))
import torch  # noqa: E402

from capk import _lib, ops  # noqa: E402

L = _lib.load()
L.capk_gemm_force_config(int(os.environ.get("CFG", "6")))
M = N = 256
for K in [int(k) for k in os.environ.get("KS", "576,640").split(",")]:
    kk = torch.arange(K, device="cuda").float()
    B = torch.zeros(N, K, device="cuda")
    B[torch.arange(N), torch.arange(N)] = 1.0
    B = B.bfloat16()
    res = {}
    for name, code in (("lo", kk % 128), ("hi", kk // 128)):
        A = code[None, :].expand(M, K).contiguous().bfloat16()
        C = torch.empty(M, N, device="cuda", dtype=torch.float32)
        ops.gemm(A, True, B, True, M, N, K, C, lda=K, ldb=K, ldc=N)
        res[name] = C
    kused = res["hi"] * 128 + res["lo"]
    want = torch.arange(N, device="cuda").float()[None, :].expand(M, N)
    bad = (kused != want)
    print(f"K={K}: wrong {int(bad.sum())} of {M * N}")
    if bad.any():
        rows = bad.any(1).nonzero().flatten().tolist()
        print("  bad rows m:", rows[:24], "... count", len(rows))
        cols = bad.any(0).nonzero().flatten().tolist()
        print("  bad cols count", len(cols), "per-col bad rows (first cols):", [int(bad[:, c].sum()) for c in cols[:8]])
        print("  bad columns n:", cols[:40], "..." if len(cols) > 40 else "")
        for n in cols[:6]:
            print(f"  n={n}: k used (rows 0..3) {kused[:4, n].tolist()}  distinct {sorted(set(kused[:, n].tolist()))[:8]}")
