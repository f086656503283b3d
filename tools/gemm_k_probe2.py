"""Per-K-tile one-hot probe (debug aid): B row n has its single 1 at k = 64*t0 + n % 64; A
codes k by (k % 64, k // 64).  Prints, per t0, how many outputs deviate and the decoded
(lo, hi) sums of the first bad ones."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-captioning-ml-project_amd"))
import torch  # noqa: E402

from capk import _lib, ops  # noqa: E402

L = _lib.load()
L.capk_gemm_force_config(int(os.environ.get("CFG", "6")))
M = N = 256
K = int(os.environ.get("K", "576"))
nk = K // 64
kk = torch.arange(K, device="cuda").float()
for t0 in range(nk):
    B = torch.zeros(N, K, device="cuda")
    n = torch.arange(N, device="cuda")
    B[n, 64 * t0 + n % 64] = 1.0
    B = B.bfloat16()
    out = {}
    for name, code in (("lo", kk % 64), ("hi", kk // 64)):
        A = code[None, :].expand(M, K).contiguous().bfloat16()
        C = torch.empty(M, N, device="cuda", dtype=torch.float32)
        ops.gemm(A, True, B, True, M, N, K, C, lda=K, ldb=K, ldc=N)
        out[name] = C
    want_lo = (n % 64).float()[None, :].expand(M, N)
    bad = (out["lo"] != want_lo) | (out["hi"] != t0)
    msg = ""
    if bad.any():
        idx = bad.nonzero()[:3].tolist()
        msg = " e.g. " + ", ".join(f"(m={m},n={c}: lo={float(out['lo'][m, c])}, hi={float(out['hi'][m, c])})" for m, c in idx)
        cols = bad.any(0).nonzero().flatten()
        msg += f" cols {int(cols.min())}..{int(cols.max())} ({cols.numel()})"
    print(f"t0={t0}: bad {int(bad.sum())}{msg}", flush=True)
