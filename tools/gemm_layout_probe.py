"""Decode where each output element of the forced 256x256 kernel lands: A = I, B[n][k] encodes
(n, k), so C[m][n] = B[n][m] names the (n, m) it came from.  Prints the first mismatches and
a histogram of (row mod 16, col mod 32) offsets.  Debug aid for the register-direct epilogue."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-captioning-ml-project_amd"))
import torch  # noqa: E402

from capk import _lib, ops  # noqa: E402

cfg = int(os.environ.get("CFG", "6"))
L = _lib.load()
L.capk_gemm_force_config(cfg)
M = N = K = 256
A = torch.eye(M, K, device="cuda").bfloat16()
nn, kk = torch.meshgrid(torch.arange(N), torch.arange(K), indexing="ij")
code = (nn % 64) * 64 + (kk % 64)  # exact in bf16? (< 4096: 12 bits -> not exact in bf16's 8)
B = torch.zeros(N, K)
# exact small codes: two passes, one for n % 16 and one for k % 32 (each < 256: exact in bf16)
for name, val in (("n16", (nn % 16).float()), ("k32", (kk % 32).float()), ("nblk", (nn // 16).float()),
                  ("kblk", (kk // 32).float())):
    Bv = val.cuda().bfloat16()
    C = torch.empty(M, N, device="cuda", dtype=torch.float32)
    ops.gemm(A, True, Bv, True, M, N, K, C, lda=K, ldb=K, ldc=N)
    ref = Bv.float().t()  # C[m][n] = B[n][m]
    bad = (C != ref.cuda())
    print(f"{name}: cfg={L.capk_gemm_last_config()} mismatches {int(bad.sum())} / {M * N}")
    if bad.any():
        idx = bad.nonzero()[:8].tolist()
        for m, n in idx:
            print(f"   C[{m}][{n}] = {float(C[m, n])}  expected {float(ref[m, n])}")
