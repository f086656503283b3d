"""Correctness sweep of a forced GEMM configuration over K and grid shapes (debug aid):
prints the relative error of every (layout, M, N, K) against torch fp32."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-captioning-ml-project_amd"))
import torch  # noqa: E402

from capk import _lib, ops  # noqa: E402

cfg = int(os.environ.get("CFG", "6"))
L = _lib.load()
L.capk_gemm_force_config(cfg)
g = torch.Generator(device="cuda").manual_seed(0)
bad = 0
for ak, bk in ((True, True), (True, False)):
    for (M, N) in ((768, 256), (256, 256), (256, 768), (1000, 520)):
        for K in (128, 256, 512, 640, 704, 768, 1024, 1152, 2048):
            a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
            b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
            A = a if ak else a.t().contiguous()
            B = b if bk else b.t().contiguous()
            C = torch.empty(M, N, device="cuda", dtype=torch.float32)
            ops.gemm(A, ak, B, bk, M, N, K, C, lda=A.stride(0), ldb=B.stride(0), ldc=C.stride(0))
            ref = a.float() @ b.float().t()
            err = float((C - ref).norm() / ref.norm())
            rows = ((C - ref).abs().amax(dim=1) > 1e-2 * float(ref.abs().max())).nonzero().flatten()
            tag = "BAD" if err > 3e-3 else "ok"
            bad += tag == "BAD"
            print(f"{tag} ak={ak:d} bk={bk:d} M={M} N={N} K={K} cfg={L.capk_gemm_last_config()} rel={err:.2e} "
                  f"bad_rows={rows.numel()} first={rows[:4].tolist()} last={rows[-2:].tolist()}", flush=True)
print("bad:", bad)
