"""LayerNorm forward / backward throughput on the config-3 shapes (HIP events; the library is
picked by CAPK_LIB_PATH, so two builds can be alternated on one box)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-captioning-ml-project_amd"))
import torch  # noqa: E402

from capk import ops  # noqa: E402

# (name, rows, residual gradient, fused column sum): the ViT pre-norms (50 432 rows, the
# residual stream's gradient added, the fused bias column sum on the second norm of a layer)
# and the decoder's post-norms (5120 rows)
CASES = [("vit_ln_dres_dsum", 256 * 197, True, True), ("vit_ln_dres", 256 * 197, True, False),
         ("dec_ln", 256 * 20, False, False)]


def main(iters=20):
    C = 768
    for name, rows, with_res, with_sum in CASES:
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(rows, C, device="cuda", generator=g).bfloat16()
        dy = torch.randn(rows, C, device="cuda", generator=g).bfloat16()
        dres = torch.randn(rows, C, device="cuda", generator=g).bfloat16() if with_res else None
        w = torch.rand(C, device="cuda", generator=g) + 0.5
        b = torch.randn(C, device="cuda", generator=g)
        _, mean, rstd = ops.layernorm_fwd(x, w, b, 1e-6)
        dw, db = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
        dsum = torch.zeros(C, device="cuda") if with_sum else None
        out = torch.empty_like(x)
        y = torch.empty_like(x)
        fwd = lambda: ops.layernorm_fwd(x, w, b, 1e-6, out=y)
        bwd = lambda: ops.layernorm_bwd(dy, x, w, mean, rstd, dw, db, dres=dres, out=out, dsum=dsum)
        for fn, tag, nbytes in ((fwd, "fwd", 2 * rows * C * 2), (bwd, "bwd", (4 if with_res else 3) * rows * C * 2)):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / iters
            print(f"{name:18s} {tag}: {ms * 1e3:7.1f} us  {nbytes / ms / 1e9:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
