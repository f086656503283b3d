"""Vendor-library reference rate (torch.matmul -> hipBLASLt) on the config-3 GEMM shapes, for
judging libcapk's GEMM headroom only -- nothing in capk calls a BLAS.  HIP events over a
replayed graph of `iters` products, as tools/gemm_bench.py with GEMM_GRAPH=1."""
import os
import torch

T = 256 * 197
SHAPES = [("vit_qkv_fwd", T, 2304, 768), ("vit_fc1_fwd", T, 3072, 768), ("vit_fc2_fwd", T, 768, 3072),
          ("vit_o_fwd", T, 768, 768), ("lm_head_fwd", 5120, 50304, 768), ("vit_fc1_dx", T, 768, 3072),
          ("vit_fc1_dw", 3072, 768, T), ("bf16_8k", 8192, 8192, 8192), ("tdec1280_fc1", 1280, 3072, 768),
          ("tdec1280_q", 1280, 768, 768),
          # config-3 decoder train products (rows B*T = 5120)
          ("dec_o_fwd", 5120, 768, 768), ("dec_fc2_fwd", 5120, 768, 3072), ("dec_qkv_fwd", 5120, 2304, 768),
          ("dec_fc1_fwd", 5120, 3072, 768), ("dec_o_dw", 768, 768, 5120), ("dec_fc1_dw", 3072, 768, 5120)]


def main(iters=20):
    only = os.environ.get("BLAS_ONLY")
    for name, M, N, K in SHAPES:
        if only and name not in only.split(","):
            continue
        g = torch.Generator(device="cuda").manual_seed(0)
        if name.endswith("_dw"):  # dW = dY^T X: both operands MN-major in memory
            a = torch.randn(K, M, device="cuda", generator=g).bfloat16().t()
            b = torch.randn(K, N, device="cuda", generator=g).bfloat16()
        else:
            a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
            b = torch.randn(N, K, device="cuda", generator=g).bfloat16().t()
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        for _ in range(3):
            torch.matmul(a, b, out=c)
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                for _ in range(iters):
                    torch.matmul(a, b, out=c)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        gr.replay()
        torch.cuda.synchronize()
        e0.record()
        gr.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / iters
        print(f"{name:18s} M={M:6d} N={N:6d} K={K:6d}  {us:9.1f} us  {2 * M * N * K / us / 1e6:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
