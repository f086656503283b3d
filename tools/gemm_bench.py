"""Per-shape GEMM throughput of libcapk's bf16 GEMM on the config-3 shapes (HIP events)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-captioning-ml-project_amd"))
import torch  # noqa: E402

from capk import ops  # noqa: E402
from capk._lib import ACT_DERIV, ACT_GELU_ERF  # noqa: E402

T = 256 * 197
SHAPES = [  # name, M, N, K, kind
    ("vit_qkv_fwd", T, 2304, 768, "fwd"), ("vit_o_fwd", T, 768, 768, "fwd"),
    ("vit_fc1_fwd_gelu", T, 3072, 768, "fwd_gelu"), ("vit_fc2_fwd", T, 768, 3072, "fwd"),
    ("vit_qkv_dx", T, 768, 2304, "dx"), ("vit_fc2_dx_gelu", T, 3072, 768, "dx_gelu"),
    ("vit_fc1_dx", T, 768, 3072, "dx"), ("vit_o_dw", T, 768, 768, "dw"), ("vit_fc1_dw", T, 3072, 768, "dw"),
    ("vit_qkv_dw", T, 2304, 768, "dw"),
    ("lm_head_fwd", 5120, 50304, 768, "fwd"), ("lm_head_dx", 5120, 768, 50304, "dx"), ("lm_head_dw", 5120, 50304, 768, "dw"),
    ("dec_fc1_fwd", 5120, 3072, 768, "fwd_gelu"), ("dec_kv_fwd", T - 1, 1536, 768, "fwd"),
    # epilogue isolation: the FFN shapes without their activation
    ("vit_fc1_fwd_plain", T, 3072, 768, "fwd"), ("vit_fc2_dx_plain", T, 3072, 768, "dx"),
    ("vit_fc1_fwd_bias_res", T, 3072, 768, "fwd_res"),
    # the model's forms: GELU with CAPK_ACT_DERIV (kept act'(pre); backward multiplies by it)
    ("vit_fc1_fwd_gelu_deriv", T, 3072, 768, "fwd_gelu_deriv"), ("vit_fc2_dx_gelu_deriv", T, 3072, 768, "dx_gelu_deriv"),
    # config 5 (fp8 forward): CLIP-B/32 rows 256*50, GPT-2 rows 256*20, decode LM heads
    ("f8_clip_qkv", 12800, 2304, 768, "f8"), ("f8_clip_fc1", 12800, 3072, 768, "f8"),
    ("f8_clip_fc2", 12800, 768, 3072, "f8"), ("f8_gpt2_fc1", 5120, 3072, 768, "f8"),
    ("f8_lm_head", 5120, 50304, 768, "f8"), ("f8_lm_head_beam5", 1280, 50304, 768, "f8"),
    ("f8_big", 16384, 16384, 8192, "f8"), ("bf16_big", 16384, 16384, 8192, "fwd"),
    ("bf16_4k", 4096, 4096, 4096, "fwd"), ("bf16_8k", 8192, 8192, 8192, "fwd"),
    ("f8_quant_x", 12800, 3072, 768, "quant"),
    # decode steps (GPT-2 Conv1D weights N-major: "c1d"): rows = beams in flight
    ("dec256_cattn", 256, 2304, 768, "c1d"), ("dec256_cproj", 256, 768, 768, "c1d"),
    ("dec256_fc", 256, 3072, 768, "c1d_gelu"), ("dec256_proj2", 256, 768, 3072, "c1d"),
    ("dec1280_cattn", 1280, 2304, 768, "c1d"), ("dec1280_cproj", 1280, 768, 768, "c1d"),
    ("dec1280_fc", 1280, 3072, 768, "c1d_gelu"), ("dec1280_proj2", 1280, 768, 3072, "c1d"),
    ("tdec1280_qkv", 1280, 2304, 768, "fwd"), ("tdec1280_fc1", 1280, 3072, 768, "fwd_gelu"),
    ("tdec1280_fc2", 1280, 768, 3072, "fwd"),
    # config-3 decoder train shapes (rows B*T = 5120, 8 heads x 96): the N = 768 products
    ("dec_o_fwd", 5120, 768, 768, "fwd"), ("dec_fc2_fwd", 5120, 768, 3072, "fwd"),
    ("dec_o_dx", 5120, 768, 768, "dx"), ("dec_qkv_dx", 5120, 768, 2304, "dx"),
    ("dec_fc1_dx", 5120, 768, 3072, "dx"), ("dec_qkv_fwd", 5120, 2304, 768, "fwd"),
    ("dec_fc1_fwd_deriv", 5120, 3072, 768, "fwd_gelu_deriv"), ("dec_fc2_dx_deriv", 5120, 3072, 768, "dx_gelu_deriv"),
    ("dec_o_dw", 5120, 768, 768, "dw"), ("dec_fc1_dw", 5120, 3072, 768, "dw"),
    # config-2 LSTM cell step (B = 128, hidden 768, 4 gates): gates = h W_hh^T, dh = dG W_hh
    ("lstm_gates_fwd", 128, 3072, 768, "fwd"), ("lstm_dh_dx", 128, 768, 3072, "dx"),
]


def run(name, M, N, K, kind, iters=20):
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    if kind == "f8":
        qa, sa = ops.quant_fp8(torch.randn(M, K, device=dev, generator=g).bfloat16())
        qb, sb = ops.quant_fp8(torch.randn(N, K, device=dev, generator=g) * 0.02)
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fn = lambda: ops.gemm_f8(qa, sa, qb, sb, C)
    elif kind == "quant":  # activation quantisation alone: [M, N] bf16 -> fp8
        x = torch.randn(M, N, device=dev, generator=g).bfloat16()
        q = torch.empty(M, N, device=dev, dtype=torch.uint8)
        sc = torch.empty(M, device=dev, dtype=torch.uint8)
        fn = lambda: ops.quant_fp8(x, q=q, scale=sc)
    elif kind.startswith("c1d"):  # GPT-2 Conv1D: y = x @ W, W [K, N] (N-major B)
        from capk._lib import ACT_GELU_TANH
        x = torch.randn(M, K, device=dev, generator=g).bfloat16()
        w = (torch.randn(K, N, device=dev, generator=g) * 0.02).bfloat16()
        b = torch.zeros(N, device=dev)
        act = ACT_GELU_TANH if "gelu" in kind else 0
        fn = lambda: ops.conv1d(x, w, b, act=act)
    elif kind.startswith("fwd"):
        x = torch.randn(M, K, device=dev, generator=g).bfloat16()
        w = (torch.randn(N, K, device=dev, generator=g) * 0.02).bfloat16()
        b = torch.zeros(N, device=dev)
        pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16) if "gelu" in kind else None
        res = torch.randn(M, N, device=dev, generator=g).bfloat16() if "res" in kind else None
        act = (ACT_GELU_ERF | (ACT_DERIV if "deriv" in kind else 0)) if pre is not None else 0
        fn = lambda: ops.linear(x, w, b, act=act, preact=pre, residual=res)
    elif kind.startswith("dx"):  # dX[M,K'] = dY[M,N'] W[N',K'] with K'=N, N'=K of the table entry
        dy = torch.randn(M, K, device=dev, generator=g).bfloat16()
        w = (torch.randn(K, N, device=dev, generator=g) * 0.02).bfloat16()
        aux = torch.randn(M, N, device=dev, generator=g).bfloat16() if "gelu" in kind else None
        act = (ACT_GELU_ERF | (ACT_DERIV if "deriv" in kind else 0)) if aux is not None else 0
        fn = lambda: ops.linear_dx(dy, w, act_bwd=act, aux=aux)
    else:  # dW[N,K] = dY[M,N]^T X[M,K]
        dy = torch.randn(M, N, device=dev, generator=g).bfloat16()
        x = torch.randn(M, K, device=dev, generator=g).bfloat16()
        dw = torch.empty(N, K, device=dev)
        fn = lambda: ops.linear_dw(dy, x, dw)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if os.environ.get("GEMM_GRAPH") == "1":  # GPU time only: the iterations replayed as one HIP graph
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(iters):
                fn()
        gr.replay()
        torch.cuda.synchronize()
        e0.record()
        gr.replay()
        e1.record()
    else:
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    tf = 2.0 * M * N * K / (ms * 1e-3) / 1e12
    if kind == "quant":
        print(f"{name:18s} M={M:6d} N={N:6d}  {ms * 1e3:8.1f} us  {3.0 * M * N / (ms * 1e-3) / 1e9:7.1f} GB/s",
              flush=True)
        return 0.0
    print(f"{name:18s} M={M:6d} N={N:6d} K={K:6d}  {ms * 1e3:8.1f} us  {tf:7.1f} TFLOP/s", flush=True)
    return tf


if __name__ == "__main__":
    only = os.environ.get("GEMM_ONLY")
    extra = os.environ.get("GEMM_SHAPES")  # "name:M:N:K:kind,..." ad-hoc shapes (run instead of the table)
    if extra:
        SHAPES = [(f[0], int(f[1]), int(f[2]), int(f[3]), f[4]) for f in (x.split(":") for x in extra.split(","))]
    for s in SHAPES:
        if only and s[0] not in only.split(","):
            continue
        run(*s, iters=int(os.environ.get("GEMM_ITERS", "20")))
