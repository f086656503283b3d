"""Fused-attention throughput on the config-3 shapes (HIP events)."""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-captioning-ml-project_amd"))
import torch  # noqa: E402

from capk import ops  # noqa: E402
from capk.ops import HeadView  # noqa: E402

CASES = [("vit", 256, 12, 197, 197, 64, False), ("dec_self", 256, 8, 20, 20, 96, True),
         ("dec_cross", 256, 8, 20, 196, 96, False),
         # decode steps (forward only): config-3 beam-5 self (1280 rows, 20 keys) and cross (5
         # beams of 256 images against 196 memory keys), GPT-2 beam-4 / sampling steps (30 keys)
         ("dstep_self", 1280, 8, 1, 20, 96, False), ("dstep_cross5", 256, 8, 5, 196, 96, False),
         ("dstep_gpt2_b4", 1024, 12, 1, 30, 64, False), ("dstep_gpt2_s", 256, 12, 1, 30, 64, False)]
ONLY = os.environ.get("ATTN_ONLY")
# ATTN_FLUSH=1: read a 1 GB scratch buffer before every timed call (events around each call),
# so K / V come from HBM as in the model, where the other layers' K / V evict them from the
# 256 MB Infinity Cache between two calls of one layer (a read, not a fill: evicting dirty
# lines would add write-backs to the timed call)
FLUSH = os.environ.get("ATTN_FLUSH") == "1"


def main(iters=10):
    for name, B, H, Nq, Nk, hd, causal in CASES:
        if ONLY and name not in ONLY.split(","):
            continue
        D = H * hd
        g = torch.Generator(device="cuda").manual_seed(0)
        q = torch.randn(B * Nq, D, device="cuda", generator=g).bfloat16()
        kv = torch.randn(B * Nk, 2 * D, device="cuda", generator=g).bfloat16()
        o = torch.empty(B * Nq, D, device="cuda", dtype=torch.bfloat16)
        do = torch.randn_like(o)
        dq, dkv = torch.empty_like(q), torch.empty_like(kv)
        Q, K, V, O = HeadView(q, 0, Nq * D, D), HeadView(kv, 0, Nk * 2 * D, 2 * D), HeadView(kv, D, Nk * 2 * D, 2 * D), HeadView(o, 0, Nq * D, D)
        sc = 1 / math.sqrt(hd)
        fwd = lambda: ops.attention_fwd(Q, K, V, O, B, H, Nq, Nk, hd, sc, causal=causal)
        lse, _ = fwd()
        bwd = lambda: ops.attention_bwd(Q, K, V, O, HeadView(do, 0, Nq * D, D), lse, HeadView(dq, 0, Nq * D, D),
                                        HeadView(dkv, 0, Nk * 2 * D, 2 * D), HeadView(dkv, D, Nk * 2 * D, 2 * D),
                                        B, H, Nq, Nk, hd, sc, causal=causal)
        for fn, tag, mult in ((fwd, "fwd", 4), (bwd, "bwd", 10))[:1 if name.startswith("dstep") else 2]:
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if FLUSH:
                scratch = torch.ones(128 << 20, dtype=torch.int64, device="cuda")
                ms = 0.0
                for _ in range(iters):
                    scratch.max()
                    e0.record()
                    fn()
                    e1.record()
                    torch.cuda.synchronize()
                    ms += e0.elapsed_time(e1) / iters
                del scratch
            else:
                e0.record()
                for _ in range(iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / iters
            fl = mult * B * H * Nq * Nk * hd / (2 if causal else 1)
            by = (2 * B * Nq * D + 2 * B * Nk * D) * 2 * (1 if tag == "fwd" else 2)  # Q, O, K, V (x2 bwd)
            print(f"{name:10s} {tag}: {ms * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TFLOP/s  ~{by / ms / 1e9:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
