"""ViT attention backward (bf16, hd 64) timed over query / key counts: the fused single-pass
kernel's time as a function of its 32-query chunk count separates a per-workgroup fixed cost
(prologue, stores) from the per-chunk cost.  HIP events, 20 calls per point, one process.

usage: python tools/attn_sweep.py [--mode 0|1] [--b 256] [--h 12]
"""
import argparse
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-captioning-ml-project_amd"))
import torch  # noqa: E402

from capk import ops  # noqa: E402
from capk.ops import HeadView  # noqa: E402


def time_bwd(B, H, Nq, Nk, hd=64, iters=20):
    D = H * hd
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn(B * Nq, D, device="cuda", generator=g).bfloat16()
    kv = torch.randn(B * Nk, 2 * D, device="cuda", generator=g).bfloat16()
    o = torch.empty(B * Nq, D, device="cuda", dtype=torch.bfloat16)
    do = torch.randn_like(o)
    dq, dkv = torch.empty_like(q), torch.empty_like(kv)
    Q, K, V, O = (HeadView(q, 0, Nq * D, D), HeadView(kv, 0, Nk * 2 * D, 2 * D), HeadView(kv, D, Nk * 2 * D, 2 * D),
                  HeadView(o, 0, Nq * D, D))
    sc = 1 / math.sqrt(hd)
    lse, _ = ops.attention_fwd(Q, K, V, O, B, H, Nq, Nk, hd, sc)

    def bwd():
        ops.attention_bwd(Q, K, V, O, HeadView(do, 0, Nq * D, D), lse, HeadView(dq, 0, Nq * D, D),
                          HeadView(dkv, 0, Nk * 2 * D, 2 * D), HeadView(dkv, D, Nk * 2 * D, 2 * D), B, H, Nq, Nk, hd, sc)
    bwd()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        bwd()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", type=int, default=-1)
    ap.add_argument("--b", type=int, default=256)
    ap.add_argument("--h", type=int, default=12)
    a = ap.parse_args()
    L = ops.lib()
    ops.check(L.capk_attention_set_fused_bwd(a.mode), "set_fused_bwd")
    print(f"# attention backward, B={a.b} H={a.h} hd=64, mode {a.mode}: us per call (us per (image, head) round)")
    rounds = a.b * a.h / 256
    for nk in (197, 96):
        for nq in (64, 96, 128, 160, 197, 224, 256):
            us = time_bwd(a.b, a.h, nq, nk)
            print(f"Nq {nq:4d} Nk {nk:4d} chunks {(nq + 31) // 32}: {us:8.1f} us  {us / rounds:6.2f} us/round", flush=True)


if __name__ == "__main__":
    main()
