#!/bin/bash
# ViT attention backward: split dK/dV + dQ pair (CAPK_ATTN_FUSED_BWD=0) vs the fused single-pass kernel (1)
for r in 1 2; do
  for x in 0 1; do
    CAPK_ATTN_FUSED_BWD=$x ATTN_FLUSH=1 ATTN_ONLY=${ATTN_ONLY:-vit} timeout -k 10 120 python tools/attn_bench.py | sed "s/^/fused$x: /" || exit 1
  done
done
