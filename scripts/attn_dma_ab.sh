#!/bin/bash
# ViT attention: head images staged through registers vs by LDS DMA (CAPK_ATTN_DMA bit 0 forward,
# bit 1 dQ kernel, bit 2 dK/dV kernel), alternated, K/V evicted from the Infinity Cache between calls
for r in 1 2; do
  for x in 0 7 1 6; do
    CAPK_ATTN_DMA=$x ATTN_FLUSH=1 ATTN_ONLY=${ATTN_ONLY:-vit} timeout -k 10 120 python tools/attn_bench.py | sed "s/^/dma$x: /" || exit 1
  done
done
