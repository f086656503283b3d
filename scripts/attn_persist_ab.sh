#!/bin/bash
# ViT attention forward: per-(batch, head) kernel (CAPK_ATTN_PERSIST=0) vs persistent (1), alternated
for f in 1 0; do
  for x in 0 1 0 1; do
    CAPK_ATTN_PERSIST=$x ATTN_FLUSH=$f ATTN_ONLY=${ATTN_ONLY:-vit} timeout -k 10 120 python tools/attn_bench.py | sed "s/^/flush$f persist$x: /" || exit 1
  done
done
