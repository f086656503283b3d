#!/bin/bash
# decode-step products on the 2-deep (CAPK_GEMM_DEEP=0) vs 4-deep (1) 128x128 ring, alternated
SH=${DEEP_SHAPES:-tq:1280:768:768:fwd,tqkv:1280:2304:768:fwd,tfc1:1280:3072:768:fwd_gelu,tfc2:1280:768:3072:fwd,g2attn:1280:2304:768:c1d,g2fc:1280:3072:768:c1d_gelu,g2proj:1280:768:768:c1d,s256fc:256:3072:768:c1d_gelu,lstm:128:3072:768:fwd}
for r in 1 2; do
  for d in 0 1; do
    CAPK_GEMM_DEEP=$d GEMM_GRAPH=1 GEMM_SHAPES=$SH timeout -k 10 120 python tools/gemm_bench.py | sed "s/^/deep$d: /" || exit 1
  done
done
