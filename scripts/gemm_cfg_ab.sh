#!/bin/bash
# decode-step products under forced ring configurations (CAPK_GEMM_CFG, default list 1 7 8), alternated
SH=${CFG_SHAPES:-tq:1280:768:768:fwd,tqkv:1280:2304:768:fwd,tfc1:1280:3072:768:fwd_gelu,tfc2:1280:768:3072:fwd,g2attn:1280:2304:768:c1d,g2proj:1280:768:768:c1d,lstm:128:3072:768:fwd,dec5120o:5120:768:768:fwd_res}
for r in 1 2; do
  for c in ${CFGS:-1 7 8}; do
    CAPK_GEMM_CFG=$c GEMM_GRAPH=1 GEMM_SHAPES=$SH timeout -k 10 120 python tools/gemm_bench.py | sed "s/^/cfg$c: /" || exit 1
  done
done
