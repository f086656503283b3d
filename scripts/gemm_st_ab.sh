#!/bin/bash
# persistent GEMM output stores: plain (CAPK_GEMM_ST=0) vs sc1 for the kept pre-activation / act' (2) vs all bf16 outputs (3)
for r in 1 2; do
  for x in 0 2 3; do
    CAPK_GEMM_ST=$x GEMM_GRAPH=1 GEMM_ONLY=${ST_SHAPES:-vit_qkv_fwd,vit_fc1_fwd_gelu_deriv,vit_fc2_fwd,vit_fc2_dx_gelu_deriv,vit_fc1_dx,lm_head_fwd} timeout -k 10 120 python tools/gemm_bench.py | sed "s/^/st$x: /" || exit 1
  done
done
