#!/bin/bash
# Round 6: (1) first-round stagger of the fused ViT attention backward (CAPK_ATTN_STAGGER phases),
# (2) FC1 / DSUM time and FETCH per grouped-raster size (CAPK_GEMM_GROUP).  One GPU session.
set -u
OUT=gpurun_out/r6; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2; do for st in 0 2 4 6 8; do
  CAPK_ATTN_STAGGER=$st ATTN_ONLY=vit timeout -k 10 120 python tools/attn_bench.py 2>&1 | grep bwd | sed "s/^/stagger$st /" || exit 1
done; done | tee $OUT/stagger.txt
for g in 8 4 2 0; do
  CAPK_GEMM_GROUP=$g GEMM_ONLY=vit_fc1_fwd_gelu_deriv,vit_fc2_dx_gelu_deriv,vit_qkv_fwd timeout -k 10 120 python tools/gemm_bench.py 2>&1 | grep TFLOP | sed "s/^/group$g /" || exit 1
done | tee $OUT/group_time.txt
for g in 8 4 2; do
  CAPK_GEMM_GROUP=$g GEMM_ONLY=vit_fc1_fwd_gelu_deriv,vit_qkv_fwd timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/gfetch$g -o run -- python3 tools/gemm_bench.py > $OUT/gfetch$g.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $OUT/gfetch$g --match gemm8q > $OUT/gfetch$g.txt 2>&1; echo "group $g"; grep -A1 "gemm8q" $OUT/gfetch$g.txt | cut -c1-200
done
