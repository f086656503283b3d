#!/bin/bash
# Decoder-side GEMM shapes (config 3, rows 5120) under every tile configuration, and the
# fused-attention bench, graph-timed.
set -u
OUT=gpurun_out/r3dec
mkdir -p $OUT
run() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-22}; [ $rc -eq 0 ] || exit $rc; }
export GEMM_GRAPH=1 GEMM_ONLY=${SHAPES:-dec_o_fwd,dec_fc2_fwd,dec_o_dx,dec_qkv_dx,dec_fc1_dx,dec_qkv_fwd,dec_fc1_fwd_deriv,dec_fc2_dx_deriv,dec_o_dw,dec_fc1_dw}
run dflt 200 python tools/gemm_bench.py
for c in ${CFGS:-1 2 3 4 5}; do CAPK_GEMM_CFG=$c run cfg$c 200 python tools/gemm_bench.py; done
CAPK_GEMM_MAXSPLIT=1 run nosplit 200 python tools/gemm_bench.py
run attn 200 python tools/attn_bench.py
