#!/bin/bash
# Round-3 GEMM diagnosis: per-shape graph-timed GEMM throughput of the shipped kernel, of the
# main-loop-only diagnostic build (no epilogue: CAPK_DIAG_NOSTORE), torch/hipBLASLt on the
# same shapes (reference only), then the config-3 bench line.
set -u
OUT=gpurun_out/r3diag
mkdir -p $OUT
SH=vit_qkv_fwd,vit_o_fwd,vit_fc1_fwd_plain,vit_fc2_fwd,vit_qkv_dx,vit_fc1_dx,vit_fc2_dx_plain,vit_o_dw,vit_fc1_dw,vit_qkv_dw,lm_head_fwd,lm_head_dx,lm_head_dw,bf16_big
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; cat $OUT/$name.log | grep -v amdgpu.ids | tail -20; [ $rc -eq 0 ] || exit $rc; }
export GEMM_GRAPH=1 GEMM_ONLY=$SH
step gemm_ship 300 python tools/gemm_bench.py
CAPK_LIB_PATH=$PWD/image-captioning-ml-project_amd/capk/libcapk_nostore.so step gemm_nostore 300 python tools/gemm_bench.py
step blas 300 python tools/blas_probe.py
step bench3 480 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --beam-batch 0
