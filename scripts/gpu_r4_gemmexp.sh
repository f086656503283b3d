#!/bin/bash
# GEMM experiment variants (scripts/build_diag.sh exp_*) on the config-3 GEMM shapes.
set -u
OUT=gpurun_out/r4gx
mkdir -p $OUT
export GEMM_SHAPES="${GEMM_SHAPES:-qkv:50432:2304:768:fwd,o_res:50432:768:768:fwd_res,fc1g:50432:3072:768:fwd_gelu_deriv,fc2_res:50432:768:3072:fwd_res,dx768:50432:768:768:dx,dx3072:50432:768:3072:dx,dx2304:50432:768:2304:dx,fc2dxg:50432:3072:768:dx_gelu_deriv,lmfwd:5120:50304:768:fwd,big4k:4096:4096:4096:fwd}"
for v in base ${GX_VARIANTS:-exp_biasinit exp_hoist exp_biasinit+hoist}; do
  echo "== $v"
  if [ $v = base ]; then lib=""; else lib=image-captioning-ml-project_amd/capk/libcapk_diag_$v.so; fi
  CAPK_LIB_PATH=$lib timeout -k 10 200 python tools/gemm_bench.py > "$OUT/$v.log" 2>&1
  rc=$?
  grep -E "TFLOP" "$OUT/$v.log" | cut -c1-90
  [ $rc -eq 0 ] || { echo "stopping after $v (rc=$rc)"; exit $rc; }
done
exit 0
