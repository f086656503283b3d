#!/bin/bash
# Config-2 ResNet-101 small-K GEMM shapes (layer1 / layer2 1x1 convs, 3x3 dcol, stem) per tile
# configuration (CAPK_GEMM_CFG; 0 = the library's choice), graph-replayed (tools/gemm_bench.py).
set -u
OUT=gpurun_out/r4conv
mkdir -p $OUT
M1=401408; M2=100352; MS=1605632
export GEMM_SHAPES="l1_c3_fwd:$M1:256:64:fwd,l1_c1_fwd:$M1:64:256:fwd,l1_c2_fwd:$M1:64:576:fwd,l1_c2_dcol:$M1:576:64:dx,l1_c1_dx:$M1:256:64:dx,l1_c3_dx:$M1:64:256:dx,l2_c3_fwd:$M2:512:128:fwd,l2_c2_dcol:$M2:1152:128:dx,l2_c1_dx:$M2:512:128:dx,l1_c2_dw:$M1:64:576:dw,stem_fwd:$MS:64:160:fwd"
export GEMM_GRAPH=1 GEMM_ITERS=10
for c in ${CFGS:-0 1 3 4}; do
  echo "== cfg $c" | tee -a $OUT/status
  CAPK_GEMM_CFG=$c timeout -k 10 300 python tools/gemm_bench.py > $OUT/cfg$c.log 2>&1
  rc=$?; cat $OUT/cfg$c.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
done
