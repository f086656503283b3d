#!/bin/bash
# Round-4 session: GEMM tests (split-K tail round), per-shape tail on/off, bench A/B, beam test.
set -u
OUT=gpurun_out/r4s21
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gemm.py > $OUT/gemm.log 2>&1
rc=$?; tail -3 $OUT/gemm.log; [ $rc -eq 0 ] || exit $rc
export GEMM_GRAPH=1 GEMM_ITERS=30
export GEMM_SHAPES="fc2_res:50432:768:3072:fwd_res,dx3072:50432:768:3072:dx,dx2304:50432:768:2304:dx,dx768:50432:768:768:dx,big4k:4096:4096:4096:fwd"
for v in 1 0 1 0; do
  CAPK_GEMM_TAIL=$v timeout -k 10 200 python tools/gemm_bench.py > $OUT/gx_tail$v.log 2>&1
  rc=$?; echo "== tail=$v"; grep TFLOP $OUT/gx_tail$v.log | cut -c1-80; [ $rc -eq 0 ] || exit $rc
done
unset GEMM_GRAPH GEMM_ITERS GEMM_SHAPES
VARIANTS="tail:CAPK_GEMM_TAIL=1 notail:CAPK_GEMM_TAIL=0" REPS=2 bash scripts/gpu_r4_envab.sh || exit $?
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 280 --timeout-method thread tests/test_gpu_beam.py::test_transformer_beam5_config3_bf16_vs_fp32 > $OUT/beam.log 2>&1
rc=$?; grep -a "bf16 beam-5\|passed\|failed\|Error" $OUT/beam.log | head -5; [ $rc -le 1 ] || exit $rc
