#!/bin/bash
set -u
OUT=gpurun_out/r4s20
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 280 --timeout-method thread tests/test_gpu_beam.py::test_transformer_beam5_config3_bf16_vs_fp32 > $OUT/beam.log 2>&1
rc=$?; grep -a "bf16 beam-5\|passed\|failed\|Error" $OUT/beam.log | head -5; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gemm.py > $OUT/gemm.log 2>&1
rc=$?; tail -2 $OUT/gemm.log; [ $rc -le 1 ] || exit $rc
GEMM_GRAPH=1 GEMM_SHAPES="big4k:4096:4096:4096:fwd,big8k:8192:8192:8192:fwd,dec_fc2_fwd:5120:768:3072:fwd,dec_qkv_fwd:5120:2304:768:fwd" timeout -k 10 200 python tools/gemm_bench.py > $OUT/gx.log 2>&1
rc=$?; grep TFLOP $OUT/gx.log; exit $rc
