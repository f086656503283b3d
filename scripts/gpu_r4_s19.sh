#!/bin/bash
# Round-4 session: the full -m gpu suite (beam config-3 test first, printed), smoke, config-3
# bench line with CPU baseline and beam-5.
set -u
OUT=gpurun_out/r4s19
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 280 --timeout-method thread tests/test_gpu_beam.py::test_transformer_beam5_config3_bf16_vs_fp32 > $OUT/beam.log 2>&1
rc=$?; grep -a "bf16 beam-5\|passed\|failed\|Error" $OUT/beam.log | head -5; [ $rc -le 1 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 280 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -8 $OUT/tests.log; [ $rc -le 1 ] || exit $rc
