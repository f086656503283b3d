#!/bin/bash
# GEMM configuration A/B: kernel parity tests + per-shape throughput per CAPK_GEMM_CFG value.
set -u
mkdir -p gpurun_out
for c in ${CFGS:-0 1 2 3 4 5}; do
  CAPK_GEMM_CFG=$c timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -k "linear or gemm" > gpurun_out/t$c.log 2>&1
  rc=$?; echo "cfg $c tests rc=$rc"; tail -1 gpurun_out/t$c.log
  [ $rc -le 1 ] || exit $rc
  CAPK_GEMM_CFG=$c timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/g$c.log 2>&1
  rc=$?; echo "cfg $c bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
