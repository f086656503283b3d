#!/bin/bash
# Split-K granularity A/B on the config-2 (LSTM step GEMMs, M = 128) and config-3 benches.
set -u
mkdir -p gpurun_out/ab3
for v in 4 2 4 2; do
  CAPK_GEMM_SPLIT_MINKT=$v timeout -k 10 300 python bench.py --workload config2 --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/ab3/c2_$v.log 2>&1 || exit $?
  echo "c2 minkt $v: $(grep '^{' gpurun_out/ab3/c2_$v.log | cut -c80-120)"
done
for v in 4 2; do
  CAPK_GEMM_SPLIT_MINKT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab3/c3_$v.log 2>&1 || exit $?
  echo "c3 minkt $v: $(grep '^{' gpurun_out/ab3/c3_$v.log | cut -c80-120)"
done
