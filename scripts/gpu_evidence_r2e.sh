#!/bin/bash
# GEMM HBM traffic passes on the final tree (the GEMM sources changed after r2c: split-K
# cap for K >= 65536, no effect on config 3), then the config-3 bench line that reads them.
set -u
OUT=gpurun_out/r2e
mkdir -p $OUT
PROF_TAG=r2e/pmc_traffic PMC_GROUPS=scripts/pmc_traffic.txt bash scripts/gpu_counters.sh \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam-batch 0 || exit $?
echo traffic done
