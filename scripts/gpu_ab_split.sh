#!/bin/bash
# Split-K cap sweep on the config-2 bench (CAPK_GEMM_MAXSPLIT overrides the default cap).
set -u
mkdir -p gpurun_out/ab2
for s in ${SPLITS:-32 128}; do
  CAPK_GEMM_MAXSPLIT=$s timeout -k 10 300 python bench.py --workload config2 --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/ab2/c2_$s.log 2>&1 || exit $?
  echo "split cap $s: $(grep '^{' gpurun_out/ab2/c2_$s.log | cut -c1-160)"
done
timeout -k 10 300 python bench.py --workload config2 --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/ab2/c2_def.log 2>&1 || exit $?
echo "default: $(grep '^{' gpurun_out/ab2/c2_def.log | cut -c1-160)"
