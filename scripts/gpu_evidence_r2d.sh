#!/bin/bash
# Config-2 closing evidence after the BatchNorm / additive-attention / split-K changes:
# ResNet + LSTM + legacy parity tests, the config-2 bench line with its CPU baseline, and a
# rocprofv3 kernel-trace/stats profile of the config-2 train step.
set -u
OUT=gpurun_out/r2d
mkdir -p $OUT
run() {
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/status
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/status
  tail -2 $OUT/$name.log | cut -c1-250
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
run tests 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread
run bench_config2 420 python bench.py --workload config2 --steps 8 --warmup 3
PROF_TAG=r2d/prof_c2 PROF_SECS=300 PROF_CMD="bench.py --workload config2 --steps 3 --warmup 2 --no-cpu-baseline" \
  bash scripts/gpu_profile.sh || exit $?
exit 0
