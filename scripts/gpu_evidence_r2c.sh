#!/bin/bash
# Round-2 closing evidence (one GPU box): -m gpu suite, smoke, the three bench legs, rocprofv3
# kernel-trace/stats of the config-3 train and beam legs, the GEMM HBM traffic passes
# (FETCH_SIZE / WRITE_SIZE) and the SQ counter groups.  Every GPU step has its own time
# limit; any failure other than a pytest test failure ends the session.  No counter pass
# is combined with a trace domain.
set -u
OUT=gpurun_out/r2c
mkdir -p $OUT
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/status
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/status
  tail -3 $OUT/$name.log | cut -c1-300
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
run tests 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread
run smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
run bench_config3 480 python bench.py --steps 10 --warmup 3
run bench_config2 420 python bench.py --workload config2 --steps 8 --warmup 3
run bench_config5 480 python bench.py --workload config5 --steps 5 --warmup 2
PROF_TAG=r2c/prof_c3 PROF_SECS=300 PROF_CMD="bench.py --steps 5 --warmup 2 --no-cpu-baseline --beam-batch 0" \
  bash scripts/gpu_profile.sh || exit $?
PROF_TAG=r2c/prof_c3beam PROF_SECS=300 PROF_CMD="bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam-reps 3" \
  bash scripts/gpu_profile.sh || exit $?
PROF_TAG=r2c/pmc_traffic PMC_GROUPS=scripts/pmc_traffic.txt bash scripts/gpu_counters.sh \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam-batch 0 || exit $?
PROF_TAG=r2c/pmc_sq PMC_GROUPS=scripts/pmc_attn.txt bash scripts/gpu_counters.sh \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam-batch 0 || exit $?
exit 0
