#!/bin/bash
# Round-2 evidence, part 2: rocprofv3 kernel-trace/stats of each bench leg, the GEMM HBM
# traffic passes (FETCH_SIZE / WRITE_SIZE) and the SQ counter groups (MFMA busy, LDS
# waits) over the config-3 train step.  No counter pass is combined with a trace domain.
set -u
PROF_TAG=r2/prof_c3 PROF_SECS=300 PROF_CMD="bench.py --steps 3 --warmup 2 --no-cpu-baseline --beam-batch 0" \
  bash scripts/gpu_profile.sh || exit $?
PROF_TAG=r2/prof_c3beam PROF_SECS=300 PROF_CMD="bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam-reps 3" \
  bash scripts/gpu_profile.sh || exit $?
PROF_TAG=r2/prof_c2 PROF_SECS=300 PROF_CMD="bench.py --workload config2 --steps 3 --warmup 2 --no-cpu-baseline" \
  bash scripts/gpu_profile.sh || exit $?
PROF_TAG=r2/prof_c5 PROF_SECS=300 PROF_CMD="bench.py --workload config5 --steps 3 --warmup 2 --no-cpu-baseline --beam-batch 0" \
  bash scripts/gpu_profile.sh || exit $?
PROF_TAG=r2/pmc_traffic PMC_GROUPS=scripts/pmc_traffic.txt bash scripts/gpu_counters.sh \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam-batch 0 || exit $?
PROF_TAG=r2/pmc_sq PMC_GROUPS=scripts/pmc_attn.txt bash scripts/gpu_counters.sh \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam-batch 0 || exit $?
exit 0
