#!/bin/bash
# Round-end evidence session on one GPU box: full -m gpu suite -> smoke -> bench ->
# rocprofv3 kernel-trace/stats of the bench -> FETCH_SIZE / WRITE_SIZE passes for the
# GEMM traffic.  Each GPU step has its own time limit; a crash-type exit ends the session.
set -u
OUT=gpurun_out
mkdir -p $OUT
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test failures (no crash)
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/status
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/status
  tail -5 $OUT/$name.log
  ok_rc $rc || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
[[ ${STEPS:-tests,smoke,bench,prof,pmc} == *tests* ]] && \
  run tests 540 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread
run smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
run bench 420 python bench.py --steps 10 --warmup 3
[[ ${STEPS:-prof} == *prof* ]] && { PROF_TAG=prof PROF_SECS=300 bash scripts/gpu_profile.sh || exit $?; }
[[ ${STEPS:-pmc} == *pmc* ]] && { PROF_TAG=pmc PMC_GROUPS=scripts/pmc_traffic.txt bash scripts/gpu_counters.sh \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam-batch 0 || exit $?; }
exit 0
