#!/bin/bash
# Round-2 evidence, part 1 (one GPU box): full -m gpu suite, smoke, the three bench legs
# (config 3 headline with CPU baselines, config 2, config 5).  Each GPU step has its own
# time limit; a crash-type exit ends the session.
set -u
OUT=gpurun_out/r2
mkdir -p $OUT
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/status
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/status
  tail -3 $OUT/$name.log | cut -c1-300
  ok_rc $rc || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
run tests 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread
run smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
run bench_config3 480 python bench.py --steps 10 --warmup 3
run bench_config2 420 python bench.py --workload config2 --steps 8 --warmup 3
run bench_config5 480 python bench.py --workload config5 --steps 5 --warmup 2
exit 0
