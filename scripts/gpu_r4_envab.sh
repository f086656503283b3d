#!/bin/bash
# Round-4 env A/B: optional test selection, then the config-3 train bench once per
# "name:ENV=val,ENV2=val" entry of $VARIANTS (default build otherwise), then optional
# kernel-trace stats per entry of $PROF_VARIANTS.
set -u
OUT=gpurun_out/r4ab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name" | tee -a $OUT/status
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/status
  grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-3} | cut -c1-300
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
envs() { echo "$1" | cut -s -d: -f2 | tr ',' ' '; }
[[ -n "${TESTS:-}" ]] && run tsel 600 python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread ${TESTS}
for rep in $(seq 1 ${REPS:-1}); do
  for v in ${VARIANTS:-base:}; do
    n=${v%%:*}
    TAILN=1 run bench_${n}_$rep 400 env $(envs "$v") python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --beam-batch 0
  done
done
for v in ${PROF_VARIANTS:-}; do
  n=${v%%:*}
  for kv in $(envs "$v"); do export "$kv"; done
  TAILN=2 run prof_$n 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$n -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --beam-batch 0
  for kv in $(envs "$v"); do unset "${kv%%=*}"; done
done
exit 0
