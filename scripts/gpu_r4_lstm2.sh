#!/bin/bash
# Round-4 LSTM pair-slab recurrences, second pass: LSTM tests, then config 2 with the pair
# route at CAPK_PAIR_MINKT=3 / 4 and the per-GEMM route, alternating on one box.
set -u
OUT=gpurun_out/r4lstm2
mkdir -p $OUT
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name" | tee -a $OUT/status
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/status
  grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-3} | cut -c1-200
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
run tests 600 python -u -m pytest -x -q -rf --timeout 200 --timeout-method thread tests/test_gpu_lstm.py ${EXTRA_TESTS:-}
for rep in 1 2; do
  for v in ${VARIANTS:-"k3:CAPK_PAIR_MINKT=3" "k4:CAPK_PAIR_MINKT=4" "off:CAPK_LSTM_PAIR=0"}; do
    n=${v%%:*}; e=${v#*:}
    TAILN=1 run bench_${n}_$rep 400 env $e python bench.py --workload config2 --steps 8 --warmup 3 --no-cpu-baseline
  done
done
exit 0
