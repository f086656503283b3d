#!/bin/bash
# Round-4 LSTM pair-slab recurrences (config 2): the LSTM / GEMM GPU tests, then config 2
# with CAPK_LSTM_PAIR=1/0 alternating on one box, then a kernel-trace profile of config 2.
set -u
OUT=gpurun_out/r4lstm
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name" | tee -a $OUT/status
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/status
  grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-3} | cut -c1-400
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
run tests 600 python -u -m pytest -x -q -rf --timeout 200 --timeout-method thread tests/test_gpu_lstm.py tests/test_gpu_gemm.py ${EXTRA_TESTS:-}
for rep in 1 2; do
  for v in 1 0; do
    TAILN=1 run bench_pair${v}_$rep 400 env CAPK_LSTM_PAIR=$v python bench.py --workload config2 --steps 8 --warmup 3 --no-cpu-baseline
  done
done
[[ -n "${NOPROF:-}" ]] && exit 0
TAILN=2 run prof_c2 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- python3 bench.py --workload config2 --steps 5 --warmup 2 --no-cpu-baseline
exit 0
