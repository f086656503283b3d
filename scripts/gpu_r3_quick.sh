#!/bin/bash
# quick check: selected GPU tests, then beam bench and config-3 bench
set -u
OUT=gpurun_out/r3q
mkdir -p $OUT
run() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-6} | cut -c1-${CUTW:-300}; [ $rc -eq 0 ] || exit $rc; }
TAILN=3 run tests 600 python -u -m pytest ${TESTS:-tests/test_gpu_model.py tests/test_gpu_config4.py tests/test_gpu_beam.py} -x -q -rf --timeout 120 --timeout-method thread
[ -n "${BEAM:-1}" ] && TAILN=3 run beam 300 python tools/beam_bench.py --reps 3
[ -n "${PROF:-}" ] && run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 ${PROF}
exit 0
