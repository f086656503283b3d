#!/bin/bash
# Round-4 decode-step GEMM -> LayerNorm slab fusion: kernel / beam / decoder GPU tests, then
# config 3 (train + beam-5) and config 5 with CAPK_DECODE_SLABS=1/0 alternating on one box.
set -u
OUT=gpurun_out/r4dec
mkdir -p $OUT
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name" | tee -a $OUT/status
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/status
  grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-3} | cut -c1-300
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
run tests 600 python -u -m pytest -x -q -rf --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_beam.py tests/test_gpu_graphs.py tests/test_gpu_plugins.py tests/test_gpu_config4.py ${EXTRA_TESTS:-}
for rep in 1 2; do
  for v in 1 0; do
    TAILN=1 run c3_${v}_$rep 400 env CAPK_DECODE_SLABS=$v python bench.py --steps 6 --warmup 2 --no-cpu-baseline
    TAILN=1 run c5_${v}_$rep 400 env CAPK_DECODE_SLABS=$v python bench.py --workload config5 --steps 4 --warmup 2 --no-cpu-baseline
  done
done
exit 0
