#!/bin/bash
# Round-4 A/B session: GEMM split-tail on/off per shape, config-3 bench with the MFMA
# cross-attention kernels on/off, then a kernel-trace profile of the default build.
set -u
OUT=gpurun_out/r4
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name" | tee -a $OUT/status
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/status
  grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-12} | cut -c1-400
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
[[ -n "${TESTS:-}" ]] && TAILN=3 run tsel 600 python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread ${TESTS}
export GEMM_SHAPES="${GEMM_SHAPES:-dx768_197:50432:768:768:dx,dx3072_197:50432:768:3072:dx,dx2304_197:50432:768:2304:dx,res768_197:50432:768:768:fwd_res,res3072_197:50432:768:3072:fwd_res,fc1g_197:50432:3072:768:fwd_gelu_deriv,lmfwd:5120:50304:768:fwd}"
[[ ${SKIP_BENCH:-0} == 0 ]] && TAILN=1 run bench_xdec 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --beam-batch 0
[[ ${SKIP_BENCH:-0} == 0 ]] && TAILN=1 run bench_b 400 env ${BENCH_B_ENV:-CAPK_XDEC=0} python bench.py --steps 10 --warmup 3 --no-cpu-baseline --beam-batch 0
[[ ${PROF:-1} == 1 ]] && TAILN=2 run prof3 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof3 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --beam-batch 0
exit 0
