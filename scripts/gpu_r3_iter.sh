#!/bin/bash
# Round-3 iteration check: kernel/model/GEMM parity tests, then attention + decoder GEMM
# shapes + the config-3 bench line.
set -u
OUT=gpurun_out/r3iter
mkdir -p $OUT
run() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-12}; [ $rc -eq 0 ] || exit $rc; }
TAILN=6 run tests 500 python -u -m pytest ${TESTS:-tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_gemm.py} -x -q -rf --timeout 120 --timeout-method thread
[ -n "${SKIPBENCH:-}" ] && exit 0
run attn 200 python tools/attn_bench.py
GEMM_GRAPH=1 GEMM_ONLY=dec_o_fwd,dec_qkv_fwd,dec_fc1_fwd_deriv,dec_fc2_dx_deriv,dec_o_dw,dec_fc1_dw run dec 200 python tools/gemm_bench.py
TAILN=2 run bench3 400 python bench.py --steps 10 --warmup 3 ${BENCHARGS:-}
