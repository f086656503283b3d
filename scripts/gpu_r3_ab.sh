#!/bin/bash
# Same-box A/B: tests of the changed kernels, microbenches (v1 vs v2 decode), then bench.py with
# the session-start library (capk/libcapk_base.so) and the current one, back to back.
set -u
OUT=gpurun_out/r3ab
mkdir -p $OUT
run() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-12} | cut -c1-${CUTW:-400}; [ $rc -eq 0 ] || exit $rc; }
TAILN=4 run tests 600 python -u -m pytest ${TESTS:-tests/test_gpu_kernels.py tests/test_gpu_beam.py tests/test_gpu_graphs.py tests/test_gpu_config4.py} -x -q -rf --timeout 120 --timeout-method thread
run attn2 200 python tools/attn_bench.py
CAPK_DECODE_V1=1 ATTN_ONLY=dstep_self,dstep_cross5,dstep_gpt2_b4,dstep_gpt2_s run attn1 200 python tools/attn_bench.py
CUTW=600 TAILN=1 CAPK_KV_GATHER=1 CAPK_LIB_PATH=$PWD/image-captioning-ml-project_amd/capk/libcapk_base.so run bench_base 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCHARGS:-}
CUTW=600 TAILN=1 run bench_new 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCHARGS:-}
if [ -n "${C5AB:-}" ]; then
  CUTW=700 TAILN=1 CAPK_LIB_PATH=$PWD/image-captioning-ml-project_amd/capk/libcapk_base.so CAPK_KV_GATHER=1 run c5_base 400 python bench.py --workload config5 --steps 4 --warmup 2 --no-cpu-baseline --beam-batch 0
  CUTW=700 TAILN=1 run c5_new 400 python bench.py --workload config5 --steps 4 --warmup 2 --no-cpu-baseline --beam-batch 0
fi
exit 0
