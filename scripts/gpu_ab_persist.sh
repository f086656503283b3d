#!/bin/bash
# NOTE: the persistent gemm8p variant this A/B measured is not in the build;
# CAPK_GEMM_PERSIST is read only by that variant.
# A/B of the persistent 256x256 GEMM (CAPK_GEMM_PERSIST=0: one work item per WG) after the
# GEMM parity tests.  Any failure (including a test failure) ends the run.
set -u
OUT=gpurun_out/ab
mkdir -p $OUT
step() { local name=$1 secs=$2; shift 2; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "== $name rc=$rc"; tail -2 $OUT/$name.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step tests 200 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_fp8.py -x -q --timeout 60 --timeout-method thread
SH="vit_qkv_fwd,vit_o_fwd,vit_fc1_fwd_plain,vit_fc2_fwd,vit_qkv_dx,vit_fc2_dx_plain,vit_fc1_dx,vit_o_dw,vit_fc1_dw,vit_qkv_dw,lm_head_fwd,f8_clip_fc1"
CAPK_GEMM_PERSIST=0 GEMM_ONLY=$SH step gemm_p0 200 python tools/gemm_bench.py
GEMM_ONLY=$SH step gemm_p1 200 python tools/gemm_bench.py
CAPK_GEMM_PERSIST=0 step bench_p0 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --beam-batch 0
step bench_p1 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --beam-batch 0
paste $OUT/gemm_p0.log $OUT/gemm_p1.log | grep -v amdgpu.ids | awk -F'\t' '{print substr($1,1,75) " | " substr($2,40,40)}'
grep -h '^{' $OUT/bench_p0.log $OUT/bench_p1.log | cut -c100-160
exit 0
